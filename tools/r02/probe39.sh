#!/usr/bin/env bash
# Round-2 probe 39: resident kernel abort path (wait timeout) + the rest of
# its tests.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe39
mkdir -p "$O"
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_resident.py -v -x --timeout 90 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 14 "$O/pytest.log"
