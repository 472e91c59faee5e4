#!/usr/bin/env bash
# Round-2 probe 66: bench.py robustness changes (guarded adoption re-time,
# watchdog armed through shutdown): multi-process rehearsals + halo suite.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe66
mkdir -p "$O"
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_halo.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
