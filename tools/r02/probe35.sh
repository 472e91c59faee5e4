#!/usr/bin/env bash
# Round-2 probe 35: first run of the register-resident kernel: bit-exactness
# tests, then loop time against the tile kernel.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe35
mkdir -p "$O"
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_resident.py -v -x --timeout 90 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 15 "$O/pytest.log"
timeout -k 10 240 python3 -u tools/resident_sweep.py > "$O/sweep.jsonl" 2> "$O/sweep.err"
cat "$O/sweep.jsonl"
