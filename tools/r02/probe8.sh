#!/usr/bin/env bash
# Round-2 probe 8: full GPU suite with the streaming kernel in the tuner and
# the auto fuse policy, then the BASELINE configs (CLI + bench).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe8
mkdir -p "$O"
rc=0
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || rc=$?
tail -n 4 "$O/pytest_gpu.log"
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
timeout -k 10 900 tools/baseline_configs.sh > "$O/baseline.log" 2>&1
cp -r gpurun_out/baseline "$O/" || true
echo probe8 done
