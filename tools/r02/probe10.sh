#!/usr/bin/env bash
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe10
mkdir -p "$O"
timeout -k 10 60 tools/ubench/launch_cost > "$O/launch_cost.jsonl" 2>&1
cat "$O/launch_cost.jsonl"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py tests/test_service.py -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
