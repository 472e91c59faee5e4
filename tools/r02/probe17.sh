#!/usr/bin/env bash
# Round-2 probe 17: full GPU suite, RCCL tests with loopback bootstrap, smoke,
# the driver's bench command.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe17
mkdir -p "$O"
rc=0
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || rc=$?
tail -n 3 "$O/pytest_gpu.log"
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
NCCL_SOCKET_IFNAME=lo timeout -k 10 200 python3 -u -m pytest tests/test_gpu_halo.py -k rccl -q --timeout 120 --timeout-method thread > "$O/pytest_rccl_lo.log" 2>&1
tail -n 1 "$O/pytest_rccl_lo.log"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -n 1 "$O/smoke.log"
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
cut -c1-300 "$O/bench.json"
