#!/usr/bin/env bash
# Round-2 probe 50: re-verification after the container was re-created and
# the tree rebuilt: full GPU suite, smoke, the driver's bench command.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe50
mkdir -p "$O"
rc=0
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || rc=$?
tail -n 3 "$O/pytest_gpu.log"
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -n 1 "$O/smoke.log"
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
cut -c1-300 "$O/bench.json"
timeout -k 10 120 tools/ubench/isa_rates > "$O/isa_rates.txt" 2>&1
grep -e u64 -e b64 -e add3 -e v_add_u32 "$O/isa_rates.txt"
exit $rc
