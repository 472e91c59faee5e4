#!/usr/bin/env bash
# Round-2 probe 40: final-tree evidence: full GPU suite, smoke, the driver's
# bench command, and a rocprofv3 kernel-trace --stats run of it.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe40
mkdir -p "$O"
rc=0
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || rc=$?
tail -n 3 "$O/pytest_gpu.log"
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -n 1 "$O/smoke.log"
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
cut -c1-160 "$O/bench.json"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$O/prof" -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/prof_bench.json" 2> "$O/prof.err"
find "$O/prof" -name "*stats.csv" | head -n 5
exit $rc
