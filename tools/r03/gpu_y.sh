#!/usr/bin/env bash
# Round-3 call Y (container re-created again): rebuilt tree — full GPU
# suite, smoke, bench at the driver's defaults.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/y
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|Timeout" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 150 python bench.py > $O/bench_1.json 2> $O/bench_1.err || { tail -5 $O/bench_1.err; exit 1; }
tail -1 $O/bench_1.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"
