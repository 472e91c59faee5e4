#!/usr/bin/env bash
# Round-3 call AU: final tree (all CPU rows vectorised) — full GPU suite, smoke, bench at the
# driver's defaults (twice), then the BASELINE configs in steady state.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/au
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|Timeout" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 150 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  tail -1 $O/bench_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"
done
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { tail -5 $O/bench_driver_cmd.err; exit 1; }
tail -1 $O/bench_driver_cmd.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench (driver cmd)', d['ms_per_step'], d['value'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"
echo "call au done"
