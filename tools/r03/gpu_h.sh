#!/usr/bin/env bash
# Round-3 call H: full GPU suite, smoke, bench x3, float tuning check, hybrid tables (passive waits).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/h
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|Timeout" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 150 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  tail -1 $O/bench_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"
done
timeout -k 10 200 python -u tools/r03/float_sweep.py quick > $O/float_sweep_quick.jsonl 2> $O/float_sweep.err || exit 1
grep '"auto"' $O/float_sweep_quick.jsonl
timeout -k 10 500 python tools/ref_tables.py mpi-cpu --backends omp --channels grey,rgb --sizes 1260,2520,5040 --ranks 1,2,4,9 --runs 5 --out $O/hybrid_bound.jsonl > /dev/null 2> $O/hybrid.err
python - <<'PY'
import json
for l in open("gpurun_out/r03/h/hybrid_bound.jsonl"):
    r = json.loads(l)
    print(r["channels"], r["height"], r["ranks"], r["omp_threads"], r.get("rank0_cpus"), round(r["loop_s"], 4),
          [round(x, 4) for x in r["loop_all_s"]])
PY
