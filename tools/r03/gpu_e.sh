#!/usr/bin/env bash
# Round-3 call E: float temporal kernel tests, halo/multiproc suites, float-filter benches, hybrid tables.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "float" -x -q --timeout 120 --timeout-method thread > $O/pytest_float.log 2>&1
rc=$?; tail -3 $O/pytest_float.log; [ $rc -ge 124 ] && exit 1
for f in box edge gaussian; do
  timeout -k 10 150 python bench.py --filter $f --steps 100 --warmup 10 > $O/bench_$f.json 2> $O/bench_$f.err
  rc=$?; echo "bench $f rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/bench_$f.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', d['ms_per_step'], d['loop_only'], d['config']['fuse'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_multiproc.py -x -q --timeout 300 --timeout-method thread > $O/pytest_halo.log 2>&1
rc=$?; tail -8 $O/pytest_halo.log; [ $rc -ge 124 ] && exit 1
timeout -k 10 500 python tools/ref_tables.py mpi-cpu --backends omp --channels grey,rgb --sizes 1260,2520,5040 --ranks 1,2,4,9 --runs 5 --out $O/hybrid_bound.jsonl > /dev/null 2> $O/hybrid.err
python - <<'PY'
import json
for l in open("gpurun_out/r03/e/hybrid_bound.jsonl"):
    r = json.loads(l)
    print(r["channels"], r["height"], r["ranks"], r["omp_threads"], r.get("rank0_cpus"), round(r["loop_s"], 4),
          [round(x, 4) for x in r["loop_all_s"]])
PY
# per-rank proxies of the 8-way split, every halo mode (exchange modes: RCCL send/recv to self)
for m in preload slot_exchange slot_exchange_direct event overlap; do
  timeout -k 10 150 python bench.py --emulate 8:3 --emulate-halo $m --steps 200 --warmup 20 > $O/emulate8_$m.json 2> $O/emulate8_$m.err
  rc=$?; echo "emulate $m rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/emulate8_$m.err; exit 1; }
  python -c "import json; d=json.load(open('$O/emulate8_$m.json')); print('$m', d['ms_per_step'], d['config']['exchanges_per_step'], d['config']['halo_depth'], d['config']['step_graphs'], d['loop_only']['ms_per_step'])"
done
