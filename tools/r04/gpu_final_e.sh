#!/bin/bash
# Round 4 (session 2): the whole GPU suite, smoke and the driver's command on
# the final defaults (4 slots, head streaming on the slots' streams), 200
# images, the 8-way proxy, the one-shot CLI's ring staging A/B, and the
# reference's CUDA table with `conv --backend auto` (two-stage pricing).
set -o pipefail
OUT=gpurun_out/r04/final_e
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:12s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} mism {d.get('mismatches')} vs {d.get('vs_baseline')}")
PY
}
for i in a b c; do one bench_$i --gpus 1 --steps 20 --warmup 5 || exit 1; done
one s200 --steps 200 --warmup 5 || exit 1
one e8 --emulate 8:3 --steps 300 --warmup 10 || exit 1
C=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for j in "8192 8192 100 rgb" "32768 32768 200 grey"; do
  set -- $j
  for rg in 0 1; do
    n=cli_${1}_${4}_ring$rg
    PCONV_RING=$rg timeout -k 10 300 $C /tmp/x.raw $1 $2 $3 $4 --synthetic 7 --backend hip --json --quiet --out /tmp/o.raw > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['e2e_s'],4), d['phases_s'])" $OUT/$n.json
  done
done
AUTO_OUT=gpurun_out/r04/auto_e bash tools/r04/gpu_auto.sh || exit 1
