#!/bin/bash
# Round 4 (session 2): why the streamed head image got slower with 4 slots
# (latency 0.83 vs 0.55 ms at 3): its copy streams from the runtime's pool
# vs dedicated queues vs the next slots' streams; and the one-shot CLI's
# ring staging (small pinned chunks, read || H2D, D2H || parallel write)
# against one pinned copy of the whole image.
set -o pipefail
OUT=gpurun_out/r04/head
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py "tests/test_gpu_engine.py::test_cli_hip_ring_staging" -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
one() {  # name, head mode, -- bench args
  local name=$1 m=$2; shift 2
  PCONV_HEAD_STREAMS=$m timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:16s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} mism {d.get('mismatches')}")
PY
}
for i in a b; do
  for m in pool cumask slots; do
    one s4_${m}_$i $m --steps 20 --warmup 5 --stream-chunks 4 || exit 1
  done
  one s3_pool_$i pool --steps 20 --warmup 5 --stream-chunks 4 --slots 3 || exit 1
done
one s4_slots_200 slots --steps 200 --warmup 5 --stream-chunks 4 --no-check || exit 1
one s4_cumask_200 cumask --steps 200 --warmup 5 --stream-chunks 4 --no-check || exit 1
C=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for j in "1920 2520 40 rgb" "8192 8192 100 rgb" "32768 32768 200 grey"; do
  set -- $j
  for rg in 0 1; do
    n=cli_${1}_${4}_ring$rg
    PCONV_RING=$rg timeout -k 10 300 $C /tmp/x.raw $1 $2 $3 $4 --synthetic 7 --backend hip --json --quiet --out /tmp/o.raw > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['e2e_s'],4), d['phases_s'])" $OUT/$n.json
  done
done
