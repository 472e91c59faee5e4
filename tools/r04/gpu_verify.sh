#!/bin/bash
# Round 4 (session 2): the whole GPU suite, smoke and the driver's bench
# command on the current tree.
set -o pipefail
OUT=gpurun_out/r04/verify
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
for i in a b; do
  timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench failed"; tail -5 $OUT/bench_$i.err; exit 1; }
  tail -1 $OUT/bench_$i.json
done
# the driver's command with head streaming (the first image of the burst row-streamed)
for c in 2 4; do
  for i in a b; do
    timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 --stream-chunks $c > $OUT/bench_h${c}_$i.json 2> $OUT/bench_h${c}_$i.err || { echo "bench h$c failed"; tail -5 $OUT/bench_h${c}_$i.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], d.get('mismatches'))" $OUT/bench_h${c}_$i.json
  done
done
# single-image latency of a row-streamed image: SDMA chunk copies vs CU copy kernels (capped grids)
for cc in sdma kernel64 kernel128 kernel256; do
  for c in 4 8; do
    n=lat_${cc}_c$c
    PCONV_STREAM_COPIES=$cc timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 --stream-chunks $c --loop-steps 3 > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail -5 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], d.get('mismatches'))" $OUT/$n.json
  done
done
