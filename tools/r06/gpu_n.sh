#!/bin/bash
# Round 6, call N: two compute lanes for the streamed head (head_lanes=2, a
# wavefront over chunks and levels) — correctness on the GPU, then
# single-image latency over lanes x chunk weights, then the driver's line A/B.
set -o pipefail
OUT=gpurun_out/r06/n
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py \
  -k "two_lanes or lanes_headline or head_stream_modes" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
probe() {  # name, lanes, weights
  timeout -k 10 120 python -u tools/r06/latency_probe.py --images 40 --trace 6 --lanes $2 --weights $3 \
    > $OUT/lat_$1.json 2> $OUT/lat_$1.err || { echo "probe $1 failed"; tail -5 $OUT/lat_$1.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['lanes'], d['weights'], d['latency_ms_median'], d['min'], [r[-1] for r in d['chunk_trace_ms'][-1]])" $OUT/lat_$1.json
}
for pass in a b; do
  for l in 1 2; do
    probe ${pass}_l${l}_1221 $l 1,2,2,1 || exit 1
    probe ${pass}_l${l}_12221 $l 1,2,2,2,1 || exit 1
    probe ${pass}_l${l}_122221 $l 1,2,2,2,2,1 || exit 1
    probe ${pass}_l${l}_1222221 $l 1,2,2,2,2,2,1 || exit 1
    probe ${pass}_l${l}_111111 $l 1,1,1,1,1,1 || exit 1
    probe ${pass}_l${l}_2334 $l 2,3,3,4 || exit 1
  done
done
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'])" $OUT/$name.json
}
for r in 0 1 2; do
  one drv_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  one lanes2_$r --gpus 1 --steps 20 --warmup 5 --head-lanes 2 --stream-weights 1,2,2,2,2,1 || exit 1
done
