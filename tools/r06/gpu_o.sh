#!/bin/bash
# Round 6, call O: streamed chunk weights on the driver's line — the default
# 1,2,2,1 against 2,3,3,4 and 5,5,5,6 (single images 0.537-0.541 vs
# 0.544-0.553 ms in calls M and N), interleaved, with the weights tests.
set -o pipefail
OUT=gpurun_out/r06/o
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py \
  -k "weights" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], d['config']['stream_weights'])" $OUT/$name.json
}
for r in 0 1 2 3 4 5; do
  one w1221_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  one w2334_$r --gpus 1 --steps 20 --warmup 5 --stream-weights 2,3,3,4 || exit 1
  one w5556_$r --gpus 1 --steps 20 --warmup 5 --stream-weights 5,5,5,6 || exit 1
done
