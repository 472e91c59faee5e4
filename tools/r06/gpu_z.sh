#!/bin/bash
# Round 6, call Z: lazy_head — a burst's first image held until the next
# submit (then a step graph) or drain (then row-streamed): its test, then the
# driver's command A/B (6 interleaved pairs; latency_ms must stay streamed).
set -o pipefail
OUT=gpurun_out/r06/z
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py \
  -k "lazy_head or head_stream_modes or weights_headline" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], d['config']['lazy_head'])" $OUT/$name.json
}
for r in 0 1 2 3 4 5; do
  one eager_$r --gpus 1 --steps 20 --warmup 5 --lazy-head off || exit 1
  one lazy_$r --gpus 1 --steps 20 --warmup 5 --lazy-head on || exit 1
done
python tools/r06/distributions.py "eager=$OUT/eager_*.json" "lazy=$OUT/lazy_*.json"
