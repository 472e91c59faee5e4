#!/bin/bash
# Round 6, call R: two single-image levers — drain() polling the streams
# (spin_wait) instead of blocking, and each streamed chunk's download issued
# right after its own launches (interleave_downloads) — tests, latency
# probes (2 x 2), then the driver's line A/B.
set -o pipefail
OUT=gpurun_out/r06/r
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py \
  -k "spin_wait or weights_headline" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
probe() {  # name, extra args
  timeout -k 10 120 python -u tools/r06/latency_probe.py --images 60 $2 \
    > $OUT/lat_$1.json 2> $OUT/lat_$1.err || { echo "probe $1 failed"; tail -5 $OUT/lat_$1.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['spin'], d['interleave'], d['latency_ms_median'], d['min'], d['max'])" $OUT/lat_$1.json
}
for pass in a b c d; do
  probe ${pass}_block "" || exit 1
  probe ${pass}_spin "--spin" || exit 1
  probe ${pass}_inter "--interleave" || exit 1
  probe ${pass}_both "--spin --interleave" || exit 1
done
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], c['spin_wait'], c['interleave_downloads'])" $OUT/$name.json
}
for r in 0 1 2 3; do
  one base_$r --gpus 1 --steps 20 --warmup 5 --spin-wait off --interleave-downloads off || exit 1
  one both_$r --gpus 1 --steps 20 --warmup 5 --spin-wait on --interleave-downloads on || exit 1
done
