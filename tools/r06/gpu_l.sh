#!/bin/bash
# Round 6, call L: single-image latency against reps per launch (fuse) and
# chunk count — a streamed chunk's launches cost ~11-15 us each whatever its
# rows (call K), so fewer, deeper launches per chunk may shorten the chain.
set -o pipefail
OUT=gpurun_out/r06/l
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for f in 8 10 14 20; do
  for c in 4 6 8; do
    timeout -k 10 120 python -u tools/r06/latency_probe.py --images 30 --trace 6 --chunks $c --fuse $f \
      > $OUT/lat_f${f}_c${c}.json 2> $OUT/lat_f${f}_c${c}.err || { echo "probe f=$f c=$c failed"; tail -5 $OUT/lat_f${f}_c${c}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['latency_ms_median'], d['min'], [r[-1] for r in d['chunk_trace_ms'][-1]])" $OUT/lat_f${f}_c${c}.json
  done
done
