#!/bin/bash
# Round 6, call S: the chunk launches' shapes — tuned over the model's top 6
# (default) or every instantiated shape (a chunk's grid is small, so the
# latency-bound shapes the model ranks low may win), single-image latency.
set -o pipefail
OUT=gpurun_out/r06/s
mkdir -p $OUT
export PYTHONUNBUFFERED=1
probe() {  # name, extra args
  timeout -k 10 180 python -u tools/r06/latency_probe.py --images 60 --trace 6 $2 \
    > $OUT/lat_$1.json 2> $OUT/lat_$1.err || { echo "probe $1 failed"; tail -5 $OUT/lat_$1.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['tune_candidates'], d['latency_ms_median'], d['min'], [r[3] for r in d['chunk_trace_ms'][-1]], [t[2:3]+t[4:] for t in d['tuned']])" $OUT/lat_$1.json
}
for pass in a b c; do
  probe ${pass}_top6 "" || exit 1
  probe ${pass}_all "--tune-candidates 32" || exit 1
done
