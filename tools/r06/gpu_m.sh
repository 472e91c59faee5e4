#!/bin/bash
# Round 6, call M: single-image latency against the streamed chunk sizes
# (--stream-weights).  Call K/L: a chunk's launches cost ~0.06-0.07 ms
# whatever its rows and the downloads trail the compute, so a model of the
# chunk chain (uploads ~46 GB/s, launches 0.055 ms + rows, downloads 46
# GB/s + 8 us each) ranks 5 near-even chunks ~0.04 ms under 1,2,2,1.
set -o pipefail
OUT=gpurun_out/r06/m
mkdir -p $OUT
export PYTHONUNBUFFERED=1
probe() {  # name, weights
  timeout -k 10 120 python -u tools/r06/latency_probe.py --images 40 --trace 6 --weights $2 \
    > $OUT/lat_$1.json 2> $OUT/lat_$1.err || { echo "probe $1 failed"; tail -5 $OUT/lat_$1.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['weights'], d['latency_ms_median'], d['min'], [r[-1] for r in d['chunk_trace_ms'][-1]])" $OUT/lat_$1.json
}
for pass in a b; do
  probe ${pass}_1221 1,2,2,1 || exit 1
  probe ${pass}_12221 1,2,2,2,1 || exit 1
  probe ${pass}_34455 3,4,4,5,5 || exit 1
  probe ${pass}_23334 2,3,3,3,4 || exit 1
  probe ${pass}_11111 1,1,1,1,1 || exit 1
  probe ${pass}_5556 5,5,5,6 || exit 1
  probe ${pass}_144454 1,4,4,4,5,4 || exit 1
  probe ${pass}_2334 2,3,3,4 || exit 1
  probe ${pass}_12333 1,2,3,3,3 || exit 1
done
