#!/bin/bash
# Round 6, call K: where one head-streamed image's 0.54 ms goes, without a
# profiler — timing events after each chunk's upload, launches and download.
set -o pipefail
OUT=gpurun_out/r06/k
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for c in 4 3 6; do
  timeout -k 10 200 python -u tools/r06/latency_probe.py --images 20 --trace 10 --chunks $c > $OUT/lat_c$c.json 2> $OUT/lat_c$c.err || { echo "probe failed"; tail -5 $OUT/lat_c$c.err; exit 1; }
  cat $OUT/lat_c$c.json
done
