#!/bin/bash
# Round 6, call P: (1) near-even 4-chunk weights for the single image (call
# O: 5,5,5,6 0.533-0.535 and 2,3,3,4 0.534-0.538 vs 1,2,2,1 0.548-0.552 ms,
# window ms/step unchanged); (2) value_sync — the streamed chunks' hand-offs
# as stream memory operations instead of events — its tests, then latency
# with the wait-passed timestamps of the chunk trace.
set -o pipefail
OUT=gpurun_out/r06/p
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py \
  -k "value_sync" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
probe() {  # name, weights, extra args
  timeout -k 10 120 python -u tools/r06/latency_probe.py --images 60 --trace 6 --weights $2 $3 \
    > $OUT/lat_$1.json 2> $OUT/lat_$1.err || { echo "probe $1 failed"; tail -5 $OUT/lat_$1.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['weights'], d['value_sync'], d['latency_ms_median'], d['min'], [r[-1] for r in d['chunk_trace_ms'][-1]])" $OUT/lat_$1.json
}
for pass in a b c; do
  probe ${pass}_1221 1,2,2,1 || exit 1
  probe ${pass}_1221_vs 1,2,2,1 --value-sync || exit 1
  probe ${pass}_1111 1,1,1,1 || exit 1
  probe ${pass}_5556 5,5,5,6 || exit 1
  probe ${pass}_5556_vs 5,5,5,6 --value-sync || exit 1
  probe ${pass}_4445 4,4,4,5 || exit 1
  probe ${pass}_3334 3,3,3,4 || exit 1
  probe ${pass}_4555 4,5,5,5 || exit 1
  probe ${pass}_45556 4,5,5,5,6 || exit 1
  probe ${pass}_45556_vs 4,5,5,5,6 --value-sync || exit 1
  probe ${pass}_122221_vs 1,2,2,2,2,1 --value-sync || exit 1
done
