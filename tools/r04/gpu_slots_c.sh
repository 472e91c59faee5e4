#!/bin/bash
# Round 4 (session 2): the 4-slot collapse without a profiler attached: stage
# timelines (bench --trace, timing events between the stages of each image)
# of the 8-way per-rank proxy with 3 / 4 slot streams from the runtime's
# pool ("plain") and on CU-masked dedicated queues ("cumask").
set -o pipefail
OUT=gpurun_out/r04/slots_c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for mode in plain cumask; do
  for s in 3 4; do
    n=${mode}_s$s
    PCONV_SLOT_STREAMS=$mode timeout -k 10 150 python -u bench.py --emulate 8:3 --steps 300 --warmup 30 --slots $s \
      --graph-capture off --trace 120 --trace-out $OUT/$n.trace.json --no-check > $OUT/$n.json 2> $OUT/$n.err \
      || { echo "bench $n failed"; tail -5 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms/step', d['ms_per_step'])" $OUT/$n.json $n
    python tools/pipeline_trace.py $OUT/$n.trace.json > $OUT/$n.trace.txt && sed -n 1,8p $OUT/$n.trace.txt
  done
done
