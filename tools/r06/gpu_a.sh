#!/bin/bash
# Round 6, call A: is the driver's 20-image window bimodal, and why?
#  1. the driver's exact command as the first GPU process of a fresh box, then
#     9 more times: every line carries the replayed windows (plain + marked),
#     the tuner's picks and the process's hardware queues;
#  2. three runs with the HIP runtime's copy log (which SDMA engine each copy
#     was given, and the free-engine mask it saw), windows replayed too.
set -o pipefail
OUT=gpurun_out/r06/a
mkdir -p $OUT
export PYTHONUNBUFFERED=1
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d.get("windows") or {}
print(f"{sys.argv[2]:8s} ms/step {d['ms_per_step']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']} "
      f"q {d.get('hw_queues')} win {w.get('ms_per_step')} marked {w.get('marked_ms_per_step')}")
PY
}
for i in 0 1 2 3 4 5 6 7 8 9; do one drv_$i --gpus 1 --steps 20 --warmup 5 || exit 1; done
for i in 0 1 2; do
  AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x900 one log_$i --gpus 1 --steps 20 --warmup 5 || exit 1
  grep -cE "copy_engine|Query copy engine|SDMA" $OUT/log_$i.err || true
done
