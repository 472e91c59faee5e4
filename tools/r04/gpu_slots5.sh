#!/bin/bash
# Round 4 (session 2, end): 4 vs 5 vs 6 images in flight on CU-masked slot
# queues, on the last tree (N=1 driver command and the 8-way proxy).
set -o pipefail
OUT=gpurun_out/r04/slots5
mkdir -p $OUT
export PYTHONUNBUFFERED=1
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-check "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:10s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']}")
PY
}
for i in a b; do
  for s in 4 5 6; do one n1_s${s}_$i --steps 20 --warmup 5 --slots $s || exit 1; done
done
for s in 4 5 6; do one e8_s$s --emulate 8:3 --steps 300 --warmup 10 --slots $s || exit 1; done
