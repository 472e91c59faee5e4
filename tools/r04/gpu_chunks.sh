#!/bin/bash
# Round 4 (session 2): streamed single-image latency vs chunk count (head
# streaming on the slots' streams) and vs every image streamed (step graphs
# off, pool copy streams).
set -o pipefail
OUT=gpurun_out/r04/chunks
mkdir -p $OUT
export PYTHONUNBUFFERED=1
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-check "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:12s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']}")
PY
}
for c in 2 3 4 5 6 8; do one c$c --steps 20 --warmup 5 --stream-chunks $c || exit 1; done
one c4_again --steps 20 --warmup 5 --stream-chunks 4 || exit 1
one c3_again --steps 20 --warmup 5 --stream-chunks 3 || exit 1
one direct4 --steps 20 --warmup 5 --stream-chunks 4 --step-graphs off || exit 1
one direct3 --steps 20 --warmup 5 --stream-chunks 3 --step-graphs off || exit 1
