#!/bin/bash
# Round 4 (session 2): fewer, deeper fused launches for the streamed head
# image (4 chunks x levels launches issued one by one from the host):
# latency, throughput and the device loop against --fuse.
set -o pipefail
OUT=gpurun_out/r04/fuse_lat
mkdir -p $OUT
export PYTHONUNBUFFERED=1
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d['config']
print(f"{sys.argv[2]:10s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} loop {d['loop_only']['ms_per_step']} fuse {c.get('fuse')} halo {c.get('halo_depth')} mism {d.get('mismatches')}")
PY
}
for i in a b; do
  one def_$i --steps 20 --warmup 5 || exit 1
  for f in 8 10 14; do one f${f}_$i --steps 20 --warmup 5 --fuse $f || exit 1; done
done
