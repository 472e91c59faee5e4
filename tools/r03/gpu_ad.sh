#!/usr/bin/env bash
# Round-3 call AD: after the pair-sum step — repetitions per launch for the
# 8-way band (per-rank proxy, bench --emulate 8:3) and the headline, and the
# headline at the driver's defaults.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ad
mkdir -p $O
run() {  # name secs args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], 'loop', d['loop_only']['ms_per_step'], 'fuse', d['config']['fuse'], 'floor', d['copy_floor']['floor_ms'])"
}
run head 150
for f in 8 10 13 20; do
  run e8_f$f 120 --emulate 8:3 --fuse $f
done
for f in 10 13; do
  run head_f$f 120 --fuse $f --steps 100 --warmup 10
done
run e8_default 120 --emulate 8:3
echo "call ad done"
