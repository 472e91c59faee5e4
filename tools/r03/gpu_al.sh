#!/usr/bin/env bash
# Round-3 call AL: repetitions per launch of the float kernel (box / edge,
# 1920x2520 RGB and grey) after the clamp removal; loop_only of bench.py.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/al
mkdir -p $O
for ch in rgb grey; do
  for f in box edge; do
    for fu in 3 4 6 8; do
      timeout -k 10 90 python3 bench.py --channels $ch --filter $f --fuse $fu --steps 30 --warmup 5 > $O/${ch}_${f}_$fu.json 2> $O/err.txt || { tail -3 $O/err.txt; exit 1; }
      tail -1 $O/${ch}_${f}_$fu.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ch $f fuse $fu', d['loop_only']['us_per_rep'], 'us/rep', d['config']['fuse'])"
    done
  done
done
echo "call al done"
