#!/usr/bin/env bash
# Round-2 probe 43: 32768^2 grey, deeper fusion with the tall tiles.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe43
mkdir -p "$O"
PCONV_STREAM=0 timeout -k 10 500 python3 -u tools/band_sweep.py --width 32768 --height 32768 --channels grey --worlds 1 --fuse 8,10,12 --reps 120 --iters 2 --rounds 2 \
  --shapes "4,16,8;4,20,8;4,12,8" > "$O/sweep.jsonl" 2> "$O/sweep.err"
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    d = json.loads(l); print(d['fuse'], d['shape'], d['us_per_rep'])"
