#!/usr/bin/env bash
# Round-2 probe 45: fusion depth x tall tiles for grey frames of every size
# (the auto_fuse policy), {4,24,8} added.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe45
mkdir -p "$O"
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --width 32768 --height 32768 --channels grey --worlds 1 --fuse 8,12,16 --reps 240 --iters 2 --rounds 3 \
  --shapes "4,20,8;4,24,8" > "$O/g32768.jsonl" 2> "$O/err.txt"
echo g32768 done
for sz in 8192 4096; do
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --width $sz --height $sz --channels grey --worlds 1 --fuse 8,12 --reps 240 --iters 6 --rounds 3 \
  --shapes "auto;4,16,8;4,20,8;4,24,8" > "$O/g$sz.jsonl" 2>> "$O/err.txt"
done
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --width 1920 --height 2520 --channels grey --worlds 1,8 --fuse 8,12 --reps 120 --iters 10 --rounds 3 \
  --shapes "auto" > "$O/g1920.jsonl" 2>> "$O/err.txt"
python3 -c "
import json
for f in ('g32768', 'g8192', 'g4096', 'g1920'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, 'w', d['world'], 'fuse', d['fuse'], d['shape'], d['us_per_rep'])"
