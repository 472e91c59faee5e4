#!/usr/bin/env bash
# Round-2 probe 44: deeper fusion on frames beyond the Infinity Cache,
# repeated (32768^2 grey, 16384^2 grey, 8192^2 RGB).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe44
mkdir -p "$O"
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --width 32768 --height 32768 --channels grey --worlds 1 --fuse 8,12,14,16 --reps 240 --iters 2 --rounds 3 \
  --shapes "4,16,8;4,20,8" > "$O/g32768.jsonl" 2> "$O/err.txt"
echo g32768 done
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --width 16384 --height 16384 --channels grey --worlds 1 --fuse 8,12,16 --reps 240 --iters 4 --rounds 3 \
  --shapes "4,16,8;4,20,8" > "$O/g16384.jsonl" 2>> "$O/err.txt"
echo g16384 done
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --width 8192 --height 8192 --channels rgb --worlds 1 --fuse 6,8,10,12 --reps 120 --iters 4 --rounds 3 \
  --shapes "4,12,8;4,20,8;4,16,8" > "$O/rgb8192.jsonl" 2>> "$O/err.txt"
python3 -c "
import json
for f in ('g32768', 'g16384', 'rgb8192'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, d['fuse'], d['shape'], d['us_per_rep'])"
