#!/usr/bin/env bash
# Round-2 probe 14: tuned picks (two-pass tuning, 6 candidates, taller
# shapes, streaming kernel) on the BASELINE frames at fuse 6 / 8.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe14
mkdir -p "$O"
for i in 1 2; do
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1 --fuse 6,8 --reps 24 --iters 2 --rounds 2 --width 32768 --height 32768 --channels grey --shapes auto >> "$O/grey32768_auto.jsonl" 2>> "$O/err.log"
done
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 40 --iters 10 --rounds 2 --shapes auto >> "$O/rgb1920_auto.jsonl" 2>> "$O/err.log"
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 6,8 --reps 24 --iters 3 --rounds 2 --width 8192 --height 8192 --shapes auto >> "$O/rgb8192_auto.jsonl" 2>> "$O/err.log"
cat "$O"/*.jsonl
