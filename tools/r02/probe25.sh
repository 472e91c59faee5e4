#!/usr/bin/env bash
# Round-2 probe 25: per-launch fixed cost vs per-step cost of the tile kernel
# (fuse 2/4/8/16, pinned shapes) on the headline frame — input to the
# register-resident persistent-kernel estimate.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe25
mkdir -p "$O"
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1 --fuse 2,4,8,16 --reps 80 --iters 10 --rounds 3 \
  --shapes "4,8,8;4,20,8;4,16,8;4,12,8;4,4,16" > "$O/sweep.jsonl" 2> "$O/sweep.err"
cat "$O/sweep.jsonl" | cut -c1-200
