#!/usr/bin/env bash
# Round-2 probe 9: per-launch fixed cost of the headline tile kernel —
# empty / memory-only launches of its grid shape, and a fuse 1..8 sweep with
# the tile shape pinned (fit: launch time = fixed + steps x per-step).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe9
mkdir -p "$O"
timeout -k 10 60 tools/ubench/launch_cost > "$O/launch_cost.jsonl" 2>&1
cat "$O/launch_cost.jsonl"
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 1,2,3,4,5,6,7,8 --reps 840 --iters 2 --rounds 2 --shapes "4,8,8" > "$O/fuse_pinned_448.jsonl" 2> "$O/fuse_pinned.err"
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 1,2,3,4,5,6,7,8 --reps 840 --iters 2 --rounds 2 --shapes auto > "$O/fuse_auto.jsonl" 2>> "$O/fuse_pinned.err"
echo probe9 done
