#!/usr/bin/env bash
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe13
mkdir -p "$O"
timeout -k 10 60 python3 tools/r02/model_rank.py > "$O/model_rank.txt" 2>&1 || true
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1 --fuse 6,8 --reps 24 --iters 2 --rounds 2 --width 32768 --height 32768 --channels grey --shapes auto > "$O/grey32768_auto.jsonl" 2> "$O/err.log"
cat "$O/grey32768_auto.jsonl"
