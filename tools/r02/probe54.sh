#!/usr/bin/env bash
# Round-2 probe 54: A/B of the buffer-op tile candidate (PCONV_PREFETCH=0 vs
# default) on the driver's bench command and the emulated 8-way rank, same box,
# interleaved.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe54
mkdir -p "$O"
: > "$O/ab.jsonl"
for i in 1 2; do
  for pf in 0 default; do
    for em in "" "--emulate 8:3"; do
      if [ "$pf" = 0 ]; then export PCONV_PREFETCH=0; else unset PCONV_PREFETCH; fi
      timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 $em > "$O/b.json" 2>> "$O/err.txt"
      python3 -c "
import json,sys
d=json.load(open('$O/b.json')); print(json.dumps({'prefetch':'$pf','emulate':'$em','ms':d['ms_per_step'],'loop':d['loop_only']['ms_per_step'],'lat':d['latency_ms'],'floor':d['copy_floor']['floor_ms']}))" >> "$O/ab.jsonl"
    done
  done
done
unset PCONV_PREFETCH
cat "$O/ab.jsonl"
