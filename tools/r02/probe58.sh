#!/usr/bin/env bash
# Round-2 probe 58: fusion depth for the emulated per-rank bands of the
# headline (N = 2/4/8, pre-loaded 40-row ghost zones): fewer, deeper launches
# against the default 8, interleaved, two rounds.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe58
mkdir -p "$O"
: > "$O/fuse.jsonl"
for round in 1 2; do
  for em in 8:3 4:1 2:0; do
    for f in 8 10 14 20; do
      timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 40 --warmup 10 --emulate $em --fuse $f > "$O/b.json" 2>> "$O/err.txt"
      python3 -c "
import json
d=json.load(open('$O/b.json')); print(json.dumps({'round':$round,'emulate':'$em','fuse':$f,'ms':d['ms_per_step'],'loop':d['loop_only']['ms_per_step'],'lat':d['latency_ms'],'launches':d['config']['launches_per_step']}))" >> "$O/fuse.jsonl"
    done
  done
done
cat "$O/fuse.jsonl"
