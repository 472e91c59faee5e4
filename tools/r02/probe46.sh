#!/usr/bin/env bash
# Round-2 probe 46: BASELINE.json configs on the final tree: N=1 bench and the
# emulated per-rank step of the 8-way split (one GPU; proxy, labelled so).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe46
mkdir -p "$O"
B="timeout -k 10 300 python3 -u bench.py"
$B --width 1920 --height 2520 --channels grey --reps 40 --steps 20 --warmup 5 >> "$O/configs.jsonl" 2>> "$O/err.txt"
$B --width 8192 --height 8192 --channels rgb --reps 100 --steps 10 --warmup 3 >> "$O/configs.jsonl" 2>> "$O/err.txt"
$B --width 8192 --height 8192 --channels rgb --reps 100 --steps 10 --warmup 3 --emulate 8:3 >> "$O/configs.jsonl" 2>> "$O/err.txt"
$B --width 32768 --height 32768 --channels grey --reps 200 --steps 5 --warmup 2 >> "$O/configs.jsonl" 2>> "$O/err.txt"
$B --width 32768 --height 32768 --channels grey --reps 200 --steps 5 --warmup 2 --emulate 8:3 >> "$O/configs.jsonl" 2>> "$O/err.txt"
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    if not l.startswith('{'): continue
    d = json.loads(l); c = d['config']
    print(c['model'], d.get('emulated', '')[:30], 'ms/step', d['ms_per_step'], 'value', d['value'], 'loop us/rep', d['loop_only']['us_per_rep'], 'floor', d['copy_floor']['floor_ms'])"
