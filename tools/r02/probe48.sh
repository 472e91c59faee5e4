#!/usr/bin/env bash
# Round-2 probe 48: why the grey headline-size step (0.255 ms) is slower than
# its copies (0.11 ms per H2D+D2H pair): pipeline variants and a stage trace.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe48
mkdir -p "$O"
B="timeout -k 10 120 python3 -u bench.py --width 1920 --height 2520 --channels grey --reps 40"
$B --steps 20 --warmup 5 >> "$O/v.jsonl" 2>> "$O/err.txt"; echo default >> "$O/labels.txt"
$B --steps 50 --warmup 10 >> "$O/v.jsonl" 2>> "$O/err.txt"; echo steps50 >> "$O/labels.txt"
$B --steps 20 --warmup 5 --slots 1 >> "$O/v.jsonl" 2>> "$O/err.txt"; echo slots1 >> "$O/labels.txt"
$B --steps 20 --warmup 5 --graph-capture off >> "$O/v.jsonl" 2>> "$O/err.txt"; echo nograph >> "$O/labels.txt"
PCONV_STREAM=0 $B --steps 20 --warmup 5 >> "$O/v.jsonl" 2>> "$O/err.txt"; echo nostream >> "$O/labels.txt"
$B --steps 20 --warmup 5 --graph-capture off --trace 30 --trace-out "$O/trace.json" >> "$O/v.jsonl" 2>> "$O/err.txt"; echo trace >> "$O/labels.txt"
python3 -c "
import json
labels = open('$O/labels.txt').read().split()
rows = [json.loads(l) for l in open('$O/v.jsonl') if l.startswith('{')]
for lab, d in zip(labels, rows):
    print(lab, d['ms_per_step'], 'lat', d['latency_ms'], 'loop', d['loop_only']['ms_per_step'], 'graphs', d['config']['step_graphs'], 'launches', d['config']['launches_per_step'])
t = json.load(open('$O/trace.json'))
ms = t['ms'][-10:]
for r in ms: print('trace', [round(x, 3) for x in r])
"
