#!/usr/bin/env bash
# Round-2 probe 36: resident kernel time vs repetitions (per-step arithmetic
# inside a phase, per-phase hand-off) on the headline frame.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe36
mkdir -p "$O"
timeout -k 10 240 python3 -u tools/resident_sweep.py --frames 1920x2520:rgb --reps 1,2,4,8,16,24,32,40 > "$O/sweep.jsonl" 2> "$O/sweep.err"
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    d = json.loads(l); print(d['path'], d['reps'], d['launches'], d['ms_per_loop'])"
