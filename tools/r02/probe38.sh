#!/usr/bin/env bash
# Round-2 probe 38: deeper fusion for the 8-way band (fewer, larger launches).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe38
mkdir -p "$O"
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 8,4 --fuse 8,10,14,20 --reps 40 --shapes auto --iters 20 --rounds 3 > "$O/sweep.jsonl" 2> "$O/sweep.err"
python3 -c "
import json
for l in open('$O/sweep.jsonl'):
    d = json.loads(l); print(d['world'], d['fuse'], d['launches'], d['us_per_rep'], d.get('tuned_keys'))"
