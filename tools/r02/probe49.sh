#!/usr/bin/env bash
# Round-2 probe 49: D2H by a CU copy kernel (H2D on SDMA) vs the pitched SDMA
# D2H in the serving pipeline, interleaved on one box, with the box's copy
# rates for context.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe49
mkdir -p "$O"
timeout -k 5 120 tools/ubench/copy_bw 2520 20 > "$O/copy_bw.txt" 2>&1
tail -n 15 "$O/copy_bw.txt" | grep -E "concurrent \(per pair\)|SDMA H2D|D2H pitched"
for i in 1 2 3 4; do
  for m in sdma kernel; do
    timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --check --d2h $m >> "$O/n1_$m.jsonl" 2>> "$O/err.txt"
    timeout -k 10 120 python3 -u bench.py --emulate 8:3 --steps 40 --warmup 5 --d2h $m >> "$O/e8_$m.jsonl" 2>> "$O/err.txt"
  done
done
python3 -c "
import json
for f in ('n1_sdma', 'n1_kernel', 'e8_sdma', 'e8_kernel'):
    rows = [json.loads(l) for l in open('$O/' + f + '.jsonl') if l.startswith('{')]
    print(f, [r['ms_per_step'] for r in rows], 'mism', [r.get('mismatches') for r in rows], 'lat', [r['latency_ms'] for r in rows])"
