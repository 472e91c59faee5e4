#!/usr/bin/env bash
# Round-3 call M: copy-only pipeline period of the emulated 8-way rank (reps 0 / 1 / 40, same 40-row ghost zone).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/m
mkdir -p $O
for r in 0 1 40; do
  timeout -k 10 150 python bench.py --emulate 8:3 --reps $r --halo 40 > $O/emu8_reps$r.json 2> $O/emu8_reps$r.err || { tail -3 $O/emu8_reps$r.err; exit 1; }
  tail -1 $O/emu8_reps$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('emu8 reps=$r', d['ms_per_step'], d['loop_only']['ms_per_step'], d['copy_floor'])"
done
for r in 0 40; do
  timeout -k 10 150 python bench.py --reps $r --halo 8 > $O/n1_reps$r.json 2> $O/n1_reps$r.err || { tail -3 $O/n1_reps$r.err; exit 1; }
  tail -1 $O/n1_reps$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n1 reps=$r', d['ms_per_step'], d['loop_only']['ms_per_step'], d['copy_floor'])"
done
