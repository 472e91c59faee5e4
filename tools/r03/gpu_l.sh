#!/usr/bin/env bash
# Round-3 call L: tuner candidate-set A/B on the headline and 8-way device loops;
# copy-only pipeline period of the emulated 8-way rank.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/l
mkdir -p $O
timeout -k 10 200 python -u tools/r03/loop_probe.py > $O/loop_default.jsonl 2> $O/loop_default.err || { tail -5 $O/loop_default.err; exit 1; }
cat $O/loop_default.jsonl
PCONV_TUNE_CANDIDATES=19 timeout -k 10 300 python -u tools/r03/loop_probe.py > $O/loop_all.jsonl 2> $O/loop_all.err || { tail -5 $O/loop_all.err; exit 1; }
cat $O/loop_all.jsonl
for r in 0 1 40; do
  timeout -k 10 150 python bench.py --emulate 8:3 --reps $r --halo 40 > $O/emu8_reps$r.json 2> $O/emu8_reps$r.err || { tail -3 $O/emu8_reps$r.err; exit 1; }
  tail -1 $O/emu8_reps$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('emu8 reps=$r', d['ms_per_step'], d['loop_only']['ms_per_step'], d['copy_floor'])"
done
