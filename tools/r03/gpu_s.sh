#!/usr/bin/env bash
# Round-3 call S: images in flight (slots) vs the period of the emulated
# 8-way rank (preload and slot-exchange pipelines) and of the 1-GPU headline.
# Call R's trace showed the 8-way slot chain (H2D, exchange, 5 launches, D2H
# plus graph-relaunch gaps, ~170 us) divided over 3 slots setting the period.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/s
mkdir -p $O
for s in 3 4 5 6; do
  for m in preload slot_exchange; do
    timeout -k 10 150 python bench.py --emulate 8:3 --emulate-halo $m --slots $s > $O/e8_${m}_s$s.json 2> $O/e8_${m}_s$s.err \
      || { tail -5 $O/e8_${m}_s$s.err; exit 1; }
    tail -1 $O/e8_${m}_s$s.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m slots $s', d['ms_per_step'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"
  done
done
for s in 3 4 5; do
  timeout -k 10 150 python bench.py --slots $s > $O/n1_s$s.json 2> $O/n1_s$s.err || { tail -5 $O/n1_s$s.err; exit 1; }
  tail -1 $O/n1_s$s.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline slots $s', d['ms_per_step'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"
done
