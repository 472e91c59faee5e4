#!/usr/bin/env bash
# Round-3 call U: hardware queues x images in flight for the emulated 8-way
# rank (call S: 4+ slots slowed it 1.5-2x at GPU_MAX_HW_QUEUES = 8; call T's
# trace showed single 9-us launches stretched to ~50 us with the GPU idle —
# a queue-scheduling stall, not contention).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/u
mkdir -p $O
for q in 4 6 8 16; do
  for s in 3 4; do
    for m in preload slot_exchange; do
      timeout -k 10 150 python bench.py --emulate 8:3 --emulate-halo $m --slots $s --hw-queues $q > $O/e8_${m}_s${s}_q$q.json 2> $O/e8_${m}_s${s}_q$q.err \
        || { tail -5 $O/e8_${m}_s${s}_q$q.err; exit 1; }
      tail -1 $O/e8_${m}_s${s}_q$q.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m slots $s queues $q', d['ms_per_step'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"
    done
  done
done
