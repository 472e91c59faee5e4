#!/usr/bin/env bash
# Round-2 probe 11: per-rank step of the N-way split (one GPU, --emulate)
# with the D2H copy vs the zero-copy store fused into the last launch.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe11
mkdir -p "$O"
for emu in 8:3 8:0 4:1 2:0; do
  for zc in off on; do
    for i in 1 2; do
      timeout -k 10 120 python3 -u bench.py --emulate $emu --zero-copy-out $zc --steps 200 --warmup 20 > "$O/emu_${emu/:/_}_zc${zc}_$i.json" 2> "$O/emu.err"
      python3 -c "import json,sys; d=json.load(open('$O/emu_${emu/:/_}_zc${zc}_$i.json')); print('$emu', 'zc=$zc', d['ms_per_step'], d['config']['zero_copy_out'], d['latency_ms'], d['copy_floor'])"
    done
  done
done
echo probe11 done
