#!/usr/bin/env bash
# Round-3 call T: traces of the emulated 8-way rank with 4 images in flight
# (call S: 4 slots doubled the period: 0.109 vs 0.055 ms) and, for
# comparison, 3 — which engine or gap serialises.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/t
mkdir -p $O
for s in 4 3; do
  for m in preload slot_exchange; do
    timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof_${m}_s$s -o run -- \
      python3 bench.py --emulate 8:3 --emulate-halo $m --slots $s --steps 100 --warmup 20 > $O/prof_${m}_s$s.log 2>&1 \
      || { tail -5 $O/prof_${m}_s$s.log; exit 1; }
    grep '^{' $O/prof_${m}_s$s.log | tail -1 | cut -c1-200
  done
done
