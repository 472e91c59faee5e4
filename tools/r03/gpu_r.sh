#!/usr/bin/env bash
# Round-3 call R: kernel + copy traces of the emulated 8-way rank (rank 3)
# in the pre-loaded and the slot-exchange pipelines — which engine sets the
# period (tools/r03/slot_timeline.py analyses the CSVs on the CPU).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/r
mkdir -p $O
for m in preload slot_exchange; do
  timeout -k 10 150 python bench.py --emulate 8:3 --emulate-halo $m --steps 300 --warmup 30 > $O/$m.json 2> $O/$m.err \
    || { tail -5 $O/$m.err; exit 1; }
  tail -1 $O/$m.json | cut -c1-160
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof_$m -o run -- \
    python3 bench.py --emulate 8:3 --emulate-halo $m --steps 300 --warmup 30 > $O/prof_$m.log 2>&1 \
    || { tail -5 $O/prof_$m.log; exit 1; }
  ls $O/prof_$m
done
