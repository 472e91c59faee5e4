#!/usr/bin/env bash
# Does holding an RCCL communicator (as every N>1 rank does) slow the
# per-rank serving pipeline?  bench --emulate 8:3 with / without a 1-rank comm.
B="timeout -k 5 120 python bench.py --emulate 8:3 --steps 400 --warmup 40 --loop-steps 5"
for S in 3; do
  for X in "" "--emulate-rccl" "" "--emulate-rccl"; do
    line=$($B --slots $S $X 2>/dev/null | grep '^{')
    echo "slots=$S ${X:-no-comm} $(echo "$line" | grep -oE '"ms_per_step": [0-9.]+' | head -1)"
  done
done
