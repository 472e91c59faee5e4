#!/usr/bin/env bash
# Per-rank step of an N-way split on one GPU (bench.py --emulate N:r, an
# interior rank) over images in flight x fuse depth x concurrency.
# Output: one "key=value ... ms_per_step=X" line per run.
set -u
STEPS=${STEPS:-400}
SPECS=${SPECS:-8:3 4:1 2:1}
for SPEC in $SPECS; do
  for S in ${SLOTS:-3 4 6}; do
    for F in ${FUSES:-auto 16}; do
      for C in ${CONC:-off on}; do
        fa=""; [ "$F" != auto ] && fa="--fuse $F"
        line=$(timeout -k 5 120 python bench.py --emulate $SPEC --slots $S --concurrent $C $fa \
               --steps $STEPS --warmup 40 --loop-steps 50 2>/dev/null | grep '^{')
        ms=$(echo "$line" | grep -oE '"ms_per_step": [0-9.]+' | head -1 | grep -oE '[0-9.]+$')
        lp=$(echo "$line" | grep -oE '"us_per_rep": [0-9.]+' | head -1 | grep -oE '[0-9.]+$')
        fu=$(echo "$line" | grep -oE '"fuse": [0-9]+' | head -1 | grep -oE '[0-9]+$')
        echo "emulate=$SPEC slots=$S fuse=$F($fu) concurrent=$C ms_per_step=$ms loop_us_per_rep=$lp"
      done
    done
  done
done
