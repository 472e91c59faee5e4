#!/usr/bin/env bash
# Sweep SWAR temporal tile shapes (PCONV_SWAR_SHAPE=lw,m,nw) over band sizes.
# usage: tools/shape_sweep.sh [fuse] [worlds]
F=${1:-8}
WS=${2:-"1 2 4 8"}
SHAPES=$(python -c "import sys; sys.path.insert(0,'.'); import pconv; print(' '.join('%d,%d,%d'%s for s in pconv.native.swar_shapes()))")
for W in $WS; do
  for S in auto $SHAPES; do
    if [ "$S" = auto ]; then unset PCONV_SWAR_SHAPE; else export PCONV_SWAR_SHAPE=$S; fi
    R=$(( W > 1 ? 1 : 0 ))
    out=$(python tools/kernel_sweep.py --fuse $F --world $W --rank $R --rounds 2 --iters 10 2>/dev/null | tail -1)
    us=$(echo "$out" | grep -oE '"us_per_rep": [0-9.]+' | grep -oE '[0-9.]+$')
    echo "world=$W fuse=$F shape=$S us_per_rep=$us"
  done
done
