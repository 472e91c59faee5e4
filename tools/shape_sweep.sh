#!/usr/bin/env bash
# Sweep SWAR temporal tile shapes (PCONV_SWAR_SHAPE=M,NW) over band sizes.
# usage: tools/shape_sweep.sh [fuse]
F=${1:-8}
for W in 1 2 4 8; do
  for S in auto 8,8 8,4 16,4 4,8 4,16 2,16; do
    if [ "$S" = auto ]; then unset PCONV_SWAR_SHAPE; else export PCONV_SWAR_SHAPE=$S; fi
    R=$(( W > 1 ? 1 : 0 ))
    out=$(python tools/kernel_sweep.py --fuse $F --world $W --rank $R --rounds 2 --iters 10 2>/dev/null | tail -1)
    echo "world=$W shape=$S $out" | cut -c1-200
  done
done
