#!/usr/bin/env bash
# ms/step of the serving pipeline over band heights x slots x concurrency.
for H in ${HEIGHTS:-315 630 2520}; do
  for S in 1 2 3 4; do
    for C in off on; do
      [ $S = 1 ] && [ $C = on ] && continue
      st=$(( H > 1000 ? 100 : 300 ))
      r=$(python bench.py --height $H --slots $S --concurrent $C --steps $st --warmup 20 2>/dev/null | grep -oE '"ms_per_step": [0-9.]+' | head -1 | grep -oE '[0-9.]+$')
      echo "height=$H slots=$S concurrent=$C ms_per_step=$r"
    done
  done
done
