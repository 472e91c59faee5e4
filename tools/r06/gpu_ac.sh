#!/bin/bash
# Round 6, call AC: the final tree's driver line on one more box (x10).
set -o pipefail
OUT=gpurun_out/r06/ac
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
for r in 0 1 2 3 4 5 6 7 8 9; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv_$r.json 2> $OUT/drv_$r.err || { echo "bench $r failed"; tail -5 $OUT/drv_$r.err; exit 1; }
done
python tools/r06/summ_windows.py $OUT/drv_*.json
python tools/r06/distributions.py "AC=$OUT/drv_*.json"
