#!/bin/bash
# Round 5, eighth GPU call: rocprofv3 kernel + memory-copy traces (stats) of
# the driver's command and of the 8-way per-rank proxy on the final tree.
set -o pipefail
OUT=gpurun_out/r05/h
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/drv -o run \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv.log 2>&1 || { echo "drv trace failed"; tail -20 $OUT/drv.log; exit 1; }
grep '^{' $OUT/drv.log | tail -1 | cut -c1-200
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/e8 -o run \
  -- python3 bench.py --emulate 8:3 --steps 100 --warmup 10 > $OUT/e8.log 2>&1 || { echo "e8 trace failed"; tail -20 $OUT/e8.log; exit 1; }
grep '^{' $OUT/e8.log | tail -1 | cut -c1-200
find $OUT -name "*stats.csv" | sort
