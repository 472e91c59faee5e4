#!/bin/bash
# Round 6, call J: a timing event before the first image of every burst
# (the effect the completion marks showed), A/B against --mark-timed; the
# engine / stream GPU tests; the driver's command x10.
set -o pipefail
OUT=gpurun_out/r06/j
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
for r in 0 1 2 3 4 5 6 7 8 9; do one drv_$r --gpus 1 --steps 20 --warmup 5 || exit 1; done
python tools/r06/summ_windows.py $OUT/drv_*.json
for r in 0 1 2 3 4 5; do
  one plain_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 2 || exit 1
  one marked_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 2 --mark-timed || exit 1
done
python tools/r06/summ_windows.py $OUT/plain_*.json $OUT/marked_*.json
