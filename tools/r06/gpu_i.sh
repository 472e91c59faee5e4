#!/bin/bash
# Round 6, call I: every image's completion event recorded right behind it
# (the effect the completion marks showed), A/B against --mark-timed; the
# engine / stream GPU tests; the driver's command x10.
set -o pipefail
OUT=gpurun_out/r06/i
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
for r in 0 1 2 3 4 5 6 7 8 9; do one drv_$r --gpus 1 --steps 20 --warmup 5 || exit 1; done
python tools/r06/summ_windows.py $OUT/drv_*.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_engine.py tests/test_gpu_stream.py \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 0 1 2 3; do
  one plain_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 2 || exit 1
  one marked_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 2 --mark-timed || exit 1
done
python tools/r06/summ_windows.py $OUT/plain_*.json $OUT/marked_*.json
