#!/bin/bash
# Round 5, thirteenth GPU call: chunk count of the streamed head image with
# its uploads alternating over two streams (--stream-chunks 3/4/5/6/8), the
# driver's command, 2 interleaved rounds; the head streaming tests first.
set -o pipefail
OUT=gpurun_out/r05/m
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu_stream.py \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for c in 3 4 5 6 8; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --stream-chunks $c > $OUT/c${c}_$r.json 2> $OUT/c${c}_$r.err || { echo "bench failed"; tail -5 $OUT/c${c}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], d['mismatches'])" $OUT/c${c}_$r.json
  done
done
