#!/bin/bash
# Round 5, twelfth GPU call: streamed head image with its chunk copies
# alternating over two slots' streams (--head-alt-copies 0/1/2/3): the head
# streaming tests, then the driver's command per setting, interleaved (3
# rounds), for latency_ms and ms/step.
set -o pipefail
OUT=gpurun_out/r05/l
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu_stream.py -k head_stream \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for alt in 0 1 2 3; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --head-alt-copies $alt > $OUT/alt${alt}_$r.json 2> $OUT/alt${alt}_$r.err || { echo "bench failed"; tail -5 $OUT/alt${alt}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], d['mismatches'])" $OUT/alt${alt}_$r.json
  done
done
