#!/bin/bash
# Round 5, fifth GPU call: the row-streaming kernel (bit-exact tests, then
# timed against the tile kernels on the production loops); the kernel and
# streaming tests after the step-form removal and the head-download stream
# change; head streaming vs step graphs per band size and burst length
# (tools/r05/burst.py); the driver's command.
set -o pipefail
OUT=gpurun_out/r05/e
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "stream_kernel" > $OUT/tests_stream.log 2>&1 || { echo "stream tests failed"; tail -30 $OUT/tests_stream.log; exit 1; }
tail -2 $OUT/tests_stream.log
timeout -k 10 400 python -u tools/r05/stream_ab.py > $OUT/stream_ab.jsonl 2> $OUT/stream_ab.err || { echo "stream A/B failed"; tail -20 $OUT/stream_ab.err; exit 1; }
cat $OUT/stream_ab.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_stream.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u tools/r05/burst.py > $OUT/burst.jsonl 2> $OUT/burst.err || { echo "burst failed"; tail -20 $OUT/burst.err; exit 1; }
cat $OUT/burst.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv_$i.json 2> $OUT/drv_$i.err || { echo "bench failed"; tail -5 $OUT/drv_$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['mismatches'])" $OUT/drv_$i.json
done
