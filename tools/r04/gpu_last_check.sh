#!/bin/bash
# Round 4 (session 2, end): the rebuilt binaries of the last tree — stream /
# engine GPU tests, smoke, and the driver's command once.
set -o pipefail
OUT=gpurun_out/r04/last_check
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
