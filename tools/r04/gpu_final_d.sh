#!/bin/bash
# Round 4 (session 2): the whole GPU suite, smoke and the driver's command on
# the final defaults (4 images in flight), then the reference's CUDA table
# with `conv --backend auto` after its two-stage pricing (sample, then first full repetition).
set -o pipefail
OUT=gpurun_out/r04/final_d
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
for i in a b c; do
  timeout -k 10 150 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench failed"; tail -5 $OUT/bench_$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], d.get('mismatches'), d['config']['images_in_flight'])" $OUT/bench_$i.json
done
AUTO_OUT=gpurun_out/r04/auto_d bash tools/r04/gpu_auto.sh || exit 1
