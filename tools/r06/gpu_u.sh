#!/bin/bash
# Round 6, call U: concurrent copy floors measured as one long run per rank
# (CopyProbe: >= 20 ms of copies at the solo rate, its mean) — the copy
# tests, then the N = 2 / 4 / 8 rehearsals of the driver's SCALE command
# with N ranks on the one GPU (N x contention on one link expected).
set -o pipefail
OUT=gpurun_out/r06/u
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_engine.py \
  -k "copy" > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
sed -e 's#^OUT=gpurun_out/r06/t#OUT=gpurun_out/r06/u#' -e '/n8_rgb8192\|n8_grey32768/d' tools/r06/gpu_t.sh > $OUT/rehearsal.sh
bash $OUT/rehearsal.sh || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv.json 2> $OUT/drv.err || { echo "drv failed"; tail -5 $OUT/drv.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/drv.json').read().strip().splitlines()[-1]); print('drv', d['ms_per_step'], d['latency_ms'], d['copy_floor'])"
