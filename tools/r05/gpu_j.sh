#!/bin/bash
# Round 5, tenth GPU call: emulated-rank halo modes with the resident MPI
# loop (RCCL send/recv to self), and the per-rank resident loop of the 2-,
# 4- and 8-way splits of the headline (event mode).
set -o pipefail
OUT=gpurun_out/r05/j
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_multiproc.py -k emulated_rank > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for e in 2:0 4:1 8:3; do
  n=${e%%:*}
  timeout -k 10 300 python -u bench.py --emulate $e --emulate-halo event --steps 100 --warmup 10 > $OUT/e${n}_event.json 2> $OUT/e${n}_event.err || { echo "bench failed"; tail -5 $OUT/e${n}_event.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], json.dumps(d.get('resident_loop')))" $OUT/e${n}_event.json
done
