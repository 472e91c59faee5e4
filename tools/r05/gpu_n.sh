#!/bin/bash
# Round 5, fourteenth GPU call: the resident MPI loop with HIP-IPC pulls
# (resident_loop_ipc): multi-process bench rehearsals and emulated ranks,
# then the per-rank proxies of the 2-, 4- and 8-way bands.
set -o pipefail
OUT=gpurun_out/r05/n
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_multiproc.py \
  > $OUT/tests_multiproc.log 2>&1 || { echo "multiproc tests failed"; tail -40 $OUT/tests_multiproc.log; exit 1; }
tail -1 $OUT/tests_multiproc.log
for e in 2:0 4:1 8:3; do
  n=${e%%:*}
  timeout -k 10 300 python -u bench.py --emulate $e --emulate-halo ipc --steps 100 --warmup 10 > $OUT/e${n}_ipc.json 2> $OUT/e${n}_ipc.err || { echo "bench failed"; tail -5 $OUT/e${n}_ipc.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], json.dumps(d.get('resident_loop_ipc')))" $OUT/e${n}_ipc.json
done
