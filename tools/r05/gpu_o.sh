#!/bin/bash
# Round 5, fifteenth GPU call, after the fault of call n: the self-neighbour
# IPC transport of an emulated band now takes the neighbour's frame layout
# from its own engine (it read row_band(height, 1, 0) = the whole image, past
# the band's frame).  The new byte-placement test first (short limit), then
# the IPC suite and the multi-process / emulated bench tests, then the
# per-rank resident loops through IPC.
set -o pipefail
OUT=gpurun_out/r05/o
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ipc.py \
  -k self_neighbour > $OUT/tests_self.log 2>&1 || { echo "self-neighbour test failed"; tail -40 $OUT/tests_self.log; exit 1; }
tail -1 $OUT/tests_self.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu_ipc.py \
  > $OUT/tests_ipc.log 2>&1 || { echo "ipc tests failed"; tail -40 $OUT/tests_ipc.log; exit 1; }
tail -1 $OUT/tests_ipc.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_multiproc.py \
  > $OUT/tests_multiproc.log 2>&1 || { echo "multiproc tests failed"; tail -40 $OUT/tests_multiproc.log; exit 1; }
tail -1 $OUT/tests_multiproc.log
for e in 2:0 4:1 8:3; do
  n=${e%%:*}
  timeout -k 10 300 python -u bench.py --emulate $e --emulate-halo ipc --steps 100 --warmup 10 > $OUT/e${n}_ipc.json 2> $OUT/e${n}_ipc.err || { echo "bench failed"; tail -5 $OUT/e${n}_ipc.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], json.dumps(d.get('resident_loop_ipc')))" $OUT/e${n}_ipc.json
done
