#!/bin/bash
# Round 5, ninth GPU call: bench.py's resident MPI-loop measurement at N>1
# (halo_modes.event.resident_loop): the multi-process bench rehearsals.
set -o pipefail
OUT=gpurun_out/r05/i
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_multiproc.py \
  > $OUT/tests_multiproc.log 2>&1 || { echo "multiproc tests failed"; tail -40 $OUT/tests_multiproc.log; exit 1; }
tail -1 $OUT/tests_multiproc.log
port=29631
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $port \
  bench.py --gpus 4 --steps 20 --warmup 5 --transport gloo-host > $OUT/n4.json 2> $OUT/n4.err || { echo "n4 failed"; tail -20 $OUT/n4.err; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['ms_per_step'], d['halo_select'], json.dumps(d.get('resident_loop')))" $OUT/n4.json
