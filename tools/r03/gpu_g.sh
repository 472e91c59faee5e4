#!/usr/bin/env bash
# Round-3 call G: float kernel tests + shape/fuse sweep, the multiproc test that went silent, 8-way emulations.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "float" -x -q --timeout 120 --timeout-method thread > $O/pytest_float.log 2>&1
rc=$?; tail -3 $O/pytest_float.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u tools/r03/float_sweep.py > $O/float_sweep.jsonl 2> $O/float_sweep.err
rc=$?; echo "sweep rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/float_sweep.err; exit 1; }
timeout -k 10 170 python -u -m pytest tests/test_gpu_multiproc.py -k "test_multiprocess_bands_one_gpu" -x -v --timeout 150 --timeout-method thread > $O/pytest_mp.log 2>&1
rc=$?; tail -30 $O/pytest_mp.log; [ $rc -ge 124 ] && exit 1
for m in preload slot_exchange slot_exchange_direct event overlap; do
  timeout -k 10 150 python bench.py --emulate 8:3 --emulate-halo $m --steps 200 --warmup 20 > $O/emulate8_$m.json 2> $O/emulate8_$m.err
  rc=$?; echo "emulate $m rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/emulate8_$m.err; exit 1; }
  python -c "import json; d=json.load(open('$O/emulate8_$m.json')); print('$m', d['ms_per_step'], d['config']['exchanges_per_step'], d['config']['halo_depth'], d['config']['step_graphs'], d['loop_only']['ms_per_step'])"
done
