#!/bin/bash
# Round 5, seventh GPU call: the IPC pull with every lane's granules in
# flight at once (pull_sides: no per-granule branches, 16 KB per workgroup
# and side): the IPC tests, the pull probe from HBM and pinned host memory
# per workgroup count, the 8-way proxy with IPC halos.
set -o pipefail
OUT=gpurun_out/r05/g
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu_ipc.py \
  > $OUT/tests_ipc.log 2>&1 || { echo "ipc tests failed"; tail -30 $OUT/tests_ipc.log; exit 1; }
tail -1 $OUT/tests_ipc.log
timeout -k 10 200 python -u tools/r05/ipc_probe.py --workgroups 0,8,16,29,32,64 > $OUT/ipc_probe.jsonl 2> $OUT/ipc_probe.err || { echo "probe failed"; tail -20 $OUT/ipc_probe.err; exit 1; }
cat $OUT/ipc_probe.jsonl
for m in grid single; do
  timeout -k 10 300 python -u bench.py --emulate 8:3 --emulate-halo ipc --ipc-pull $m --steps 300 --warmup 10 > $OUT/e8_ipc_$m.json 2> $OUT/e8_ipc_$m.err || { echo "bench failed"; tail -5 $OUT/e8_ipc_$m.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['copy_floor']['pair_ms'], d.get('mismatches'))" $OUT/e8_ipc_$m.json
done
