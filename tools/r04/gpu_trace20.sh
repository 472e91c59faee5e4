#!/bin/bash
# Round 4 (session 2): where the driver's 20-image window loses time — a
# kernel + copy trace of exactly its command (stagger on / off); the auto
# backend's GPU tests and the handoff comparison on the final policy.
set -o pipefail
OUT=gpurun_out/r04/trace20
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k auto -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_auto.txt 2>&1 || { echo "auto tests failed"; tail -40 $OUT/pytest_auto.txt; exit 1; }
tail -1 $OUT/pytest_auto.txt
for st in 1 0; do
  PCONV_STAGGER=$st timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/st$st -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-check > $OUT/st$st.json 2> $OUT/st$st.err \
    || { echo "trace st$st failed"; tail -5 $OUT/st$st.err; exit 1; }
  tail -1 $OUT/st$st.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('stagger', $st, d['ms_per_step'])"
  python tools/r04/copy_kernel_timeline.py $OUT/st$st --first 400 > $OUT/st${st}_timeline.txt
done
C=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for j in "8192 8192 100 rgb" "32768 32768 200 grey"; do
  set -- $j
  for ho in 0 1; do
    n=auto_${1}_${4}_ho$ho
    PCONV_AUTO_HANDOFF=$ho timeout -k 10 300 $C /tmp/x.raw $1 $2 $3 $4 --synthetic 7 --backend auto --json --quiet --out /tmp/o.raw > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['e2e_s'],4), d['cpu_reps'], d['gpu_reps'], d['auto_choice'])" $OUT/$n.json
  done
  timeout -k 10 300 $C /tmp/x.raw $1 $2 $3 $4 --synthetic 7 --backend hip --json --quiet --out /tmp/o.raw > $OUT/hip_${1}_$4.json 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['e2e_s'],4))" $OUT/hip_${1}_$4.json
done
