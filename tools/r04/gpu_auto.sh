#!/bin/bash
# Round 4 (session 2): the reference's CUDA table (README.pdf p.7, 48 cells,
# one cold process per run) with `conv --backend auto` (CPU repetitions while
# the GPU comes up, GPU takes over; short jobs never touch the GPU) next to
# `--backend hip`, back to back and with an idle gap before each process;
# plus a handoff run on a job long enough for the GPU to take over.
set -o pipefail
OUT=${AUTO_OUT:-gpurun_out/r04/auto}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
T="timeout -k 10 600 python -u tools/ref_tables.py cuda --runs 3 --tmp /tmp/pconv_ref"
$T --out $OUT/cuda_auto.jsonl --extra --backend auto > $OUT/cuda_auto.log 2>&1 || { echo "auto table failed"; tail -5 $OUT/cuda_auto.log; exit 1; }
$T --out $OUT/cuda_hip.jsonl --extra --backend hip > $OUT/cuda_hip.log 2>&1 || { echo "hip table failed"; tail -5 $OUT/cuda_hip.log; exit 1; }
$T --gap 1.0 --out $OUT/cuda_auto_idle.jsonl --extra --backend auto > $OUT/cuda_auto_idle.log 2>&1 || { echo "auto idle table failed"; tail -5 $OUT/cuda_auto_idle.log; exit 1; }
python tools/ref_tables.py report $OUT/cuda_auto.jsonl --md $OUT/cuda_auto.md > /dev/null && tail -3 $OUT/cuda_auto.md
python tools/ref_tables.py report $OUT/cuda_hip.jsonl --md $OUT/cuda_hip.md > /dev/null && tail -3 $OUT/cuda_hip.md
C=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for j in "1920 2520 400 rgb" "4096 4096 60 rgb" "8192 8192 100 rgb" "32768 32768 200 grey"; do
  set -- $j
  n=handoff_${1}x${2}_${4}_$3
  timeout -k 10 300 $C /tmp/x.raw $1 $2 $3 $4 --synthetic 7 --backend auto --json --quiet --out /tmp/o.raw > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; exit 1; }
  timeout -k 10 300 $C /tmp/x.raw $1 $2 $3 $4 --synthetic 7 --backend hip --json --quiet --out /tmp/o.raw > $OUT/${n}_hip.json 2> $OUT/${n}_hip.err || { echo "$n hip failed"; exit 1; }
  python -c "
import json,sys
a=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], 'auto e2e', round(a['e2e_s'],4), 'cpu_reps', a['cpu_reps'], 'gpu_reps', a['gpu_reps'], a['auto_choice'], '| hip e2e', round(b['e2e_s'],4))
" $OUT/$n.json $OUT/${n}_hip.json $n
done
