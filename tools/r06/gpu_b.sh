#!/bin/bash
# Round 6, call B: which copy engine serves which slot stream?
#  1. one run of the driver's command with the HIP runtime's full log; the
#     copy / engine lines kept;
#  2. interleaved A/B of ROCr's SDMA engine policies (gang copies,
#     recommended engines) against the default, 3 rounds.
set -o pipefail
OUT=gpurun_out/r06/b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
ls -la /sys/class/kfd/kfd/proc/ > $OUT/kfd_proc.txt 2>&1 || true
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x7fffffff one fulllog --gpus 1 --steps 20 --warmup 5 --diag-windows 2 || exit 1
grep -aiE "engine|sdma|blit|copy|rect|graph" $OUT/fulllog.err | head -c 30000000 > $OUT/fulllog_copy.txt || true
grep -aiE "engine|sdma" $OUT/fulllog.err | head -c 3000000 > $OUT/fulllog_engine.txt || true
wc -l $OUT/fulllog.err $OUT/fulllog_copy.txt $OUT/fulllog_engine.txt
rm -f $OUT/fulllog.err
for r in 0 1 2; do
  one base_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  HSA_ENABLE_SDMA_GANG=0 one nogang_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  HSA_ENABLE_SDMA_RECOMMENDED_ENG=0 one norec_$r --gpus 1 --steps 20 --warmup 5 || exit 1
done
python tools/r06/summ_windows.py $OUT/*.json
