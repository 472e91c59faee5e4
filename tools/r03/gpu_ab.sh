#!/usr/bin/env bash
# Round-3 call AB: pair-sum SWAR step (P_j = X_j + X_{j+CH}, H_k = P_{k-CH} + P_k;
# no VOP3 / add3 in the step) — kernel GPU tests first (bit-exact vs the
# oracles), then A/B against bin/conv_old (the tree before the change).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resident.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?; tail -3 $O/pytest_kernels.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest_kernels.log | head -30; exit 1; }
B=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin
one() {  # tag bin args...
  local tag=$1 bin=$2; shift 2
  timeout -k 10 120 $B/$bin x.raw "$@" --synthetic 1 --json --quiet --out /tmp/ab.raw > /tmp/ab.json 2>$O/err.txt || { cat $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/ab.json')); print('$tag', '$bin', round(d['loop_s']*1e3,4), d.get('mismatches'))" | tee -a $O/ab.txt
}
for r in 1 2 3; do
  for bin in conv_old conv; do
    one g32768 $bin 32768 32768 200 grey
    one rgb1920 $bin 1920 2520 40 rgb --check
    one grey1920 $bin 1920 2520 40 grey --check
    one rgb8192 $bin 8192 8192 100 rgb
    one band8 $bin 1920 395 40 rgb --check
    one g16384 $bin 16384 16384 40 grey
  done
done
rm -f /tmp/ab.raw
echo "call ab done"
