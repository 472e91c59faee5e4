#!/usr/bin/env bash
# Round-3 call AA: (1) issue cost of the exact VALU encodings of the SWAR
# step (tools/ubench/valu_issue.hip); (2) A/B of the SWAR kernels with and
# without the add3 split (keep() in kernels/swar_device.hpp): bin/conv_old is
# the tree before the change, bin/conv after; alternating runs, loop time of
# the CLI (hipEvents), tuner on in both.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/aa
mkdir -p $O
B=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin
timeout -k 10 120 tools/ubench/bin/valu_issue > $O/valu_issue.txt 2>&1 || { cat $O/valu_issue.txt; exit 1; }
cat $O/valu_issue.txt
one() {  # tag bin args...
  local tag=$1 bin=$2; shift 2
  timeout -k 10 120 $B/$bin x.raw "$@" --synthetic 1 --json --quiet --out /tmp/ab.raw > /tmp/ab.json 2>$O/err.txt || { cat $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/ab.json')); print('$tag', '$bin', d['loop_s']*1e3, d.get('mismatches'))" | tee -a $O/ab.txt
}
for r in 1 2 3; do
  for bin in conv_old conv; do
    one g32768 $bin 32768 32768 200 grey
    one rgb1920 $bin 1920 2520 40 rgb --check
    one grey1920 $bin 1920 2520 40 grey --check
    one rgb8192 $bin 8192 8192 100 rgb
    one band8 $bin 1920 395 40 rgb --check
  done
done
rm -f /tmp/ab.raw
echo "call aa done"
