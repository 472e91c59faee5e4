#!/bin/bash
# Round 6, call W: DPP vs LDS-permute lane crossing in the SWAR step (two
# builds of the extension, ab/dpp and ab/lds, swapped in place between runs):
# the kernel tests on the LDS build, then the tuned loops A/B/A/B/A/B.
set -o pipefail
OUT=gpurun_out/r06/w
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
PKG=parallel-image-convolution-using-mpi-openmp-and-cuda_amd
SO=$(basename ab/dpp/_pconv_native*.so)
use() { cp ab/$1/$SO $PKG/$SO; }
use lds
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_stream.py -k "not native_bench" > $OUT/tests_lds.txt 2>&1 || { echo "lds tests failed"; tail -30 $OUT/tests_lds.txt; use dpp; exit 1; }
tail -1 $OUT/tests_lds.txt
for r in 0 1 2; do
  for v in dpp lds; do
    use $v
    timeout -k 10 300 python -u tools/r06/xlane_ab.py --variant $v > $OUT/ab_${v}_$r.jsonl 2> $OUT/ab_${v}_$r.err || { echo "ab $v failed"; tail -5 $OUT/ab_${v}_$r.err; use dpp; exit 1; }
    python -c "import json,sys; [print(sys.argv[1], d['loop'], d['us_per_rep']) for d in map(json.loads, open(sys.argv[1]))]" $OUT/ab_${v}_$r.jsonl
  done
done
use dpp
