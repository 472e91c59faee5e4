#!/usr/bin/env bash
# Round-3 diagnosis of the round-2 segfault (RCCL send/recv inside a hipGraph
# capture, 1-rank self communicator): every (stack, op, capture mode) in its
# own process with NCCL_DEBUG=INFO and the native crash reporter, so a crash
# names its step, its native frames and the RCCL build.
#   stacks: the conv CLI (ROCm's HIP runtime + librccl) first, then a torch
#   process (torch's bundled HIP runtime + librccl).
# The script stops at the first crash, abort or timeout (nothing more runs on
# the GPU after it); its output files name the failing case.
set -uo pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r03/capture}
STACKS=${2:-"cli torch"}
mkdir -p "$O"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for stack in $STACKS; do
  for op in sendrecv allreduce; do
    for mode in none global thread_local relaxed; do
      f="$O/${stack}_${op}_${mode}"
      if [ "$stack" = cli ]; then
        NCCL_DEBUG=INFO timeout -k 5 90 "$CONV" --selftest rccl-capture --op $op --mode $mode > "$f.out" 2> "$f.err"
      else
        NCCL_DEBUG=INFO timeout -k 5 90 python3 -c "
import sys; sys.path.insert(0, '.')
import pconv
pconv.native.install_crash_handler()
print(pconv.native.rccl_capture_probe('$op', '$mode', 4096, 0))
" > "$f.out" 2> "$f.err"
      fi
      rc=$?
      echo "$stack $op $mode rc=$rc $(head -c 300 "$f.out")"
      if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then
        echo "stopping after rc=$rc ($stack $op $mode)"; tail -n 40 "$f.err"; exit 1
      fi
    done
  done
done
