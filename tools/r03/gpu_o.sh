#!/usr/bin/env bash
# Round-3 call O: RCCL on a stream that joined a capture through an event (the
# split exchange phase) — CLI stack first, then torch; stops at the first crash.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/o
mkdir -p $O
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for stack in cli torch; do
  for op in sendrecv_fork allreduce_fork; do
    for mode in none relaxed global; do
      f="$O/${stack}_${op}_${mode}"
      if [ "$stack" = cli ]; then
        timeout -k 5 90 "$CONV" --selftest rccl-capture --op $op --mode $mode > "$f.out" 2> "$f.err"
      else
        timeout -k 5 90 python3 -c "
import sys; sys.path.insert(0, '.')
import pconv
pconv.native.install_crash_handler()
print(pconv.native.rccl_capture_probe('$op', '$mode', 4096, 0))
" > "$f.out" 2> "$f.err"
      fi
      rc=$?
      echo "$stack $op $mode rc=$rc $(grep '^{' "$f.out" | head -c 200)"
      if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then
        echo "stopping after rc=$rc ($stack $op $mode)"; grep -v "NCCL INFO" "$f.err" | tail -n 45; exit 1
      fi
    done
  done
done
