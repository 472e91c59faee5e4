#!/bin/bash
# Round 4 (session 2): host API timeline beside the copies and kernels of the
# streamed single images (is the ~85 us stall mid-image the host issuing?).
set -o pipefail
OUT=gpurun_out/r04/api_trace
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tr -o run \
  -- python3 bench.py --gpus 1 --steps 4 --warmup 1 --no-check > $OUT/tr.json 2> $OUT/tr.err \
  || { echo "trace failed"; tail -5 $OUT/tr.err; exit 1; }
ls $OUT/tr
