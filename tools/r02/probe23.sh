#!/usr/bin/env bash
# Round-2 probe 23: runtime log of one cold conv process (idle GPU) to place
# the frames + first-kernel phase (code-object load).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe23
mkdir -p "$O"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
sleep 3
AMD_LOG_LEVEL=4 timeout -k 5 60 $CONV x.raw 1920 630 10 grey --synthetic 1 --json --out /tmp/p23.raw > "$O/conv_log4.txt" 2>&1
tail -n 1 "$O/conv_log4.txt" | cut -c1-400
