#!/bin/bash
# Round 4 (session 2): per-rank 8-way proxy in every halo mode with 3/4 slots
# (single-dispatch IPC exchange), N=1 with 3/4 slots, the native stack's
# steps (conv --bench: ROCm 7.2 HIP runtime) next to torch's, and the
# BASELINE large frames in steady state and one image alone.
set -o pipefail
bash tools/r04/gpu_e2.sh || exit 1
bash tools/r04/gpu_big.sh || exit 1
