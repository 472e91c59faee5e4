#!/usr/bin/env bash
# rocprofv3 evidence for the stencil kernels (run on the GPU box).
#   pass 1: kernel trace + stats (per-kernel durations, launch gaps)
#   pass 2: SQ/GRBM counters (VALU instructions, wave cycles, busy) — own run,
#           kernel-trace only (no sys/runtime trace with --pmc on this pool)
#   pass 3: TCC counters (FETCH_SIZE / WRITE_SIZE: HBM/MALL traffic)
# Outputs: gpurun_out/prof_<tag>/ ; summaries are copied to profiles/ by hand.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TAG=${1:-rgb}
shift || true
ARGS=${*:-"--fuse 1,8 --rounds 1 --iters 5"}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/kernel_sweep.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_sq" -o run \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -- \
  python3 tools/kernel_sweep.py $ARGS > "$OUT/pmc_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_tcc" -o run \
  --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum -- \
  python3 tools/kernel_sweep.py $ARGS > "$OUT/pmc_tcc.log" 2>&1
echo "profile $TAG done"
