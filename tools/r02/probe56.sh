#!/usr/bin/env bash
# Round-2 probe 56: memory counters of the current production kernels: the
# headline's buffer-op tile kernel (tuned, and pinned to {4,8,8} paired) and
# 32768^2 grey at the new fuse depth 12 (tuned).
set -euo pipefail
export TMPDIR=/tmp
tools/r02/pmc_mem.sh head_pf 1920 2520 rgb 40 8 5
PCONV_PREFETCH=1 PCONV_SWAR_SHAPE=4,8,8 PCONV_SWAR_ALT=1 tools/r02/pmc_mem.sh head_pf_pinned 1920 2520 rgb 40 8 5
tools/r02/pmc_mem.sh big_f12 32768 32768 grey 200 12 1
python3 tools/summarize_pmc_mem.py gpurun_out/r02/pmc_head_pf --rows 2520 --row-bytes 5760 --steps 8 > gpurun_out/r02/pmc_head_pf/summary.md
python3 tools/summarize_pmc_mem.py gpurun_out/r02/pmc_head_pf_pinned --rows 2520 --row-bytes 5760 --steps 8 > gpurun_out/r02/pmc_head_pf_pinned/summary.md
python3 tools/summarize_pmc_mem.py gpurun_out/r02/pmc_big_f12 --rows 32768 --row-bytes 32768 --steps 12 > gpurun_out/r02/pmc_big_f12/summary.md
head -12 gpurun_out/r02/pmc_head_pf_pinned/summary.md
