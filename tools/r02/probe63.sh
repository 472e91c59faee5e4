#!/usr/bin/env bash
# Round-2 probe 63: why the buffer-op tile kernel is slow on grey frames:
# the same counters for k_swar and k_swar_pf pinned to {4,8,8} paired on
# 1920x2520 grey.
set -euo pipefail
export TMPDIR=/tmp
PCONV_PREFETCH=0 PCONV_SWAR_SHAPE=4,8,8 PCONV_SWAR_ALT=1 tools/r02/pmc_mem.sh grey_tile 1920 2520 grey 40 8 5
PCONV_PREFETCH=1 PCONV_SWAR_SHAPE=4,8,8 PCONV_SWAR_ALT=1 tools/r02/pmc_mem.sh grey_buf 1920 2520 grey 40 8 5
for t in grey_tile grey_buf; do
  python3 tools/summarize_pmc_mem.py gpurun_out/r02/pmc_$t --rows 2520 --row-bytes 1920 --steps 8 > gpurun_out/r02/pmc_$t/summary.md
  sed -n 3,6p gpurun_out/r02/pmc_$t/summary.md
done
