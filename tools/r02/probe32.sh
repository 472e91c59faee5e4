#!/usr/bin/env bash
# Round-2 probe 32: PCIe copy rates with transparent-huge-page host buffers
# (hipHostRegister) against hipHostMalloc, full frame and the 8-way band.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe32
mkdir -p "$O"
{ cat /sys/kernel/mm/transparent_hugepage/enabled; cat /sys/kernel/mm/transparent_hugepage/defrag; } > "$O/thp.txt" 2>&1 || true
timeout -k 5 120 tools/ubench/copy_bw 2520 20 > "$O/malloc_2520.txt" 2>&1
timeout -k 5 120 tools/ubench/copy_bw 2520 20 thp > "$O/thp_2520.txt" 2>&1
timeout -k 5 120 tools/ubench/copy_bw 395 40 > "$O/malloc_395.txt" 2>&1
timeout -k 5 120 tools/ubench/copy_bw 395 40 thp > "$O/thp_395.txt" 2>&1
cat "$O/thp.txt"
for f in malloc_2520 thp_2520 malloc_395 thp_395; do echo "== $f"; tail -n 12 "$O/$f.txt"; done
