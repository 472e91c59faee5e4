#!/usr/bin/env bash
# Round-2 probe 47: 2-D copy rates by row width (grey 1920-byte rows vs RGB
# 5760-byte rows), same box.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe47
mkdir -p "$O"
timeout -k 5 120 tools/ubench/copy_bw 2520 20 pinned 1920 2048 > "$O/grey_1920.txt" 2>&1
timeout -k 5 120 tools/ubench/copy_bw 2520 20 pinned 5760 5888 > "$O/rgb_5760.txt" 2>&1
timeout -k 5 120 tools/ubench/copy_bw 315 40 pinned 1920 2048 > "$O/grey_1920_315.txt" 2>&1
for f in grey_1920 rgb_5760 grey_1920_315; do echo "== $f"; tail -n 15 "$O/$f.txt"; done
