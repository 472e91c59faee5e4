#!/usr/bin/env bash
# Round-2 probe 34: D2H as a hipGraph memcpy node, contiguous vs pitched.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe34
mkdir -p "$O"
timeout -k 5 120 tools/ubench/copy_bw 2520 20 > "$O/copy_bw_2520.txt" 2>&1
timeout -k 5 120 tools/ubench/copy_bw 315 40 > "$O/copy_bw_315.txt" 2>&1
for f in 2520 315; do echo "== $f"; tail -n 15 "$O/copy_bw_$f.txt"; done
