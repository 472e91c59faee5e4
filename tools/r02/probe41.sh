#!/usr/bin/env bash
# Round-2 probe 41: rocprofv3 kernel + copy trace (csv, --stats) of the
# driver's bench command on the final tree.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe41
mkdir -p "$O"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof" -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/prof_bench.json" 2> "$O/prof.err"
find "$O/prof" -name "*.csv" > "$O/files.txt"
cat "$O/files.txt"
