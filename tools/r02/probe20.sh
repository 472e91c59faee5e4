#!/usr/bin/env bash
# Round-2 probe 20: the reference's CUDA table with the current CLI (kernel
# copies), back to back and as single cold runs on an idle GPU (3 s gap).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe20
mkdir -p "$O"
timeout -k 10 200 python3 -u tools/ref_tables.py cuda --runs 3 --out "$O/cuda_b2b.jsonl" > "$O/b2b.log" 2>&1
tail -n 1 "$O/b2b.log"
timeout -k 10 800 python3 -u tools/ref_tables.py cuda --runs 3 --gap 3 --out "$O/cuda_idle.jsonl" > "$O/idle.log" 2>&1
python3 tools/ref_tables.py report "$O/cuda_b2b.jsonl" "$O/cuda_idle.jsonl" --md "$O/cuda_tables.md" > /dev/null
grep -E "faster in|Median" "$O/cuda_tables.md"
