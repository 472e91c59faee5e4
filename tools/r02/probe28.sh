#!/usr/bin/env bash
# Round-2 probe 28: the reference's CUDA table as single cold runs on an idle
# GPU after the start-up changes (code-object preload thread, model-picked
# tile shapes in one-shot runs).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe28
mkdir -p "$O"
timeout -k 10 900 python3 -u tools/ref_tables.py cuda --runs 3 --gap 3 --out "$O/cuda_idle.jsonl" > "$O/idle.log" 2>&1
python3 tools/ref_tables.py report "$O/cuda_idle.jsonl" --md "$O/cuda_idle.md" > /dev/null
grep -E "faster in|Median" "$O/cuda_idle.md"
