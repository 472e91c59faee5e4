#!/usr/bin/env bash
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe15
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 24 --iters 2 --rounds 2 --width 32768 --height 32768 --channels grey --shapes "4,16,8;4,20,8;4,16,16" > "$O/grey32768_tall.jsonl" 2> "$O/err.log"
for i in 1 2; do
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 24 --iters 2 --rounds 2 --width 32768 --height 32768 --channels grey --shapes auto >> "$O/grey32768_auto.jsonl" 2>> "$O/err.log"
done
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 40 --iters 10 --rounds 2 --shapes auto > "$O/rgb1920_auto.jsonl" 2>> "$O/err.log"
timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 40 --iters 10 --rounds 2 --channels grey --shapes auto > "$O/grey1920_auto.jsonl" 2>> "$O/err.log"
cat "$O"/*.jsonl | cut -c1-250
