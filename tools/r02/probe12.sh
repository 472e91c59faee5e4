#!/usr/bin/env bash
# Round-2 probe 12: taller-wave tile shapes ({4,12|16,4|8}) — bit-exactness
# of every shape, then the all-shape sweep on the BASELINE frames.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe12
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 40 --iters 10 --rounds 2 --shapes all > "$O/rgb1920_all.jsonl" 2> "$O/err.log"
echo rgb1920 ok
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 40 --iters 10 --rounds 2 --channels grey --shapes all > "$O/grey1920_all.jsonl" 2>> "$O/err.log"
echo grey1920 ok
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1 --fuse 8 --reps 24 --iters 2 --rounds 1 --width 32768 --height 32768 --channels grey --shapes "4,8,8;4,12,8;4,16,8;4,12,4;4,16,4;8,4,8;8,8,8" > "$O/grey32768.jsonl" 2>> "$O/err.log"
echo grey32768 ok
PCONV_STREAM=0 timeout -k 10 300 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 8 --reps 24 --iters 3 --rounds 2 --width 8192 --height 8192 --shapes all > "$O/rgb8192_all.jsonl" 2>> "$O/err.log"
echo probe12 done
