#!/usr/bin/env bash
# Round-2 probe 7: row-streaming kernel with 4 / 6 / 8 levels — bit-exactness,
# then us/rep on the BASELINE frames (tile kernel only vs tuned incl. stream vs
# stream forced) at fuse 4 / 6 / 8.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe7
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -k streaming -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
for mode in 0 -1 1; do
  PCONV_STREAM=$mode timeout -k 10 240 python3 -u tools/band_sweep.py --worlds 1 --fuse 4,6,8 --channels grey --width 32768 --height 32768 --reps 24 --iters 2 --rounds 2 --shapes auto >> "$O/grey32768.jsonl" 2> "$O/grey32768_$mode.err"
  echo "32768 grey mode $mode ok"
  PCONV_STREAM=$mode timeout -k 10 240 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 4,6,8 --channels rgb --width 8192 --height 8192 --reps 24 --iters 3 --rounds 2 --shapes auto >> "$O/rgb8192.jsonl" 2> "$O/rgb8192_$mode.err"
  echo "8192 rgb mode $mode ok"
  PCONV_STREAM=$mode timeout -k 10 240 python3 -u tools/band_sweep.py --worlds 1,8 --fuse 4,6,8 --channels rgb --reps 24 --iters 10 --rounds 2 --shapes auto >> "$O/rgb1920.jsonl" 2> "$O/rgb1920_$mode.err"
  echo "1920 rgb mode $mode ok"
done
echo probe7 done
