#!/usr/bin/env bash
# Round-2 probe 51: persistent prefetching tile kernel (k_swar_pf): GPU tests,
# then the sweep against the relaunching tile kernel on the BASELINE frames.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe51
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -k "prefetch or every_swar_shape" -x -q --timeout 150 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
timeout -k 10 300 python3 -u tools/pf_sweep.py --width 32768 --height 32768 --channels grey --fuse 8 --reps 240 --check > "$O/g32768_f8.jsonl" 2> "$O/err.txt"
timeout -k 10 200 python3 -u tools/pf_sweep.py --width 8192 --height 8192 --channels rgb --fuse 8 --reps 200 --iters 4 --check > "$O/rgb8192_f8.jsonl" 2>> "$O/err.txt"
timeout -k 10 200 python3 -u tools/pf_sweep.py --width 1920 --height 2520 --channels rgb --fuse 8 --reps 40 --iters 20 --check > "$O/rgb1920_f8.jsonl" 2>> "$O/err.txt"
timeout -k 10 300 python3 -u tools/pf_sweep.py --width 32768 --height 32768 --channels grey --fuse 12 --reps 240 > "$O/g32768_f12.jsonl" 2>> "$O/err.txt"
python3 -c "
import json
for f in ('g32768_f8', 'rgb8192_f8', 'rgb1920_f8', 'g32768_f12'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, d['config'], d.get('us_per_rep'), d.get('mismatches_vs_first', ''), d.get('error', ''))"
