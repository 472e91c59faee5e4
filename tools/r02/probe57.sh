#!/usr/bin/env bash
# Round-2 probe 57: buffer-op tile kernel without the dead next-tile fetch in
# the one-workgroup-per-tile form: kernel tests, headline / 8192^2 RGB sweep,
# the driver's bench command.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe57
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -k "prefetch or every_swar_shape" -x -q --timeout 150 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
timeout -k 10 300 python3 -u tools/pf_sweep.py --width 1920 --height 2520 --channels rgb --fuse 8 --reps 40 --iters 20 --check > "$O/rgb1920_f8.jsonl" 2> "$O/err.txt"
timeout -k 10 300 python3 -u tools/pf_sweep.py --width 8192 --height 8192 --channels rgb --fuse 8 --reps 200 --iters 4 --check > "$O/rgb8192_f8.jsonl" 2>> "$O/err.txt"
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 -c "
import json
for f in ('rgb1920_f8', 'rgb8192_f8'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l)
        if d['config'].startswith(('tuned', 'buf_4_8_8', 'tile_4_8_8', 'buf_4_12_8', 'tile_4_12_8')): print(f, d['config'], d.get('us_per_rep'), d.get('mismatches_vs_first', ''))
d = json.load(open('$O/bench.json')); print('bench', d['ms_per_step'], d['loop_only'], d['latency_ms'], d['copy_floor'])"
