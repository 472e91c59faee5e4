#!/usr/bin/env bash
# Round-2 probe 64: buffer-op tile kernel with masked first-tile loads and
# last-tile stores (out-of-range offsets only while a next tile is in
# flight): kernel tests, grey / RGB headline sweeps, 8192^2 RGB, the driver's
# bench command.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe64
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -k "prefetch or every_swar_shape" -x -q --timeout 150 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
for spec in "1920 2520 grey 40 20" "1920 2520 rgb 40 20" "8192 8192 rgb 200 4"; do
  set -- $spec
  timeout -k 10 300 python3 -u tools/pf_sweep.py --width $1 --height $2 --channels $3 --fuse 8 --reps $4 --iters $5 --check > "$O/${3}$1.jsonl" 2>> "$O/err.txt"
done
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 -c "
import json
for f in ('grey1920', 'rgb1920', 'rgb8192'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l)
        if d['config'].startswith(('tuned', 'buf_4_8_8', 'tile_4_8_8', 'buf_4_12_8_alt1', 'tile_4_12_8_alt1')): print(f, d['config'], d.get('us_per_rep'), d.get('mismatches_vs_first', ''))
d = json.load(open('$O/bench.json')); print('bench', d['ms_per_step'], d['loop_only'], d['latency_ms'])"
