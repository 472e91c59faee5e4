#!/usr/bin/env bash
# Round-2 probe 53: buffer-op tile kernel as a tuned candidate: GPU kernel
# tests, the tuned choice per BASELINE frame, the driver's bench command.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe53
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q --timeout 150 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
timeout -k 10 300 python3 -u tools/pf_sweep.py --width 1920 --height 2520 --channels rgb --fuse 8 --reps 40 --iters 20 --check > "$O/rgb1920_f8.jsonl" 2> "$O/err.txt"
timeout -k 10 300 python3 -u tools/pf_sweep.py --width 1920 --height 2520 --channels grey --fuse 8 --reps 40 --iters 20 --check > "$O/grey1920_f8.jsonl" 2>> "$O/err.txt"
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --emulate 8:3 > "$O/bench_emul8.json" 2>> "$O/bench.err"
python3 -c "
import json
for f in ('rgb1920_f8', 'grey1920_f8'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l)
        if d['config'].startswith(('tuned', 'buf_4_8_8', 'tile_4_8_8')): print(f, d['config'], d.get('us_per_rep'), d.get('mismatches_vs_first', ''), d.get('tuned'))
for f in ('bench', 'bench_emul8'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['ms_per_step'], d['loop_only'], d['latency_ms'])"
