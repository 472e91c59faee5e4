#!/usr/bin/env bash
# Round-2 probe 37: resident kernel without the agent acquire at one
# workgroup per CU (sc1-only hand-off), exactness + loop time A/B.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe37
mkdir -p "$O"
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_resident.py -q -x --timeout 90 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
timeout -k 10 200 python3 -u tools/resident_sweep.py --frames 1920x2520:rgb,1920x2520:grey,1920x630:grey --reps 8,16,40 > "$O/sweep_noacq.jsonl" 2> "$O/sweep.err"
PCONV_RESIDENT_ACQUIRE=1 timeout -k 10 200 python3 -u tools/resident_sweep.py --frames 1920x2520:rgb --reps 8,16,40 --paths resident > "$O/sweep_acq.jsonl" 2>> "$O/sweep.err"
python3 -c "
import json
for f in ('sweep_noacq', 'sweep_acq'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, d['frame'], d['path'], d['reps'], d['ms_per_loop'])"
