#!/usr/bin/env bash
# Round-2 probe 16: split-D2H pipeline — correctness, then the per-rank step
# at N = 8 / 4 / 2 / 1 (--emulate) against the slot pipeline.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe16
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py -q -k "split_d2h or step_graphs" --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 120 python3 -u bench.py "$@" > "$O/$name.json" 2> "$O/$name.err"
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['ms_per_step'], d['config'].get('split_d2h'), d['config']['images_in_flight'], d['copy_floor']['floor_ms'])"
}
for emu in 8:3 8:0 4:1 2:0; do
  e=${emu/:/_}
  run "e${e}_slots3" --emulate $emu --steps 300 --warmup 30
  run "e${e}_split4" --emulate $emu --steps 300 --warmup 30 --pipeline split
  run "e${e}_split2" --emulate $emu --steps 300 --warmup 30 --pipeline split --slots 2
  run "e${e}_split6" --emulate $emu --steps 300 --warmup 30 --pipeline split --slots 6
done
run n1_slots3 --steps 20 --warmup 5
run n1_split4 --steps 20 --warmup 5 --pipeline split
run n1_slots3b --steps 200 --warmup 20
run n1_split4b --steps 200 --warmup 20 --pipeline split
echo probe16 done
