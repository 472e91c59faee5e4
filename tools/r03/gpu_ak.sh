#!/usr/bin/env bash
# Round-3 call AK: images in flight for the large BASELINE frames (the 4-slot
# collapse was measured on small launches; 1 GB frames keep every launch
# large).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ak
mkdir -p $O
run() {  # name secs args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], 'lat', d['latency_ms'], 'loop', d['loop_only']['ms_per_step'])"
}
G="--width 32768 --height 32768 --channels grey --reps 200"
R="--width 8192 --height 8192 --reps 100"
for s in 3 4 5; do run g_s$s 240 $G --steps 12 --warmup 3 --slots $s; done
for s in 3 4; do run e8g_s$s 150 --emulate 8:3 $G --steps 24 --warmup 4 --slots $s; done
for s in 3 4; do run r_s$s 150 $R --steps 40 --warmup 6 --slots $s; done
echo "call ak done"
