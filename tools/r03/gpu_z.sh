#!/usr/bin/env bash
# Round-3 call Z: large BASELINE frames in steady state.  The round-3 baseline
# script timed 32768^2 grey x 200 with 3 steps and 2 images in flight, which
# is dominated by pipeline fill (one image alone: ~63 ms).  Here: 2 / 3 slots
# and 10 timed steps, N=1 and the 8-way per-rank proxy; 8192^2 RGB x 100 with
# 30 steps.  One JSON line per run; stops at the first failure.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/z
mkdir -p $O
run() {  # name secs args...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'lat', d['latency_ms'], 'loop', d['loop_only']['ms_per_step'], 'floor', d['copy_floor'])"
}
G="--width 32768 --height 32768 --channels grey --reps 200"
R="--width 8192 --height 8192 --reps 100"
run g1_s2 200 $G --steps 10 --warmup 2 --slots 2
run g1_s3 200 $G --steps 10 --warmup 2 --slots 3
run e8g_s2 150 --emulate 8:3 $G --steps 20 --warmup 3 --slots 2
run e8g_s3 150 --emulate 8:3 $G --steps 20 --warmup 3 --slots 3
run r1_s3 150 $R --steps 30 --warmup 5 --slots 3
run e8r_s3 150 --emulate 8:3 $R --steps 60 --warmup 10 --slots 3
echo "call z done"
