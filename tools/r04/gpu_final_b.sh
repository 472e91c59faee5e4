#!/bin/bash
# Round 4 (session 2): 3 vs 4 images in flight in the driver's 20-image
# window (N=1 and the 8-way proxy, 3 runs each); BASELINE large frames over a
# longer window (the 10-image window is mostly pipeline fill and drain);
# stage timelines of 3 vs 4 slots without a profiler.
set -o pipefail
OUT=gpurun_out/r04/final_b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 200 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:22s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']} mism {d.get('mismatches')}", flush=True)
PY
}
for i in a b c; do
  for s in 3 4; do
    one n1_s${s}_20$i X=1 -- --steps 20 --warmup 5 --slots $s || exit 1
  done
done
for i in a b; do
  for s in 3 4; do
    one e8_s${s}_20$i X=1 -- --emulate 8:3 --steps 20 --warmup 5 --slots $s || exit 1
  done
done
G="--width 32768 --height 32768 --channels grey --reps 200 --no-check"
R="--width 8192 --height 8192 --channels rgb --reps 100 --no-check"
one g_s3_40 X=1 -- $G --steps 40 --warmup 4 --slots 3 --loop-steps 3 || exit 1
one g_s4_40 X=1 -- $G --steps 40 --warmup 4 --slots 4 --loop-steps 3 || exit 1
one r_s3_100 X=1 -- $R --steps 100 --warmup 6 --slots 3 --loop-steps 5 || exit 1
one r_s4_100 X=1 -- $R --steps 100 --warmup 6 --slots 4 --loop-steps 5 || exit 1
bash tools/r04/gpu_slots_c.sh || exit 1
