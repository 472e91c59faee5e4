#!/bin/bash
# Round 4: BASELINE's large frames in steady state:
# 32768^2 grey x 200 and 8192^2 RGB x 100 with 3 / 4 images in flight (slot
# streams on CU-masked queues), one image alone with and without row
# streaming, and a kernel + copy trace of the 32768^2 steady state.
set -o pipefail
OUT=gpurun_out/r04/big
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-check "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:22s} ms/step {d['ms_per_step']:.3f} latency {d['latency_ms']:.3f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']}")
PY
}
G="--width 32768 --height 32768 --channels grey --reps 200"
R="--width 8192 --height 8192 --channels rgb --reps 100"
one g_s3 $G --steps 10 --warmup 4 --slots 3 --loop-steps 3 || exit 1
one g_s4 $G --steps 10 --warmup 4 --slots 4 --loop-steps 3 || exit 1
one g_s4_head4 $G --steps 10 --warmup 4 --slots 4 --stream-chunks 4 --loop-steps 3 || exit 1

one r_s3 $R --steps 20 --warmup 4 --slots 3 --loop-steps 5 || exit 1
one r_s4 $R --steps 20 --warmup 4 --slots 4 --loop-steps 5 || exit 1
one r_s4_head4 $R --steps 20 --warmup 4 --slots 4 --stream-chunks 4 --loop-steps 5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_g_s3 -o run \
  -- python3 bench.py $G --steps 8 --warmup 3 --slots 3 --loop-steps 1 --no-check > $OUT/trace_g_s3.json 2> $OUT/trace_g_s3.err \
  || { echo "trace failed"; tail -5 $OUT/trace_g_s3.err; exit 1; }
d=$(dirname $(find $OUT/trace_g_s3 -name run_kernel_trace.csv | head -1))
python tools/queue_trace_summary.py $d --window 0.5 --json $OUT/trace_g_s3_summary.json | head -12
