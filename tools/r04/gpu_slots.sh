#!/bin/bash
# Round 4: root cause of the 4+-images-in-flight collapse of the 8-way
# per-rank step.  Per-rank proxy (--emulate 8:3) with
# 3..6 slots: default, with the host<->device copies on blit kernels instead
# of SDMA queues (HSA_ENABLE_SDMA=0), and with fewer hardware queues; then a
# kernel + memory-copy trace of 3 and 4 slots (no counters in these runs).
set -o pipefail
OUT=gpurun_out/r04/slots
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --emulate 8:3 --steps 300 --warmup 30 --no-check "$@" \
    > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:22s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']}")
PY
}
for s in 3 4 5 6; do one s${s} X=1 -- --slots $s || exit 1; done
for s in 3 4 6; do one s${s}_nosdma HSA_ENABLE_SDMA=0 -- --slots $s || exit 1; done
for s in 4 6; do one s${s}_q4 X=1 -- --slots $s --hw-queues 4 || exit 1; done
for s in 3 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_s$s -o run \
    -- python3 bench.py --emulate 8:3 --steps 200 --warmup 30 --no-check --slots $s > $OUT/trace_s$s.log 2>&1 \
    || { echo "trace s$s failed"; tail -5 $OUT/trace_s$s.log; exit 1; }
done
for s in 3 4; do
  d=$(dirname $(find $OUT/trace_s$s -name run_kernel_trace.csv | head -1))
  python tools/queue_trace_summary.py $d --json $OUT/trace_s${s}_summary.json | head -20
done
