#!/bin/bash
# Round 4 (session 2): streamed image with each chunk's download issued right
# behind its launches (default now) vs every download after every launch.
set -o pipefail
OUT=gpurun_out/r04/issue
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
one() {  # name, issue, -- bench args
  local name=$1 v=$2; shift 2
  PCONV_STREAM_ISSUE=$v timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:12s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} mism {d.get('mismatches')}")
PY
}
for i in a b c; do
  one late_$i late --steps 20 --warmup 5 || exit 1
  one early_$i early --steps 20 --warmup 5 || exit 1
done
one early_c6 early --steps 20 --warmup 5 --stream-chunks 6 || exit 1
one early_c8 early --steps 20 --warmup 5 --stream-chunks 8 || exit 1
one early_c3 early --steps 20 --warmup 5 --stream-chunks 3 || exit 1
one early_direct4 early --steps 20 --warmup 5 --stream-chunks 4 --step-graphs off || exit 1
G="--width 32768 --height 32768 --channels grey --reps 200 --steps 4 --warmup 2 --loop-steps 1 --no-check"
one g_late late $G || exit 1
one g_early early $G || exit 1
