#!/bin/bash
# Round 4 (session 2): tail streaming (the last image of a burst held back
# and streamed by drain) — the GPU suite, then the driver's command with
# tail streaming on / off.
set -o pipefail
OUT=gpurun_out/r04/tail
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_stream.txt 2>&1 || { echo "stream tests failed"; tail -40 $OUT/pytest_stream.txt; exit 1; }
tail -1 $OUT/pytest_stream.txt
one() {  # name, tail, -- bench args
  local name=$1 v=$2; shift 2
  PCONV_TAIL_STREAM=$v timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:10s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} mism {d.get('mismatches')}")
PY
}
for i in a b c d; do
  one t1_$i 1 --steps 20 --warmup 5 || exit 1
  one t0_$i 0 --steps 20 --warmup 5 || exit 1
done
one t1_200 1 --steps 200 --warmup 5 || exit 1
one t1_e8 1 --emulate 8:3 --steps 300 --warmup 10 || exit 1
one t1_e8_20 1 --emulate 8:3 --steps 20 --warmup 5 || exit 1
one t0_e8_20 0 --emulate 8:3 --steps 20 --warmup 5 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
