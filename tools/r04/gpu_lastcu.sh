#!/bin/bash
# Round 4 (session 2): the streamed image's last chunk downloaded by a CU copy
# on the compute stream (PCONV_STREAM_LAST_CU=1) vs SDMA behind a hop.
set -o pipefail
OUT=gpurun_out/r04/lastcu
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
one() {  # name, last_cu, -- bench args
  local name=$1 v=$2; shift 2
  PCONV_STREAM_LAST_CU=$v timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:12s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} mism {d.get('mismatches')}")
PY
}
for i in a b c; do
  one l0_$i 0 --steps 20 --warmup 5 || exit 1
  one l1_$i 1 --steps 20 --warmup 5 || exit 1
done
one l1_c6 1 --steps 20 --warmup 5 --stream-chunks 6 || exit 1
one l1_c3 1 --steps 20 --warmup 5 --stream-chunks 3 || exit 1
