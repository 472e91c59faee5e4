#!/bin/bash
# Round 5, sixth GPU call: the whole GPU suite and smoke on the tree with the
# 8 MiB head-streaming threshold and step form 2 removed; the driver's
# command; per-rank proxies of the 2-, 4- and 8-way splits (the first timed
# image no longer head-streamed below 8 MiB).
set -o pipefail
OUT=gpurun_out/r05/f
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -1 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.txt | head -30; [ $rc -eq 1 ] || exit 1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:14s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']} mism {d.get('mismatches')}")
PY
}
one drv_1 --gpus 1 --steps 20 --warmup 5 || exit 1
one drv_2 --gpus 1 --steps 20 --warmup 5 || exit 1
for e in 2:0 4:1 8:3; do
  n=${e%%:*}
  one e${n}_s20 --emulate $e --steps 20 --warmup 5 || exit 1
  one e${n}_s20_head --emulate $e --steps 20 --warmup 5 --stream-min-mb 0 || exit 1
done
