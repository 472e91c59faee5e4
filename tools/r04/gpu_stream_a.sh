#!/bin/bash
# Round 4, first GPU pass: row streaming within one image (tests + headline
# bench without / with streaming, graph and direct forms, several chunk
# counts) and the HIP-IPC cross-process halo tests.  Every GPU step has its
# own time limit; the script stops at the first failure.
set -o pipefail
OUT=gpurun_out/r04/stream_a
mkdir -p $OUT
export PYTHONUNBUFFERED=1
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_stream.py > $OUT/pytest_stream.txt 2>&1 || { echo "stream tests failed"; tail -30 $OUT/pytest_stream.txt; exit 1; }
tail -2 $OUT/pytest_stream.txt
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 150 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:12s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']} mism {d.get('mismatches')}")
PY
}
run base20 --steps 20 --warmup 5 || exit 1
for c in 2 3 4 6 8; do
  run g${c}_20 --steps 20 --warmup 5 --stream-chunks $c --no-check || exit 1
done
for c in 3 4 6; do
  run d${c}_20 --steps 20 --warmup 5 --stream-chunks $c --step-graphs off --no-check || exit 1
done
run base200 --steps 200 --warmup 30 --no-check || exit 1
run g4_200 --steps 200 --warmup 30 --stream-chunks 4 --no-check || exit 1
run d4_200 --steps 200 --warmup 30 --stream-chunks 4 --step-graphs off --no-check || exit 1
timeout -k 10 500 $PYT tests/test_gpu_ipc.py > $OUT/pytest_ipc.txt 2>&1 || { echo "ipc tests failed"; tail -40 $OUT/pytest_ipc.txt; exit 1; }
tail -2 $OUT/pytest_ipc.txt
