#!/bin/bash
# Round 4, second pass: streamed images issued directly (graph streaming
# dropped), step graphs always starting in frame 0 (no capture inside the
# timed region), fuse 16 for streamed images, a copy+kernel trace of one
# streamed configuration; then the HIP-IPC tests.
set -o pipefail
OUT=gpurun_out/r04/stream_b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_stream.py tests/test_gpu_engine.py -k "stream or rings" > $OUT/pytest_stream.txt 2>&1 || { echo "stream tests failed"; tail -30 $OUT/pytest_stream.txt; exit 1; }
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
run base20a --steps 20 --warmup 5 || exit 1
run base20b --steps 20 --warmup 5 --no-check || exit 1
for c in 2 3 4 6; do
  run d${c}_20 --steps 20 --warmup 5 --stream-chunks $c --no-check || exit 1
  run d${c}f16_20 --steps 20 --warmup 5 --stream-chunks $c --fuse 16 --halo 16 --no-check || exit 1
done
run d4_200 --steps 200 --warmup 30 --stream-chunks 4 --no-check || exit 1
run base200 --steps 200 --warmup 30 --no-check || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_d4 -o run \
  -- python3 bench.py --steps 20 --warmup 5 --stream-chunks 4 --no-check > $OUT/trace_d4.json 2> $OUT/trace_d4.err \
  || { echo "trace failed"; tail -5 $OUT/trace_d4.err; exit 1; }
timeout -k 10 500 $PYT tests/test_gpu_ipc.py > $OUT/pytest_ipc.txt 2>&1 || { echo "ipc tests failed"; tail -40 $OUT/pytest_ipc.txt; exit 1; }
tail -2 $OUT/pytest_ipc.txt
