#!/bin/bash
# Round 4, third pass: streamed images with every upload issued first and
# one event per chunk; the same with HIP's copies on blit kernels instead of
# SDMA (HSA_ENABLE_SDMA=0) to see what a cross-stream hop costs between two
# compute queues; a trace of one configuration.  Then the 4+-slot script.
set -o pipefail
OUT=gpurun_out/r04/stream_c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_stream.py tests/test_gpu_engine.py -k "stream or rings" > $OUT/pytest_stream.txt 2>&1 || { echo "stream tests failed"; tail -30 $OUT/pytest_stream.txt; exit 1; }
tail -2 $OUT/pytest_stream.txt
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --no-check "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:14s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']}")
PY
}
run base20 X=1 -- --steps 20 --warmup 5 || exit 1
for c in 2 3 4 6 8; do run d${c} X=1 -- --steps 20 --warmup 5 --stream-chunks $c || exit 1; done
run d4_conc X=1 -- --steps 20 --warmup 5 --stream-chunks 4 --concurrent on || exit 1
run base20_nosdma HSA_ENABLE_SDMA=0 -- --steps 20 --warmup 5 || exit 1
run d4_nosdma HSA_ENABLE_SDMA=0 -- --steps 20 --warmup 5 --stream-chunks 4 || exit 1
run d6_nosdma HSA_ENABLE_SDMA=0 -- --steps 20 --warmup 5 --stream-chunks 6 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_d4 -o run \
  -- python3 bench.py --steps 20 --warmup 5 --stream-chunks 4 --no-check > $OUT/trace_d4.json 2> $OUT/trace_d4.err \
  || { echo "trace failed"; tail -5 $OUT/trace_d4.err; exit 1; }
bash tools/r04/gpu_slots.sh
