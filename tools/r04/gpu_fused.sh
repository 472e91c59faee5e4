#!/bin/bash
# Round 4 (session 2): the streamed image with its final level storing straight
# into pinned host memory (PCONV_STREAM_FUSED_D2H=1: no download copies, no
# launch -> D2H hop) against the download copies: GPU tests, one-image
# latency and the driver's command, and one large image alone.
set -o pipefail
OUT=gpurun_out/r04/fused
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_stream.txt 2>&1 || { echo "stream tests failed"; tail -40 $OUT/pytest_stream.txt; exit 1; }
tail -1 $OUT/pytest_stream.txt
one() {  # name, fused, -- bench args
  local name=$1 f=$2; shift 2
  PCONV_STREAM_FUSED_D2H=$f timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:14s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} mism {d.get('mismatches')}")
PY
}
for i in a b; do
  one d20_c0_$i 0 --steps 20 --warmup 5 || exit 1
  one d20_c4f0_$i 0 --steps 20 --warmup 5 --stream-chunks 4 || exit 1
  one d20_c4f1_$i 1 --steps 20 --warmup 5 --stream-chunks 4 || exit 1
done
one d20_c8f1 1 --steps 20 --warmup 5 --stream-chunks 8 || exit 1
one d20_c2f1 1 --steps 20 --warmup 5 --stream-chunks 2 || exit 1
one s200_c0 0 --steps 200 --warmup 5 --no-check || exit 1
one s200_c4f1 1 --steps 200 --warmup 5 --no-check --stream-chunks 4 || exit 1
G="--width 32768 --height 32768 --channels grey --reps 200 --steps 4 --warmup 2 --loop-steps 1 --no-check --stream-chunks 4"
one g_f0 0 $G || exit 1
one g_f1 1 $G || exit 1
R="--width 8192 --height 8192 --channels rgb --reps 100 --steps 10 --warmup 3 --loop-steps 2 --no-check --stream-chunks 4"
one r_f0 0 $R || exit 1
one r_f1 1 $R || exit 1
