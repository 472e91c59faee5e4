#!/bin/bash
# Round 4 (session 2): wave kernel with dedicated loader / storer workgroups:
# tests, timeline, sweep of loaders x storers x parts.
set -o pipefail
OUT=gpurun_out/r04/wave4
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_wave.txt 2>&1 || { echo "wave tests failed"; tail -40 $OUT/pytest_wave.txt; exit 1; }
tail -1 $OUT/pytest_wave.txt
one() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 150 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:22s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} mism {d.get('mismatches')}", flush=True)
PY
}
W="--steps 5 --warmup 2 --stream-chunks -1 --loop-steps 1 --no-check"
one trace_default PCONV_WAVE_TRACE=$OUT/trace_default.jsonl -- $W || exit 1
python tools/wave_trace.py $OUT/trace_default.jsonl
for l in 16 32 64; do
  for st in 16 32; do
    for p in 2 4; do
      one w_l${l}_s${st}_p$p PCONV_WAVE_LOADERS=$l PCONV_WAVE_STORERS=$st PCONV_WAVE_PARTS=$p -- $W || exit 1
    done
  done
done
one trace_l64_s32 PCONV_WAVE_LOADERS=64 PCONV_WAVE_STORERS=32 PCONV_WAVE_TRACE=$OUT/trace_l64_s32.jsonl -- $W || exit 1
python tools/wave_trace.py $OUT/trace_l64_s32.jsonl
one head_sdma4 X=1 -- --steps 5 --warmup 2 --stream-chunks 4 --loop-steps 1 --no-check || exit 1
one wave_check X=1 -- --steps 20 --warmup 5 --stream-chunks -1 || exit 1
