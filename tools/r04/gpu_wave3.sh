#!/bin/bash
# Round 4 (session 2): wave kernel with the flattened 8-deep copy loop: tests,
# timeline, and a sweep of load parts x load lead x grid.
set -o pipefail
OUT=gpurun_out/r04/wave3
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
for p in 2 4 8; do
  for l in 2 8 16; do
    for g in 256 0; do
      one w_p${p}_l${l}_g$g PCONV_WAVE_PARTS=$p PCONV_WAVE_LEAD=$l PCONV_WAVE_GRID=$g -- $W || exit 1
    done
  done
done
one trace_p8_l8 PCONV_WAVE_PARTS=8 PCONV_WAVE_LEAD=8 PCONV_WAVE_TRACE=$OUT/trace_p8_l8.jsonl -- $W || exit 1
python tools/wave_trace.py $OUT/trace_p8_l8.jsonl
one head_sdma4 X=1 -- --steps 5 --warmup 2 --stream-chunks 4 --loop-steps 1 --no-check || exit 1
one base X=1 -- --steps 5 --warmup 2 --loop-steps 1 --no-check || exit 1
