#!/bin/bash
# Round 4 (session 2): wave-kernel timeline (per-task trace) and grid / poll
# sweep; burst stagger of the step-graph pipeline (A/B at 20 and 200 images,
# N=1 and the 8-way per-rank proxy).
set -o pipefail
OUT=gpurun_out/r04/wave2
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
one wave_trace PCONV_WAVE_TRACE=$OUT/trace.jsonl -- --steps 3 --warmup 1 --stream-chunks -1 --loop-steps 1 --no-check || exit 1
python tools/wave_trace.py $OUT/trace.jsonl
for g in 64 128 256 0; do
  for z in 1 4; do
    one wave_g${g}_z$z PCONV_WAVE_GRID=$g PCONV_WAVE_SLEEP=$z -- --steps 5 --warmup 2 --stream-chunks -1 --loop-steps 1 --no-check || exit 1
  done
done
one wave_trace_g128 PCONV_WAVE_GRID=128 PCONV_WAVE_TRACE=$OUT/trace_g128.jsonl -- --steps 3 --warmup 1 --stream-chunks -1 --loop-steps 1 --no-check || exit 1
python tools/wave_trace.py $OUT/trace_g128.jsonl
for i in a b c; do
  one st_on_20$i X=1 -- --steps 20 --warmup 5 || exit 1
  one st_off_20$i PCONV_STAGGER=0 -- --steps 20 --warmup 5 || exit 1
done
one st_on_200 X=1 -- --steps 200 --warmup 30 || exit 1
one st_off_200 PCONV_STAGGER=0 -- --steps 200 --warmup 30 || exit 1
one st_on_h4_20 X=1 -- --steps 20 --warmup 5 --stream-chunks 4 || exit 1
one e8_st_on_20 X=1 -- --emulate 8:3 --steps 20 --warmup 5 || exit 1
one e8_st_off_20 PCONV_STAGGER=0 -- --emulate 8:3 --steps 20 --warmup 5 || exit 1
one e8_st_on_300 X=1 -- --emulate 8:3 --steps 300 --warmup 30 || exit 1
one e8_st_off_300 PCONV_STAGGER=0 -- --emulate 8:3 --steps 300 --warmup 30 || exit 1
