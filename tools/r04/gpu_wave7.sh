#!/bin/bash
# Round 4 (session 2): wave kernel with dynamic ready-task claiming (default)
# vs the ordered ticket queue: tests (both), latency, timeline.
set -o pipefail
OUT=gpurun_out/r04/wave7
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_wave.txt 2>&1 || { echo "wave tests failed"; tail -40 $OUT/pytest_wave.txt; exit 1; }
tail -1 $OUT/pytest_wave.txt
PCONV_WAVE_DYN=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_wave_ordered.txt 2>&1 || { echo "wave tests (ordered) failed"; tail -40 $OUT/pytest_wave_ordered.txt; exit 1; }
tail -1 $OUT/pytest_wave_ordered.txt
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
for l in 32 64; do
  for z in 1 2; do
    one dyn_l${l}_z$z PCONV_WAVE_LOADERS=$l PCONV_WAVE_SLEEP=$z -- $W || exit 1
  done
done
one ordered PCONV_WAVE_DYN=0 PCONV_WAVE_GAP=8 -- $W || exit 1
one trace_dyn PCONV_WAVE_TRACE=$OUT/trace_dyn.jsonl -- $W || exit 1
python tools/wave_trace.py $OUT/trace_dyn.jsonl
one dyn_check X=1 -- --steps 20 --warmup 5 --stream-chunks -1 || exit 1
one head_sdma4 X=1 -- --steps 5 --warmup 2 --stream-chunks 4 --loop-steps 1 --no-check || exit 1
