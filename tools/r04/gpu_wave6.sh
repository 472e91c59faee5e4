#!/bin/bash
# Round 4 (session 2): wave kernel with write-through (sc1) hand-offs vs
# plain stores + release; level gap.
set -o pipefail
OUT=gpurun_out/r04/wave6
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_wave.txt 2>&1 || { echo "wave tests failed"; tail -40 $OUT/pytest_wave.txt; exit 1; }
tail -1 $OUT/pytest_wave.txt
PCONV_WAVE_WT=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_wave_plain.txt 2>&1 || { echo "wave tests (plain stores) failed"; tail -40 $OUT/pytest_wave_plain.txt; exit 1; }
tail -1 $OUT/pytest_wave_plain.txt
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
for wt in 1 0; do
  for gap in 1 8 32; do
    one w_wt${wt}_gap$gap PCONV_WAVE_WT=$wt PCONV_WAVE_GAP=$gap -- $W || exit 1
  done
done
one trace_wt1_gap8 PCONV_WAVE_GAP=8 PCONV_WAVE_TRACE=$OUT/trace_wt1_gap8.jsonl -- $W || exit 1
python tools/wave_trace.py $OUT/trace_wt1_gap8.jsonl
one wave_check X=1 -- --steps 20 --warmup 5 --stream-chunks -1 || exit 1
