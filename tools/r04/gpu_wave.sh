#!/bin/bash
# Round 4 (session 2): wave images (one persistent launch per serving step,
# kernels/stencil_wave.hip): GPU tests, single-image latency and throughput
# at the headline config, a kernel trace of the wave launch.
set -o pipefail
OUT=gpurun_out/r04/wave
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wave.py -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_wave.txt 2>&1 || { echo "wave tests failed"; tail -60 $OUT/pytest_wave.txt; exit 1; }
tail -3 $OUT/pytest_wave.txt
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
one base20 X=1 -- --steps 20 --warmup 5 || exit 1
one wave20a X=1 -- --steps 20 --warmup 5 --stream-chunks -1 || exit 1
one wave20b X=1 -- --steps 20 --warmup 5 --stream-chunks -1 || exit 1
one wave200 X=1 -- --steps 200 --warmup 30 --stream-chunks -1 || exit 1
one waveall20 PCONV_WAVE_ALL=1 -- --steps 20 --warmup 5 --stream-chunks -1 || exit 1
one waveall200 PCONV_WAVE_ALL=1 -- --steps 200 --warmup 30 --stream-chunks -1 || exit 1
one waveall200_s1 PCONV_WAVE_ALL=1 -- --steps 100 --warmup 10 --stream-chunks -1 --slots 1 || exit 1
one plain20 PCONV_SLOT_STREAMS=plain -- --steps 20 --warmup 5 || exit 1
one plain200 PCONV_SLOT_STREAMS=plain -- --steps 200 --warmup 30 || exit 1
one base200 X=1 -- --steps 200 --warmup 30 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_wave -o run \
  -- python3 bench.py --steps 20 --warmup 5 --stream-chunks -1 --no-check > $OUT/trace_wave.log 2>&1 \
  || { echo "trace failed"; tail -5 $OUT/trace_wave.log; exit 1; }
f=$(find $OUT/trace_wave -name run_kernel_trace.csv | head -1)
python - "$f" <<'PY'
import csv, sys, statistics
rows = list(csv.DictReader(open(sys.argv[1])))
w = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_wave" in r["Kernel_Name"]]
print(f"k_wave dispatches {len(w)}: median {statistics.median(w):.1f} us, min {min(w):.1f}, max {max(w):.1f}" if w else "no k_wave")
PY
