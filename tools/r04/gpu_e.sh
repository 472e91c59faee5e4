#!/bin/bash
# Round 4: single-dispatch IPC exchange (tests + 8-way proxy), CU-masked slot
# streams by default (3/4/5 slots, N=1 and the 8-way proxy), a trace of the
# 4-slot CU-masked pipeline.
set -o pipefail
OUT=gpurun_out/r04/e
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_ipc.py > $OUT/pytest_ipc.txt 2>&1 || { echo "ipc tests failed"; tail -40 $OUT/pytest_ipc.txt; exit 1; }
tail -2 $OUT/pytest_ipc.txt
timeout -k 10 500 $PYT tests/test_gpu_stream.py tests/test_gpu_engine.py -k "stream or rings or multi_rank" > $OUT/pytest_stream.txt 2>&1 || { echo "stream tests failed"; tail -40 $OUT/pytest_stream.txt; exit 1; }
tail -2 $OUT/pytest_stream.txt
one() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --no-check "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:22s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']}")
PY
}
E="--emulate 8:3 --steps 300 --warmup 30"
for s in 3 4 5; do one s$s X=1 -- $E --slots $s || exit 1; done
for m in preload slot_exchange ipc; do
  for s in 3 4; do one e8_${m}_s$s X=1 -- --emulate 8:3 --emulate-halo $m --steps 300 --warmup 30 --slots $s || exit 1; done
done
one e8_ipc3k_s4 PCONV_IPC_KERNELS=3 -- --emulate 8:3 --emulate-halo ipc --steps 300 --warmup 30 --slots 4 || exit 1
for s in 3 4; do
  one n1_s${s}_20a X=1 -- --steps 20 --warmup 5 --slots $s || exit 1
  one n1_s${s}_20b X=1 -- --steps 20 --warmup 5 --slots $s || exit 1
  one n1_s${s}_200 X=1 -- --steps 200 --warmup 30 --slots $s || exit 1
done
one n1_s4_plain_200 PCONV_SLOT_STREAMS=plain -- --steps 200 --warmup 30 --slots 4 || exit 1
for s in 3 4; do
  for c in 2 4; do
    one n1_s${s}_head${c}_20a X=1 -- --steps 20 --warmup 5 --slots $s --stream-chunks $c || exit 1
    one n1_s${s}_head${c}_20b X=1 -- --steps 20 --warmup 5 --slots $s --stream-chunks $c || exit 1
  done
done
one n1_s4_head4_200 X=1 -- --steps 200 --warmup 30 --slots 4 --stream-chunks 4 || exit 1
one e8_s4_head2 X=1 -- $E --slots 4 --stream-chunks 2 || exit 1
# the same steps on the native stack (conv --bench: ROCm's HIP runtime, no torch)
for s in 3 4; do
  one nat_n1_s${s}_200 X=1 -- --native --steps 200 --warmup 30 --slots $s || exit 1
  one nat_e8_s${s} X=1 -- --native $E --slots $s || exit 1
done
PCONV_SLOT_STREAMS=cumask timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_s4 -o run \
  -- python3 bench.py $E --slots 4 --no-check > $OUT/trace_s4.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace_s4.log; exit 1; }
d=$(dirname $(find $OUT/trace_s4 -name run_kernel_trace.csv | head -1))
python tools/queue_trace_summary.py $d --json $OUT/trace_s4_summary.json | head -12
