#!/bin/bash
# Round 4 (session 2): the per-rank 8-way proxy with 3/4 slots in every halo
# mode (preload, RCCL slot exchange, single-dispatch IPC), the N=1 serving
# step at 200 images with 3/4 slots and head streaming, and the same steps on
# the native stack (conv --bench: ROCm 7.2's HIP runtime, no torch).
set -o pipefail
OUT=gpurun_out/r04/e2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --no-check "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:22s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']}", flush=True)
PY
}
E="--emulate 8:3 --steps 300 --warmup 30"
for m in preload slot_exchange ipc; do
  for s in 3 4; do one e8_${m}_s$s X=1 -- $E --emulate-halo $m --slots $s || exit 1; done
done
one e8_ipc3k_s4 PCONV_IPC_KERNELS=3 -- $E --emulate-halo ipc --slots 4 || exit 1
for s in 3 4; do
  one n1_s${s}_200 X=1 -- --steps 200 --warmup 30 --slots $s || exit 1
  one n1_s${s}_h4_200 X=1 -- --steps 200 --warmup 30 --slots $s --stream-chunks 4 || exit 1
done
for s in 3 4; do
  one nat_n1_s${s}_200 X=1 -- --native --steps 200 --warmup 30 --slots $s || exit 1
  one nat_e8_s${s} X=1 -- --native $E --slots $s || exit 1
done
