#!/bin/bash
# Round 5, third GPU call: the driver's 20-image window spreads 0.339-0.441
# ms between identical runs (profiles/r05/b); A/B of the hardware-queue pool
# size (bench.py sets GPU_MAX_HW_QUEUES=8; the CU-masked slot streams have
# their own queues) over 6 interleaved runs each; then the 8-way RCCL
# slot-exchange proxy, the teardown probe and the SQ counters.
set -o pipefail
OUT=gpurun_out/r05/c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:14s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']} mism {d.get('mismatches')}")
PY
}
for i in 1 2 3 4 5 6; do
  one q8_$i --gpus 1 --steps 20 --warmup 5 || exit 1
  one q4_$i --gpus 1 --steps 20 --warmup 5 --hw-queues 4 || exit 1
done
one e8_rccl --emulate 8:3 --emulate-halo slot_exchange --steps 300 --warmup 10 || exit 1
one e8_ipc_grid --emulate 8:3 --emulate-halo ipc --steps 300 --warmup 10 || exit 1
bash tools/r05/teardown.sh > $OUT/teardown.txt 2>&1 || { echo "teardown probe failed"; tail -5 $OUT/teardown.txt; exit 1; }
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05/teardown/next.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    by[r["prev"]].append(r["next"]["hip_init_ms"])
for k, v in by.items():
    v.sort()
    print(f"prev={k:9s} next hip_init ms median {v[len(v)//2]:7.1f} all {v}")
PY
O=gpurun_out/r05/pmc bash tools/r05/gpu_pmc.sh || exit 1
