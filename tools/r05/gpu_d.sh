#!/bin/bash
# Round 5, fourth GPU call: the SWAR step forms A/B on the tuned production
# launches; the driver's command with the new queue budget (4 runs); the
# 8-way proxy with 4 vs 8 pool queues; the reference's CUDA table with
# --backend hip back to back and after an idle gap (one-shot CLI phases);
# then the N = 8 rehearsal of the driver's SCALE command.
set -o pipefail
OUT=gpurun_out/r05/d
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/r05/form_ab.py > $OUT/form_ab.jsonl 2> $OUT/form_ab.err || { echo "form A/B failed"; tail -20 $OUT/form_ab.err; exit 1; }
cat $OUT/form_ab.jsonl
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:14s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']} mism {d.get('mismatches')}")
PY
}
for i in 1 2 3 4; do one drv_$i --gpus 1 --steps 20 --warmup 5 || exit 1; done
for i in 1 2; do
  one e8_q8_$i --emulate 8:3 --steps 300 --warmup 10 || exit 1
  one e8_q4_$i --emulate 8:3 --steps 300 --warmup 10 --hw-queues 4 || exit 1
done
T="timeout -k 10 600 python -u tools/ref_tables.py cuda --runs 3 --tmp /tmp/pconv_ref"
$T --out $OUT/cuda_hip.jsonl --extra --backend hip > $OUT/cuda_hip.log 2>&1 || { echo "hip table failed"; tail -5 $OUT/cuda_hip.log; exit 1; }
python tools/ref_tables.py report $OUT/cuda_hip.jsonl --md $OUT/cuda_hip.md > /dev/null && tail -3 $OUT/cuda_hip.md
$T --gap 1.0 --out $OUT/cuda_hip_idle.jsonl --extra --backend hip > $OUT/cuda_hip_idle.log 2>&1 || { echo "hip idle table failed"; tail -5 $OUT/cuda_hip_idle.log; exit 1; }
python tools/ref_tables.py report $OUT/cuda_hip_idle.jsonl --md $OUT/cuda_hip_idle.md > /dev/null && tail -3 $OUT/cuda_hip_idle.md
OUT=gpurun_out/r05/scale8 bash tools/r05/scale8_rehearsal.sh || exit 1
