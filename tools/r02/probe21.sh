#!/usr/bin/env bash
# Round-2 probe 21: runtime knobs against the one-shot CLI's start-up phases
# (first hardware queue, kernarg pool, code object), single cold processes
# with a 3 s idle gap (probe 19: back-to-back processes wait for the previous
# one's driver teardown).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe21
mkdir -p "$O"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
one() {  # label, env assignments...
  local label=$1; shift
  for i in 1 2 3; do
    sleep 3
    line=$(env "$@" timeout -k 5 60 $CONV x.raw 1920 630 10 grey --synthetic 1 --json --out /tmp/p21.raw 2>/dev/null | tail -n 1)
    echo "{\"label\": \"$label\", \"r\": $line}" >> "$O/knobs.jsonl"
  done
  echo "$label done"
}
one default X_NONE=1
one kernarg_pool_256k HSA_KERNARG_POOL_SIZE=262144
one aql_queue_4k ROC_AQL_QUEUE_SIZE=4096
one host_kernarg HIP_FORCE_DEV_KERNARG=0
one cu_mask_skip HSA_CU_MASK_SKIP_INIT=1
one no_scratch_reclaim HSA_NO_SCRATCH_RECLAIM=1
one no_interrupt HSA_ENABLE_INTERRUPT=0
one sysmem_pool0 DEBUG_CLR_SYSMEM_POOL=0
one queue_devmem0 HSA_ALLOCATE_QUEUE_DEV_MEM=0
python3 - <<'P'
import json, statistics, collections
rows = collections.defaultdict(list)
for l in open("gpurun_out/r02/probe21/knobs.jsonl"):
    d = json.loads(l); rows[d["label"]].append(d["r"])
for k, rs in rows.items():
    ph = collections.defaultdict(list)
    for r in rs:
        for p, v in r["phases_s"].items(): ph[p].append(v * 1e3)
    print(f"{k:20s} e2e {statistics.median(r['e2e_s'] for r in rs) * 1e3:6.1f} ms | " +
          " ".join(f"{p} {statistics.median(v):.1f}" for p, v in ph.items()))
P
