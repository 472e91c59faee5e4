#!/usr/bin/env bash
# Round-2 probe 30: which runtime buffer is the 16 MB host allocation of the
# first queue (~10 ms): staging / transfer / pinned-transfer size knobs.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe30
mkdir -p "$O"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
one() {
  local label=$1; shift
  for i in 1 2 3; do
    sleep 3
    line=$(env "$@" timeout -k 5 60 $CONV x.raw 1920 630 10 grey --synthetic 1 --json --check --out /tmp/p30.raw 2>/dev/null | tail -n 1)
    echo "{\"label\": \"$label\", \"r\": $line}" >> "$O/knobs.jsonl"
  done
  sleep 3
  env "$@" AMD_LOG_LEVEL=4 timeout -k 5 60 $CONV x.raw 1920 630 10 grey --synthetic 1 --json --out /tmp/p30.raw 2>&1 | grep -E "Allocate hsa (host|device) memory" | cut -c60-200 > "$O/allocs_$label.txt" || true
}
one default X_NONE=1
one staging1 GPU_STAGING_BUFFER_SIZE=1
one xfer1 GPU_XFER_BUFFER_SIZE=1
one pinned_xfer1 GPU_PINNED_XFER_SIZE=1
one resource_cache0 GPU_RESOURCE_CACHE_SIZE=0
python3 - <<'P'
import json, collections
rows = collections.defaultdict(list)
for l in open("gpurun_out/r02/probe30/knobs.jsonl"):
    d = json.loads(l); rows[d["label"]].append(d["r"])
for k, rs in rows.items():
    print(f"{k:16s} queue", [round(r["phases_s"]["queue"] * 1e3, 1) for r in rs], "mism", [r["mismatches"] for r in rs])
P
for f in "$O"/allocs_*.txt; do echo "== $f"; cat "$f"; done
