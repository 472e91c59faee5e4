#!/usr/bin/env bash
# Round-2 probe 26: code object loaded on a helper thread during the first
# queue creation (PCONV_PRELOAD A/B), single cold processes on an idle GPU.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe26
mkdir -p "$O"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for i in 1 2 3 4 5; do
  for mode in 1 0; do
    sleep 3
    line=$(PCONV_PRELOAD=$mode timeout -k 5 60 $CONV x.raw 1920 630 10 grey --synthetic 1 --json --check --out /tmp/p26.raw 2>/dev/null | tail -n 1)
    echo "{\"preload\": $mode, \"r\": $line}" >> "$O/preload_ab.jsonl"
  done
done
python3 - <<'P'
import json, statistics, collections
rows = collections.defaultdict(list)
for l in open("gpurun_out/r02/probe26/preload_ab.jsonl"):
    d = json.loads(l); rows[d["preload"]].append(d["r"])
for k, rs in sorted(rows.items()):
    ph = collections.defaultdict(list)
    for r in rs:
        for p, v in r["phases_s"].items(): ph[p].append(v * 1e3)
    print(f"preload={k} e2e " + " ".join(f"{r['e2e_s']*1e3:.1f}" for r in rs) + " | mism " + str([r['mismatches'] for r in rs]) + " | " +
          " ".join(f"{p} {statistics.median(v):.1f}" for p, v in ph.items()))
P
