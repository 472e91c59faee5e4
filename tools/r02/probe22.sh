#!/usr/bin/env bash
# Round-2 probe 22: ROCr knobs against hsa_init() itself (47-55 ms on an idle
# GPU), fresh processes with a 3 s idle gap.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe22
mkdir -p "$O"
H=tools/ubench/hsa_cost
one() {
  local label=$1; shift
  for i in 1 2 3; do
    sleep 3
    echo "{\"label\": \"$label\", \"r\": $(env "$@" timeout -k 5 60 $H)}" >> "$O/hsa_knobs.jsonl"
  done
}
one default X_NONE=1
one disable_image HSA_DISABLE_IMAGE=1
one tools_noregister HSA_TOOLS_DISABLE_REGISTER=1
one no_pc_sampling HSA_DISABLE_PC_SAMPLING=1
one no_dxg HSA_ENABLE_DXG_DETECTION=0
one no_copy_agents HSA_DISCOVER_COPY_AGENTS=0
one no_sdma HSA_ENABLE_SDMA=0
one all_off HSA_DISABLE_IMAGE=1 HSA_TOOLS_DISABLE_REGISTER=1 HSA_DISABLE_PC_SAMPLING=1 HSA_ENABLE_DXG_DETECTION=0
python3 - <<'P'
import json, statistics, collections
rows = collections.defaultdict(list)
for l in open("gpurun_out/r02/probe22/hsa_knobs.jsonl"):
    d = json.loads(l); rows[d["label"]].append(d["r"])
for k, rs in rows.items():
    print(f"{k:18s} hsa_init " + " ".join(f"{r['hsa_init_ms']:.1f}" for r in rs) +
          " | kfd_open " + " ".join(f"{r['kfd_open_ms']:.1f}" for r in rs) + f" | agents {rs[0]['agents']} status {rs[0]['status']}")
P
