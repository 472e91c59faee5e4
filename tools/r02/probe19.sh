#!/usr/bin/env bash
# Round-2 probe 19: is the 100-200 ms /dev/kfd open of a fresh process the
# previous process's KFD teardown?  Same fresh processes with idle gaps.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe19
mkdir -p "$O"
H=tools/ubench/hsa_cost
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for gap in 0 0.25 0.5 1 2 3; do
  for i in 1 2 3; do
    sleep $gap
    echo "{\"gap_s\": $gap, \"r\": $(timeout -k 5 60 $H)}" >> "$O/hsa_gap.jsonl"
  done
done
wall() {
  local t0 t1 line
  t0=$(date +%s%N)
  line=$(timeout -k 5 60 "$@" --synthetic 1 --json --out /tmp/p19.raw 2>/dev/null | tail -n 1)
  t1=$(date +%s%N)
  echo "{\"wall_ms\": $(( (t1 - t0) / 1000000 )), \"report\": $line}"
}
for gap in 0 3; do
  for i in 1 2 3; do
    sleep $gap
    echo "{\"gap_s\": $gap, \"r\": $(wall $CONV x.raw 1920 630 10 grey)}" >> "$O/conv_gap.jsonl"
  done
done
python3 - <<'P'
import json
O = "gpurun_out/r02/probe19"
for l in open(f"{O}/hsa_gap.jsonl"):
    d = json.loads(l); r = d["r"]
    print("hsa gap", d["gap_s"], "kfd_open", r["kfd_open_ms"], "hsa_init", r["hsa_init_ms"])
for l in open(f"{O}/conv_gap.jsonl"):
    d = json.loads(l); r = d["r"]; rep = r["report"]
    print("conv gap", d["gap_s"], "wall", r["wall_ms"], "since_exec", rep.get("since_exec_s"), "e2e", rep.get("e2e_s"),
          "hip_init", (rep.get("phases_s") or {}).get("hip_init"))
P
