#!/usr/bin/env bash
# Round-2 probe 27: one-shot CLI warm-up run and shape tuning vs end-to-end
# time (single cold processes, idle GPU).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe27
mkdir -p "$O"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for cell in "630 10 grey" "2520 40 rgb" "5040 100 grey"; do
  set -- $cell
  for i in 1 2 3; do
    for mode in "w1_tune 1 -1" "w0_tune 0 -1" "w1_model 1 0" "w0_model 0 0"; do
      set -- $mode
      label=$1; w=$2; t=$3
      set -- $cell
      sleep 3
      if [ "$t" = "0" ]; then export PCONV_AUTOTUNE=0; else unset PCONV_AUTOTUNE; fi
      line=$(timeout -k 5 60 $CONV x.raw 1920 $1 $2 $3 --synthetic 1 --json --warmup $w --out /tmp/p27.raw 2>/dev/null | tail -n 1)
      echo "{\"cell\": \"$cell\", \"mode\": \"$label\", \"r\": $line}" >> "$O/cli_modes.jsonl"
    done
  done
  echo "$cell done"
done
unset PCONV_AUTOTUNE
python3 - <<'P'
import json, statistics, collections
rows = collections.defaultdict(list)
for l in open("gpurun_out/r02/probe27/cli_modes.jsonl"):
    d = json.loads(l); rows[(d["cell"], d["mode"])].append(d["r"])
for (cell, mode), rs in sorted(rows.items()):
    print(f"{cell:14s} {mode:9s} e2e med {statistics.median(r['e2e_s'] for r in rs)*1e3:6.1f} | loop {statistics.median(r['loop_s'] for r in rs)*1e3:.3f} | warmup {statistics.median(r['phases_s'].get('warmup', 0) for r in rs)*1e3:.2f} | post-init {statistics.median(r['e2e_s'] - r['phases_s']['hip_init'] for r in rs)*1e3:.1f}")
P
