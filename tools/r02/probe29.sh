#!/usr/bin/env bash
# Round-2 probe 29: what the first hardware queue's ~20 ms holds (runtime
# log timestamps) and whether the blit-engine setting moves it.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe29
mkdir -p "$O"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for v in default 0 1 2; do
  for i in 1 2 3; do
    sleep 3
    if [ "$v" = default ]; then unset GPU_BLIT_ENGINE_TYPE; else export GPU_BLIT_ENGINE_TYPE=$v; fi
    line=$(timeout -k 5 60 $CONV x.raw 1920 630 10 grey --synthetic 1 --json --check --out /tmp/p29.raw 2>/dev/null | tail -n 1)
    echo "{\"blit\": \"$v\", \"r\": $line}" >> "$O/blit.jsonl"
  done
done
unset GPU_BLIT_ENGINE_TYPE
sleep 3
AMD_LOG_LEVEL=4 timeout -k 5 60 $CONV x.raw 1920 630 10 grey --synthetic 1 --json --out /tmp/p29.raw > "$O/log4.txt" 2>&1
python3 - <<'P'
import json, statistics, collections
rows = collections.defaultdict(list)
for l in open("gpurun_out/r02/probe29/blit.jsonl"):
    d = json.loads(l); rows[d["blit"]].append(d["r"])
for k, rs in rows.items():
    print(k, "queue", [round(r["phases_s"]["queue"] * 1e3, 1) for r in rs], "hip_init", [round(r["phases_s"]["hip_init"] * 1e3, 1) for r in rs], "mism", [r["mismatches"] for r in rs])
P
grep -n "hipStreamCreate\|Created SWq\|Allocate hsa\|acquireQueue\|ShaderName\|Loading\|blit\|Blit" "$O/log4.txt" | cut -c1-220 | sed -n 1,30p
