#!/usr/bin/env bash
# Round-3 call AS: the hybrid table's smallest image (1920x1260) after the CPU
# vectorisation (n=2 and n=4 faster than n=1 for every
# image >= 1920x1260).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/as
mkdir -p $O
timeout -k 10 300 python tools/ref_tables.py mpi-cpu --backends omp --channels grey,rgb --sizes 1260 \
  --ranks 1,2,4,9 --runs 5 --out $O/hybrid_omp_1260.jsonl --bind off --wait passive > /dev/null 2> $O/err.txt
echo "rc=$?"
python - <<'PY'
import json
for l in open("gpurun_out/r03/as/hybrid_omp_1260.jsonl"):
    r = json.loads(l); print(r["channels"], r["height"], r["ranks"], r.get("omp_threads"), round(r["loop_s"], 4), [round(x, 4) for x in r["loop_all_s"]])
PY
