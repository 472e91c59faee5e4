#!/usr/bin/env bash
# Round-3 call AR: the reference's MPI / MPI+OpenMP tables on the box's CPU
# share after the CPU rows got their AVX2 clones (production policy: unbound
# teams of budget / ranks, passive OpenMP waits).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ar
mkdir -p $O
timeout -k 10 400 python tools/ref_tables.py mpi-cpu --backends omp --channels grey,rgb --sizes 2520,5040 \
  --ranks 1,2,4,9 --runs 3 --out $O/hybrid_omp.jsonl --bind off --wait passive > /dev/null 2> $O/hybrid_omp.err
echo "omp rc=$?"
timeout -k 10 400 python tools/ref_tables.py mpi-cpu --backends cpu --channels grey,rgb --sizes 2520,5040 \
  --ranks 1,2,4,9 --runs 3 --out $O/mpi_cpu.jsonl --bind off --wait passive > /dev/null 2> $O/mpi_cpu.err
echo "cpu rc=$?"
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03/ar/*.jsonl")):
    print(f.split("/")[-1])
    for l in open(f):
        r = json.loads(l)
        print("  ", r.get("backend"), r["channels"], r["height"], r["ranks"], r.get("omp_threads"), round(r["loop_s"], 4))
PY
