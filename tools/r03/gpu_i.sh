#!/usr/bin/env bash
# Round-3 call I: hybrid MPI+OpenMP policy A/B on the box's CPU share (binding x wait policy).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/i
mkdir -p $O
run() {  # name, extra args
  timeout -k 10 280 python tools/ref_tables.py mpi-cpu --backends omp --channels grey,rgb --sizes 2520,5040 \
    --ranks 1,2,4,9 --runs 3 --out $O/hybrid_$1.jsonl "${@:2}" > /dev/null 2> $O/hybrid_$1.err
  echo "$1 rc=$?"
}
run bind_spin20k --bind on --spin 20000
run nobind_spin20k --bind off --spin 20000
run bind_passive --bind on --wait passive
run nobind_passive --bind off --wait passive
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03/i/hybrid_*.jsonl")):
    print(f.split("/")[-1])
    for l in open(f):
        r = json.loads(l)
        print("  ", r["channels"], r["height"], r["ranks"], r["omp_threads"], round(r["loop_s"], 4),
              [round(x, 4) for x in r["loop_all_s"]])
PY
