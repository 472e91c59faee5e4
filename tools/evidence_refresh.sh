#!/usr/bin/env bash
# Evidence refresh for the current tree (GPU box, repo root): headline bench,
# the per-rank emulations of N=2/4/8, a rocprofv3 kernel+copy trace of the
# headline bench and the BASELINE.json configurations.  Each GPU step has its
# own time limit; the script stops at the first failure.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/refresh
mkdir -p "$O"
b() { local name=$1; shift; timeout -k 10 120 python3 -u bench.py "$@" > "$O/$name.json" 2> "$O/$name.err"; echo "$name: $(cut -c1-200 "$O/$name.json")"; }
b bench_n1
b emu_2_0 --emulate 2:0
b emu_4_1 --emulate 4:1
b emu_8_0 --emulate 8:0
b emu_8_3 --emulate 8:3
b emu_8_3_rccl --emulate 8:3 --emulate-rccl
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trace_bench" -o run \
  -- python3 bench.py --steps 50 --warmup 10 > "$O/trace_bench.log" 2>&1
echo "trace done"
timeout -k 10 900 tools/baseline_configs.sh > "$O/baseline.log" 2>&1
echo "refresh done"
