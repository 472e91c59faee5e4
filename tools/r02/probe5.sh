#!/usr/bin/env bash
# Round-2 probe 5: device timelines of interior || halo (RCCL send/recv to
# self on the comm stream; D2D halo copies between bands), bench copy floor,
# MPI / MPI+OpenMP tables on this box's CPU share (<= 9 ranks: the box allows
# at most 16 processes holding a GPU handle).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe5
mkdir -p "$O"
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/ov_rccl" -o run \
  -- python3 tools/overlap_trace.py run rccl-self > "$O/ov_rccl.log" 2>&1
echo rccl-self traced
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/ov_local" -o run \
  -- python3 tools/overlap_trace.py run local-async --bands 4 --halo 16 > "$O/ov_local.log" 2>&1
echo local-async traced
timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
cut -c1-200 "$O/bench.json"
timeout -k 10 700 python3 -u tools/ref_tables.py mpi-cpu --runs 1 --ranks 1,2,4,9 --out "$O/mpi_cpu.jsonl" > "$O/mpi_cpu.log" 2>&1
echo probe5 done
