#!/usr/bin/env bash
# Round-2 probe 2: new halo/overlap tests, the CUDA-table e2e sweep with the
# phase breakdown, the MPI-table 1-GPU loop sweep, memory counters.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe2
mkdir -p "$O"
rc=0
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_halo.py -v --timeout 120 --timeout-method thread > "$O/pytest_halo.log" 2>&1 || rc=$?
tail -n 8 "$O/pytest_halo.log"
# test failures (rc 1) are read afterwards; anything else (timeout, abort, crash) ends the call
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
timeout -k 10 300 python3 -u tools/ref_tables.py cuda --out "$O/cuda.jsonl" > "$O/cuda.log" 2>&1
echo cuda table ok
timeout -k 10 120 python3 -u tools/ref_tables.py mpi-gpu --out "$O/mpi_gpu.jsonl" > "$O/mpi_gpu.log" 2>&1
echo mpi-gpu ok
tools/r02/pmc_mem.sh head 1920 2520 rgb 40 8 5
tools/r02/pmc_mem.sh big 32768 32768 grey 200 8 1
echo probe2 done
