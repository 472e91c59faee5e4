#!/usr/bin/env bash
# Round-2 probe 4: resident service (GPU test + CUDA-table sweep through it),
# driver bench with the new fields, PMC passes with a pinned tile shape, the
# MPI / MPI+OpenMP tables on this box's CPU share.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe4
mkdir -p "$O"
rc=0
timeout -k 10 300 python3 -u -m pytest tests/test_service.py tests/test_gpu_halo.py -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || rc=$?
tail -n 3 "$O/pytest.log"
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
timeout -k 10 300 python3 -u tools/ref_tables.py cuda --service --out "$O/cuda_service.jsonl" > "$O/cuda_service.log" 2>&1
echo cuda-service ok
for i in 1 2; do
  timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_$i.json" 2> "$O/bench_$i.err"
done
echo bench ok
PCONV_SWAR_SHAPE=4,8,8 PCONV_SWAR_ALT=1 tools/r02/pmc_mem.sh head_pinned 1920 2520 rgb 40 8 5
PCONV_SWAR_SHAPE=8,8,8 PCONV_SWAR_ALT=1 tools/r02/pmc_mem.sh big_pinned 32768 32768 grey 200 8 1
timeout -k 10 600 python3 -u tools/ref_tables.py mpi-cpu --runs 1 --out "$O/mpi_cpu.jsonl" > "$O/mpi_cpu.log" 2>&1
echo probe4 done
