#!/usr/bin/env bash
# Round-2 probe 6: full GPU suite (engine ctor / copy changes), cold CUDA
# table with CU copies + one hardware queue, RCCL overlap trace with the
# interior launch enqueued ahead of the transfer.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe6
mkdir -p "$O"
rc=0
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || rc=$?
tail -n 4 "$O/pytest_gpu.log"
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
timeout -k 10 300 python3 -u tools/ref_tables.py cuda --out "$O/cuda_cold.jsonl" > "$O/cuda_cold.log" 2>&1
echo cuda cold ok
timeout -k 10 300 python3 -u tools/ref_tables.py cuda --runs 1 --out "$O/cuda_cold_sdma.jsonl" --extra --copies sdma > "$O/cuda_cold_sdma.log" 2>&1
echo cuda cold sdma ok
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/ov_rccl" -o run \
  -- python3 tools/overlap_trace.py run rccl-self --iters 4 > "$O/ov_rccl.log" 2>&1
echo probe6 done
