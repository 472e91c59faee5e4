#!/usr/bin/env bash
# Round-2 probe 3: full GPU suite after the kernel edge-row change, HIP
# start-up cost per step (fresh processes, env variants), PMC passes with the
# tile shape pinned (so every pass measures the same kernel).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe3
mkdir -p "$O"
rc=0
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || rc=$?
tail -n 4 "$O/pytest_gpu.log"
if [ "$rc" -gt 1 ]; then exit "$rc"; fi
IC=tools/ubench/init_cost
for i in 1 2 3; do timeout -k 5 60 $IC >> "$O/init_default.jsonl"; done
for i in 1 2; do HIP_VISIBLE_DEVICES=0 timeout -k 5 60 $IC >> "$O/init_visible0.jsonl"; done
for i in 1 2; do GPU_MAX_HW_QUEUES=1 timeout -k 5 60 $IC >> "$O/init_hwq1.jsonl"; done
for i in 1 2; do HSA_ENABLE_SDMA=0 timeout -k 5 60 $IC >> "$O/init_nosdma.jsonl"; done
for i in 1 2; do HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 5 60 $IC >> "$O/init_nodefer.jsonl"; done
AMD_LOG_LEVEL=4 timeout -k 5 60 $IC > "$O/init_log4.txt" 2>&1
tail -n 1 "$O/init_default.jsonl"
nproc > "$O/nproc.txt"; cat /proc/cpuinfo | grep "model name" | head -1 >> "$O/nproc.txt"; ls /dev/dri >> "$O/nproc.txt" 2>&1 || true
env | grep -E "^(HIP|HSA|ROC|GPU|AMD)" >> "$O/nproc.txt" || true
PCONV_SWAR_SHAPE=4,8,8 PCONV_SWAR_ALT=1 tools/r02/pmc_mem.sh head_pinned 1920 2520 rgb 40 8 5
PCONV_SWAR_SHAPE=8,8,8 PCONV_SWAR_ALT=1 tools/r02/pmc_mem.sh big_pinned 32768 32768 grey 200 8 1
echo probe3 done
