#!/usr/bin/env bash
# Memory-hierarchy counters for the production kernels:
# HBM/MALL traffic (FETCH_SIZE, WRITE_SIZE), L2 hit/miss, EA requests and LDS
# bank conflicts, one rocprofv3 pass per counter group (a pass may hold at
# most 4 TCC / 8 SQ / 2 GRBM counters), each under its own hard time limit.
#   $1 = tag, rest = tools/loop_once.py args: W H channels reps fuse iters
set -euo pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/r02/pmc_$TAG
mkdir -p "$O"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$O/$name" -o run --pmc "$@" \
    -- python3 tools/loop_once.py $ARGS > "$O/$name.log" 2>&1
  echo "pass $name ok"
}
ARGS="$*"
pass fetch FETCH_SIZE
pass write_l2 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
pass ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
echo "pmc $TAG done"
