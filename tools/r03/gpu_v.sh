#!/usr/bin/env bash
# Round-3 call V: SQ counters of the headline loop and of the 8-way band loop
# (VERDICT r02 item 3 asks for counters behind any rejection).  Two passes of
# at most 8 SQ counters each (+1 GRBM), each its own rocprofv3 run.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/v
mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
# shapes pinned to the tuner's production picks (tuning under counters
# picks differently, and the passes must count the same kernel)
for w in headline band8; do
  if [ $w = headline ]; then export PCONV_SWAR_SHAPE=4,8,8 PCONV_PREFETCH=1 PCONV_SWAR_ALT=1;
  else export PCONV_SWAR_SHAPE=4,5,8 PCONV_PREFETCH=1 PCONV_SWAR_ALT=0; fi
  i=0
  for c in "$A" "$B"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/${w}_p$i -o run -- python3 tools/r03/pmc_loops.py $w > $O/${w}_p$i.log 2>&1 \
      || { echo "pass $w $i failed"; tail -5 $O/${w}_p$i.log; exit 1; }
    grep tuned $O/${w}_p$i.log | cut -c1-200
  done
done
