#!/bin/bash
# Round 5: SQ counters of the production launch of the
# headline loop, the 8-way band loop and the 32768^2 grey loop.  The tuner's
# pick is taken first (no profiler) and then forced, so every pass counts
# the same kernel; two passes of <= 8 SQ counters (+1 GRBM) each, each its
# own rocprofv3 run under a hard time limit.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r05/pmc}
mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
for w in ${WHICH:-headline band8 grey32768}; do
  pick=$(timeout -k 10 180 python3 tools/r05/pmc_loops.py $w --pick | tail -1) || { echo "pick $w failed"; exit 1; }
  echo "$w pick: $pick" | tee $O/${w}_pick.json
  shape=$(echo "$pick" | python3 -c "import json,sys;print(json.load(sys.stdin)['shape'])")
  form=$(echo "$pick" | python3 -c "import json,sys;print(json.load(sys.stdin)['form'])")
  pf=$(echo "$pick" | python3 -c "import json,sys;print(json.load(sys.stdin)['pf'])")
  i=0
  for c in "$A" "$B"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${w}_p$i -o run -- \
      python3 tools/r05/pmc_loops.py $w --shape $shape --form $form --pf $pf > $O/${w}_p$i.log 2>&1 \
      || { echo "pass $w $i failed"; tail -5 $O/${w}_p$i.log; exit 1; }
  done
  python3 tools/r03/pmc_breakdown.py $O/${w}_p1 $O/${w}_p2 --title "$w: $pick" --md $O/${w}.md | tail -12
done
