#!/usr/bin/env bash
# Round-3 call AH: evidence refresh after the pair-sum step — SQ counters of
# the three production loops (headline, 8-way band, 32768^2 grey; shapes
# pinned to the tuner's picks, two passes of <= 8 SQ counters each), and a
# rocprofv3 kernel + memory-copy trace with stats of the headline bench.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ah
mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
for w in ${WORKLOADS:-headline band8 grey32768}; do
  case $w in
    headline) export PCONV_SWAR_SHAPE=4,8,8 PCONV_PREFETCH=1 PCONV_SWAR_ALT=1 ;;
    band8) export PCONV_SWAR_SHAPE=4,5,8 PCONV_PREFETCH=0 PCONV_SWAR_ALT=1 ;;
    grey32768) export PCONV_SWAR_SHAPE=4,20,8 PCONV_PREFETCH=0 PCONV_SWAR_ALT=1 ;;
  esac
  iters=20; [ $w = grey32768 ] && iters=3
  i=0
  for c in "$A" "$B"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${w}_p$i -o run -- python3 tools/r03/pmc_loops.py $w --iters $iters > $O/${w}_p$i.log 2>&1 \
      || { echo "pass $w $i failed"; tail -5 $O/${w}_p$i.log; exit 1; }
    grep tuned $O/${w}_p$i.log | cut -c1-160
  done
done
unset PCONV_SWAR_SHAPE PCONV_PREFETCH PCONV_SWAR_ALT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/bench -o run -- python3 bench.py --steps 200 --warmup 30 > $O/bench_under_rocprof.json 2> $O/bench_rocprof.err \
  || { tail -5 $O/bench_rocprof.err; exit 1; }
tail -1 $O/bench_under_rocprof.json | cut -c1-200
echo "call ah done"
