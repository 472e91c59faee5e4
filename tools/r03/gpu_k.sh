#!/usr/bin/env bash
# Round-3 call K: MFMA prototype exactness, timing against the VALU kernels, SQ counters.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/k
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -k "mfma" -x -q --timeout 120 --timeout-method thread > $O/pytest_mfma.log 2>&1
rc=$?; tail -3 $O/pytest_mfma.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 150 python -u tools/r03/mfma_compare.py > $O/mfma_compare.jsonl 2> $O/mfma_compare.err || { tail -5 $O/mfma_compare.err; exit 1; }
cat $O/mfma_compare.jsonl
timeout -k 10 90 rocprofv3 --list-avail > $O/avail.txt 2>&1
want=""
for c in SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES; do
  grep -qw "$c" $O/avail.txt && want="$want $c"
done
echo "counters:$want"
set -- $want
p1="${@:1:8}"
timeout -s KILL 90 rocprofv3 --pmc $p1 --output-format csv -d $O/pmc -o run -- python3 tools/r03/mfma_compare.py --iters 3 > $O/pmc.log 2>&1
echo "pmc rc=$?"
ls $O/pmc/ 2>/dev/null | head
