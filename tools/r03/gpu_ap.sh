#!/usr/bin/env bash
# Round-3 call AP: concurrent copy-pair floor in the bench JSON — its GPU
# test, the bench rehearsals (N>1 ranks on one GPU), and the bench itself.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ap
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_multiproc.py -m gpu -x -q -k "copy_pair or bench" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
for a in "" "--steps 20 --warmup 5" "--emulate 8:3"; do
  timeout -k 10 150 python3 bench.py $a > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
  tail -1 $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench [$a]', d['ms_per_step'], d['copy_floor'])" | tee -a $O/summary.txt
done
echo "call ap done"
