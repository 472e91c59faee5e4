#!/usr/bin/env bash
# Round-3 call N: captured split (overlap) exchange images, selftests, emulations, copy-only period.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -k "slot_pipeline or selftests" -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head; exit 1; }
for m in preload overlap slot_exchange slot_exchange_direct; do
  timeout -k 10 150 python bench.py --emulate 8:3 --emulate-halo $m --steps 200 --warmup 20 > $O/emulate8_$m.json 2> $O/emulate8_$m.err || { tail -5 $O/emulate8_$m.err; exit 1; }
  tail -1 $O/emulate8_$m.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$m', d['ms_per_step'], c['exchanges_per_step'], c['halo_depth'], c['step_graphs'], d['loop_only']['ms_per_step'])"
done
bash tools/r03/gpu_m.sh
