#!/usr/bin/env bash
# Round-3 call P: split captured exchange images after the stream-role swap; emulations;
# then which half of torch's stack recurses (torch's HIP 7.0 runtime with ROCm 7.2's librccl).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py -k "slot_pipeline or selftests" -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/pytest.log | head; exit 1; }
for m in overlap preload slot_exchange slot_exchange_direct; do
  timeout -k 10 150 python bench.py --emulate 8:3 --emulate-halo $m --steps 200 --warmup 20 > $O/emulate8_$m.json 2> $O/emulate8_$m.err || { tail -5 $O/emulate8_$m.err; exit 1; }
  tail -1 $O/emulate8_$m.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$m', d['ms_per_step'], c['exchanges_per_step'], c['halo_depth'], c['step_graphs'], d['loop_only']['ms_per_step'])"
done
f=$O/torch_rccl272_sendrecv_fork_relaxed
PCONV_RCCL_LIB=/opt/rocm/lib/librccl.so.1 timeout -k 5 90 python3 -c "
import sys; sys.path.insert(0, '.')
import pconv
pconv.native.install_crash_handler()
print(pconv.native.rccl_capture_probe('sendrecv_fork', 'relaxed', 4096, 0))
print(pconv.native.runtime_info())
" > "$f.out" 2> "$f.err"
rc=$?; echo "torch HIP + ROCm librccl: rc=$rc"; cat "$f.out" | tail -2
[ $rc -ne 0 ] && { grep -v "NCCL INFO" "$f.err" | awk '!/libamdhip64.so\(\+0x2d34a8\)/ || !seen++' | tail -20; }
exit 0
