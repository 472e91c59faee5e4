#!/bin/bash
# Round 4: hypothesis tests for the 4+-slot collapse (two of four slot queues
# run every stencil launch ~5x longer): the KFD's view of the device's
# queues, then the 8-way proxy with slot streams on dedicated CU-masked
# queues (all CUs / CUs split between slots) and with alternating priorities;
# a trace of the best variant.  Then the per-rank proxy of the halo modes
# (RCCL and IPC to self) and the multi-process rehearsals.
set -o pipefail
OUT=gpurun_out/r04/slots_b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
for f in /sys/class/kfd/kfd/topology/nodes/*/properties; do
  if grep -q "simd_count [1-9]" $f; then echo "== $f"; grep -E "cpu_cores|simd_count|num_cp_queues|num_sdma|max_waves|cu_per|num_xcc|array_count|gfx_target|hive|num_gws" $f; fi
done > $OUT/kfd_props.txt 2>&1
for p in hws_max_conc_proc sched_policy cwsr_enable mes queue_preemption_timeout_ms sched_hw_submission; do
  [ -r /sys/module/amdgpu/parameters/$p ] && echo "$p $(cat /sys/module/amdgpu/parameters/$p)"
done >> $OUT/kfd_props.txt 2>&1
cat $OUT/kfd_props.txt
one() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 150 python -u bench.py --no-check "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:22s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']}")
PY
}
E="--emulate 8:3 --steps 300 --warmup 30"
for s in 3 4 6; do one s${s} X=1 -- $E --slots $s || exit 1; done
for m in cumask cusplit prio; do
  for s in 3 4 6; do one s${s}_$m PCONV_SLOT_STREAMS=$m -- $E --slots $s || exit 1; done
done
one n1_cumask PCONV_SLOT_STREAMS=cumask -- --steps 200 --warmup 30 || exit 1
one n1_s4_cumask PCONV_SLOT_STREAMS=cumask -- --steps 200 --warmup 30 --slots 4 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_s4_cumask -o run \
  -- python3 bench.py $E --slots 4 --no-check > $OUT/trace_s4_cumask.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace_s4_cumask.log; exit 1; }
d=$(dirname $(find $OUT/trace_s4_cumask -name run_kernel_trace.csv | head -1))
python tools/queue_trace_summary.py $d --json $OUT/trace_s4_cumask_summary.json | head -12
for m in preload slot_exchange ipc; do one e8_$m X=1 -- --emulate 8:3 --emulate-halo $m --steps 300 --warmup 30 || exit 1; done
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_multiproc.py -k "rehearsal or watchdog" > $OUT/pytest_multiproc.txt 2>&1 || { echo "multiproc tests failed"; tail -40 $OUT/pytest_multiproc.txt; exit 1; }
tail -2 $OUT/pytest_multiproc.txt
timeout -k 10 300 $PYT tests/test_gpu_stream.py -k native > $OUT/pytest_native.txt 2>&1 || { echo "native bench tests failed"; tail -30 $OUT/pytest_native.txt; exit 1; }
tail -2 $OUT/pytest_native.txt
