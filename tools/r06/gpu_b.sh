#!/bin/bash
# Round 6, call B: which copy engine serves which slot stream?
#  1. one run of the driver's command with the HIP runtime's full log; the
#     copy / engine lines kept;
#  2. interleaved A/B of ROCr's SDMA engine policies (gang copies,
#     recommended engines) against the default, 3 rounds.
set -o pipefail
OUT=gpurun_out/r06/b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
ls -la /sys/class/kfd/kfd/proc/ > $OUT/kfd_proc.txt 2>&1 || true
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x7fffffff one fulllog --gpus 1 --steps 20 --warmup 5 --diag-windows 2 || exit 1
grep -aiE "engine|sdma|blit|copy|rect|graph" $OUT/fulllog.err | head -c 30000000 > $OUT/fulllog_copy.txt || true
grep -aiE "engine|sdma" $OUT/fulllog.err | head -c 3000000 > $OUT/fulllog_engine.txt || true
wc -l $OUT/fulllog.err $OUT/fulllog_copy.txt $OUT/fulllog_engine.txt
rm -f $OUT/fulllog.err
for r in 0 1 2; do
  one base_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  HSA_ENABLE_SDMA_GANG=0 one nogang_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  HSA_ENABLE_SDMA_RECOMMENDED_ENG=0 one norec_$r --gpus 1 --steps 20 --warmup 5 || exit 1
done
python tools/r06/summ_windows.py $OUT/*.json
# 3. the changed native paths: IPC (uncached mailboxes, self-test), captured
#    exchanges with the interior || exchange fork, every tile shape
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ipc.py \
  > $OUT/tests_ipc.log 2>&1 || { echo "ipc tests failed"; grep -E "FAILED|ERROR|Error" $OUT/tests_ipc.log | head -20; tail -5 $OUT/tests_ipc.log; exit 1; }
tail -1 $OUT/tests_ipc.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_halo.py -k "captured or mid_image" \
  > $OUT/tests_halo.log 2>&1 || { echo "halo tests failed"; grep -E "FAILED|ERROR" $OUT/tests_halo.log | head -20; tail -5 $OUT/tests_halo.log; exit 1; }
tail -1 $OUT/tests_halo.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "every" \
  > $OUT/tests_shapes.log 2>&1 || { echo "shape tests failed"; grep -E "FAILED|ERROR" $OUT/tests_shapes.log | head -20; tail -5 $OUT/tests_shapes.log; exit 1; }
tail -1 $OUT/tests_shapes.log
# 4. resident loop proxies: exchange then launches vs the interior || exchange
#    fork; one image vs two concurrent; RCCL to self and IPC self-pulls
for e in 2:0 4:1 8:3; do
  n=${e%%:*}
  for mode in event ipc; do
    for ov in off on; do
      for im in 1 2; do
        name=e${n}_${mode}_ov${ov}_im${im}
        timeout -k 10 300 python -u bench.py --emulate $e --emulate-halo $mode --steps 100 --warmup 10 --diag-windows 0 \
          --resident-overlap $ov --resident-images $im > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; exit 1; }
        python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d.get('resident_loop') or d.get('resident_loop_ipc'); print(sys.argv[2], d['ms_per_step'], r.get('ms_per_image'), r.get('exchanges_per_image'), r.get('launches_per_image'))" $OUT/$name.json $name
      done
    done
  done
done
# 5. large-frame tile shapes
timeout -k 10 300 python -u tools/r06/shape_sweep.py > $OUT/shape_sweep.jsonl 2> $OUT/shape_sweep.err || { echo "sweep failed"; tail -5 $OUT/shape_sweep.err; exit 1; }
cat $OUT/shape_sweep.jsonl
