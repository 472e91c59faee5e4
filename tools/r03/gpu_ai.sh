#!/usr/bin/env bash
# Round-3 call AI: float temporal kernel without the v_med3_f32 clamp (the
# u8 packer saturates) — float GPU tests (bit-exact vs the float32 oracle,
# filters with negative taps and sums outside [0, 255]), then box / edge
# loop and bench times.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ai
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "float" --timeout 170 --timeout-method thread > $O/pytest_float.log 2>&1
rc=$?; tail -2 $O/pytest_float.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/pytest_float.log | head -20; exit 1; }
B=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin
for r in 1 2 3; do
  for f in box edge; do
    timeout -k 10 60 $B/conv x.raw 1920 2520 40 rgb --filter $f --synthetic 1 --check --json --quiet --out /tmp/ai.raw > /tmp/ai.json 2>$O/err.txt || { cat $O/err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/ai.json')); print('$f', round(d['loop_s']*1e6/40,3), 'us/rep', d['mismatches'])" | tee -a $O/cli.txt
  done
done
for f in box edge; do
  timeout -k 10 120 python3 bench.py --filter $f --steps 50 --warmup 10 > $O/bench_$f.json 2> $O/bench_$f.err || { tail -3 $O/bench_$f.err; exit 1; }
  tail -1 $O/bench_$f.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench $f', d['ms_per_step'], 'loop', d['loop_only']['ms_per_step'], d['loop_only']['us_per_rep'])"
done
rm -f /tmp/ai.raw
echo "call ai done"
