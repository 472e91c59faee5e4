#!/usr/bin/env bash
# Evidence refresh for the current tree (run on the GPU box, from the repo root):
# bench line, rocprofv3 kernel trace of the headline bench, SQ counters of the
# headline loop (N=1 and one rank of an 8-way split) and of 32768^2 grey,
# and the BASELINE.json configurations.  Every GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/rprof
mkdir -p "$O"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS"
timeout -k 10 120 python3 bench.py > "$O/bench_n1.json" 2> "$O/bench_n1.err"
echo "bench: $(cut -c1-160 "$O/bench_n1.json")"
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trace_bench" -o run \
  -- python3 bench.py --steps 50 --warmup 10 --loop-steps 50 > "$O/trace_bench.log" 2>&1
echo "trace done"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$O/pmc_rgb" -o run --pmc $SQ GRBM_GUI_ACTIVE \
  -- python3 tools/kernel_sweep.py --width 1920 --height 2520 --channels rgb --reps 40 --fuse 8 --rounds 1 --iters 5 \
  > "$O/pmc_rgb.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$O/pmc_rgb_w8" -o run --pmc $SQ GRBM_GUI_ACTIVE \
  -- python3 tools/kernel_sweep.py --width 1920 --height 2520 --channels rgb --reps 40 --fuse 8 --rounds 1 --iters 5 \
  --world 8 --rank 3 > "$O/pmc_rgb_w8.log" 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O/pmc_grey32k" -o run --pmc $SQ GRBM_GUI_ACTIVE \
  -- python3 tools/kernel_sweep.py --width 32768 --height 32768 --channels grey --reps 16 --fuse 8 --rounds 1 --iters 2 \
  > "$O/pmc_grey32k.log" 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d "$O/tcc_grey32k" -o run --pmc FETCH_SIZE \
  -- python3 tools/kernel_sweep.py --width 32768 --height 32768 --channels grey --reps 16 --fuse 8 --rounds 1 --iters 2 \
  > "$O/tcc_grey32k.log" 2>&1
echo "pmc done"
if [ "${BASELINE:-1}" = 1 ]; then timeout -k 10 900 tools/baseline_configs.sh > "$O/baseline.log" 2>&1; fi
echo "round profile done"
