#!/usr/bin/env bash
# The BASELINE.json configurations on ONE MI355X (run on the GPU box).
#   1) native CLI `conv` on a synthetic image: loop time (hipEvent) and
#      end-to-end time incl. HIP init, H2D, D2H and the output write;
#   2) bench.py serving step (H2D + reps + D2H per image, pipelined).
# Large frames run in steady state (round 3, call Z: 3 images in flight and
# 10+ timed steps; 2 slots x 3 steps measured mostly the pipeline fill).
# One JSON line per run in gpurun_out/baseline/*.json.  Each step has its own
# time limit; the script stops at the first failure.
set -euo pipefail
OUT=${OUT:-gpurun_out/r03/baseline}
mkdir -p "$OUT"
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
run() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  tail -n 1 "$OUT/$name.log" | tee "$OUT/$name.json"
}
run cli_64_grey_cpu     60 $CONV x.raw 64 64 1 grey --synthetic 1 --backend cpu --check --json --quiet --out /tmp/o0.raw
run cli_1920x2520_rgb   60 $CONV x.raw 1920 2520 40 rgb --synthetic 1 --check --json --quiet --out /tmp/o1.raw
run cli_1920x2520_grey  60 $CONV x.raw 1920 2520 40 grey --synthetic 1 --check --json --quiet --out /tmp/o2.raw
run cli_1920x5040_rgb   60 $CONV x.raw 1920 5040 100 rgb --synthetic 1 --check --json --quiet --out /tmp/o3.raw
run cli_8192_rgb_100   120 $CONV x.raw 8192 8192 100 rgb --synthetic 1 --json --quiet --out /tmp/o4.raw
run cli_32768_grey_200 180 $CONV x.raw 32768 32768 200 grey --synthetic 1 --json --quiet --out /tmp/o5.raw
rm -f /tmp/o[0-5].raw
run bench_1920x2520_rgb  120 python3 bench.py --steps 50 --warmup 10
run bench_1920x2520_grey 120 python3 bench.py --channels grey --steps 50 --warmup 10
run bench_8192_rgb_100   180 python3 bench.py --width 8192 --height 8192 --reps 100 --steps 30 --warmup 5
run bench_32768_grey_200 300 python3 bench.py --width 32768 --height 32768 --channels grey --reps 200 --steps 10 --warmup 2

# round 3: the reference's other filters, and per-rank proxies of the 8-GPU BASELINE configs
run cli_1920x2520_rgb_box  60 $CONV x.raw 1920 2520 40 rgb --filter box --synthetic 1 --check --json --quiet --out /tmp/o6.raw
run cli_1920x2520_rgb_edge 60 $CONV x.raw 1920 2520 40 rgb --filter edge --synthetic 1 --check --json --quiet --out /tmp/o7.raw
rm -f /tmp/o6.raw /tmp/o7.raw
run bench_1920x2520_rgb_box 120 python3 bench.py --filter box --steps 50 --warmup 10
run emu8_8192_rgb_100   180 python3 bench.py --emulate 8:3 --width 8192 --height 8192 --reps 100 --steps 60 --warmup 10
run emu8_32768_grey_200 300 python3 bench.py --emulate 8:3 --width 32768 --height 32768 --channels grey --reps 200 --steps 20 --warmup 3
echo "baseline configs done"
