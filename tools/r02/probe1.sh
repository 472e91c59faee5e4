#!/usr/bin/env bash
# Round-2 first GPU probe: GPU tests, the driver's bench command, and a
# kernel + memory-copy trace of exactly that command.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe1
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
tail -n 3 "$O/pytest_gpu.log"
for i in 1 2 3; do
  timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver_$i.json" 2> "$O/bench_driver_$i.err"
  cut -c1-400 "$O/bench_driver_$i.json"
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trace_driver" -o run \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/trace_driver.log" 2>&1
echo trace ok
