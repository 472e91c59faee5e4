#!/usr/bin/env bash
# Round-3 call AO: kernel + copy trace of the driver's command (20 timed
# images) to see how the pipeline's head and tail run.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ao
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-160
ls $O/trace
echo "call ao done"
