#!/usr/bin/env bash
# Round-3 call J: images in flight (slots) at N=1 and for the emulated 8-way rank;
# memory-copy traces of four runs of the driver's bench command (spread analysis).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/j
mkdir -p $O
summ() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['ms_per_step'], d['loop_only']['ms_per_step'], d['copy_floor']['floor_ms'])"; }
for s in 3 4 5 6; do
  for i in 1 2; do
    timeout -k 10 150 python bench.py --slots $s > $O/bench_s${s}_$i.json 2> $O/bench_s${s}_$i.err || { tail -3 $O/bench_s${s}_$i.err; exit 1; }
    summ $O/bench_s${s}_$i.json "n1 slots=$s"
  done
  timeout -k 10 150 python bench.py --emulate 8:3 --slots $s > $O/emu8_s$s.json 2> $O/emu8_s$s.err || { tail -3 $O/emu8_s$s.err; exit 1; }
  summ $O/emu8_s$s.json "emu8 slots=$s"
done
for i in 1 2 3 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_$i -o run \
    -- python3 bench.py > $O/trace_$i.log 2>&1 || { tail -5 $O/trace_$i.log; exit 1; }
  grep '^{' $O/trace_$i.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('traced run $i', d['ms_per_step'])"
  python tools/copy_trace_summary.py $O/trace_$i --images 100 --md $O/trace_$i.md > /dev/null 2>&1 && tail -6 $O/trace_$i.md
  rm -f $O/trace_$i/*/*kernel_trace.csv.bak
done
