#!/bin/bash
# Round 6, call H: the 8-way proxy in every IPC pull form and the other halo modes (300
# images), the BASELINE large frames on one GPU, and a rocprofv3 kernel +
# copy trace of the driver's command.
set -o pipefail
OUT=gpurun_out/r06/h
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py -k "two_head or head_stream_modes" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 0 1 2 3 4 5; do
  one h1_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 4 || exit 1
  one h2_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 4 --head-images 2 || exit 1
done
python tools/r06/summ_windows.py $OUT/h1_*.json $OUT/h2_*.json
for r in 0 1 2 3; do
  one plain_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 2 || exit 1
  one marked_$r --gpus 1 --steps 20 --warmup 5 --diag-windows 2 --mark-timed || exit 1
done
python tools/r06/summ_windows.py $OUT/plain_*.json $OUT/marked_*.json
one s200 --gpus 1 --steps 200 --warmup 30 --diag-windows 0 || exit 1
for e in 2:0 4:1 8:3; do
  n=${e%%:*}
  one e${n}_w20 --emulate $e --steps 20 --warmup 5 || exit 1
done
python tools/r06/summ_windows.py $OUT/e*_w20.json
one e8_preload --emulate 8:3 --steps 300 --warmup 10 --diag-windows 0 || exit 1
for p in grid single sdma; do
  one e8_ipc_$p --emulate 8:3 --emulate-halo ipc --ipc-pull $p --steps 300 --warmup 10 --diag-windows 0 || exit 1
done
one e8_slotx --emulate 8:3 --emulate-halo slot_exchange --steps 300 --warmup 10 --diag-windows 0 || exit 1
python - $OUT <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("resident_loop") or d.get("resident_loop_ipc") or {}
    print(f.split("/")[-1], d["ms_per_step"], "pair", d["copy_floor"]["pair_ms"], "lat", d.get("latency_ms"),
          "loop", d["loop_only"]["ms_per_step"], "resident", r.get("ms_per_image"), (r.get("one_image") or {}).get("ms_per_image"),
          "mism", d.get("mismatches"))
PY
one big8192 --gpus 1 --width 8192 --height 8192 --reps 100 --steps 20 --warmup 5 --diag-windows 2 || exit 1
one big32768 --gpus 1 --width 32768 --height 32768 --channels grey --reps 200 --steps 10 --warmup 3 --diag-windows 1 || exit 1
python tools/r06/summ_windows.py $OUT/big*.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --diag-windows 2 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo "rocprof failed"; tail -5 $OUT/prof_bench.err; exit 1; }
find $OUT/prof -name "*stats*" | head
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/lat -o lat -- python3 tools/r06/latency_probe.py --images 12 > $OUT/lat_probe.json 2> $OUT/lat_probe.err || { echo "latency trace failed"; tail -5 $OUT/lat_probe.err; exit 1; }
cat $OUT/lat_probe.json
python tools/r06/latency_timeline.py $OUT/lat --images 2 > $OUT/lat_timeline.txt 2>&1 || true
head -c 20000000 $OUT/lat_timeline.txt > /dev/null
find $OUT/lat -name "*.csv" -size +20M -delete
