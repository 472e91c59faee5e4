#!/bin/bash
# Round 6, call C: ROCr's SDMA gang policy on / off, 8 interleaved pairs of the
# driver's command (off is now bench.py's default); the 8-way per-rank proxy
# both ways; the resident loop with 1-4 concurrent images.
set -o pipefail
OUT=gpurun_out/r06/c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
for r in 0 1 2 3 4 5 6 7; do
  one off_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  one on_$r --gpus 1 --steps 20 --warmup 5 --sdma-gang on || exit 1
done
python tools/r06/summ_windows.py $OUT/off_*.json $OUT/on_*.json
for g in off on; do
  for r in 0 1; do
    one e8_$g$r --emulate 8:3 --steps 20 --warmup 5 --sdma-gang $g || exit 1
  done
done
python tools/r06/summ_windows.py $OUT/e8_*.json
for e in 8:3 4:1 2:0; do
  n=${e%%:*}
  for mode in event ipc; do
    for im in 2 3 4; do
      name=rl${n}_${mode}_im${im}
      one $name --emulate $e --emulate-halo $mode --steps 100 --warmup 10 --diag-windows 0 --resident-images $im || exit 1
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d.get('resident_loop') or d.get('resident_loop_ipc'); print(sys.argv[2], d['ms_per_step'], r.get('ms_per_image'))" $OUT/$name.json $name
    done
  done
done
