#!/bin/bash
# Round 6, call D: staging-buffer qualification (every slot's pinned buffers
# timed at set-up, slow ones replaced) on by default; NUMA placement of the
# staging pages; the resident loop with concurrent images.
set -o pipefail
OUT=gpurun_out/r06/d
mkdir -p $OUT
export PYTHONUNBUFFERED=1
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
for r in 0 1 2 3 4 5; do
  one q_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  one nq_$r --gpus 1 --steps 20 --warmup 5 --qualify-staging off || exit 1
done
for r in 6 7 8 9; do one q_$r --gpus 1 --steps 20 --warmup 5 || exit 1; done
python tools/r06/summ_windows.py $OUT/q_*.json $OUT/nq_*.json
python - $OUT <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*q_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    st = d.get("staging") or {}
    print(f.split("/")[-1], "replaced", st.get("replaced"), "first h2d", [r[0] for r in st.get("h2d_d2h_pair_ms_first", [])],
          "slot_bufs", [r[0] for r in d["windows"].get("slot_buffer_copy_ms", [])], "numa", json.dumps(d.get("staging_numa"))[:300])
PY
for e in 8:3 4:1 2:0; do
  n=${e%%:*}
  for mode in event ipc; do
    for im in 2 3; do
      name=rl${n}_${mode}_im${im}
      one $name --emulate $e --emulate-halo $mode --steps 100 --warmup 10 --diag-windows 0 --resident-images $im || exit 1
      python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d.get('resident_loop') or d.get('resident_loop_ipc'); print(sys.argv[2], d['ms_per_step'], r.get('ms_per_image'), r.get('one_image'))" $OUT/$name.json $name
    done
  done
done
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_engine.py -k "staging or slot_streams" tests/test_gpu_stream.py -k "native_bench or staging or slot_streams" \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|ERROR" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
