#!/bin/bash
# Round 6, call E: why one staging buffer copies slowly.  Interleaved A/B of
# staging qualification (DMA through every buffer at set-up) and a CPU cache
# flush of the input buffers after the CPU wrote them (clflush).
set -o pipefail
OUT=gpurun_out/r06/e
mkdir -p $OUT
export PYTHONUNBUFFERED=1
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
for r in 0 1 2 3; do
  one nqnf_$r --gpus 1 --steps 20 --warmup 5 --qualify-staging off --flush-staging off || exit 1
  one nqf_$r --gpus 1 --steps 20 --warmup 5 --qualify-staging off --flush-staging on || exit 1
  one qnf_$r --gpus 1 --steps 20 --warmup 5 --qualify-staging on --flush-staging off || exit 1
  one qf_$r --gpus 1 --steps 20 --warmup 5 --qualify-staging on --flush-staging on || exit 1
done
python tools/r06/summ_windows.py $OUT/*.json
python - $OUT <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    st = d.get("staging") or {}
    print(f.split("/")[-1], "replaced", st.get("replaced"), "slot buffers h2d at end", [r[0] for r in d["windows"].get("slot_buffer_copy_ms", [])])
PY
