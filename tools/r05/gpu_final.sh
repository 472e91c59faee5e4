#!/bin/bash
# Round 5, final verification on the final tree: the whole GPU suite and
# smoke, the driver's command (3 runs), the 8-way per-rank proxies
# (pre-loaded and IPC halos, event mode's resident loop), and the N = 8
# rehearsal of the driver's SCALE command for the headline.
set -o pipefail
OUT=gpurun_out/r05/final
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -1 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.txt | head -30; [ $rc -eq 1 ] || exit 1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:12s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} "
      f"mism {d.get('mismatches')} resident {json.dumps(d.get('resident_loop', {}).get('ms_per_image'))}")
PY
}
for i in 1 2 3; do one drv_$i --gpus 1 --steps 20 --warmup 5 || exit 1; done
one e8_preload --emulate 8:3 --steps 300 --warmup 10 || exit 1
one e8_ipc --emulate 8:3 --emulate-halo ipc --steps 300 --warmup 10 || exit 1
one e8_event --emulate 8:3 --emulate-halo event --steps 100 --warmup 10 || exit 1
OUT=gpurun_out/r05/final/scale8 bash tools/r05/scale8_rehearsal.sh headline || exit 1
