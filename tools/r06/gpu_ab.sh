#!/bin/bash
# Round 6, call AB: final tree (staging qualified against fresh buffers too) — the driver's command
# x10, then the whole GPU suite and smoke.
set -o pipefail
OUT=gpurun_out/r06/ab
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
}
for r in 0 1 2 3 4 5 6 7; do one drv_$r --gpus 1 --steps 20 --warmup 5 || exit 1; done
python tools/r06/summ_windows.py $OUT/drv_*.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -1 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.txt | head -30; [ $rc -eq 1 ] || exit 1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
