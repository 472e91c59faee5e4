#!/bin/bash
# Round 6, call Y: is the streamed head worth it inside a 20-image window?
# The driver's command A/B: head streamed (default) vs every image one step
# graph (--stream-chunks 0), 6 interleaved pairs.
set -o pipefail
OUT=gpurun_out/r06/y
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']; print(sys.argv[1], d['ms_per_step'], d['latency_ms'], d['copy_floor']['pair_ms'], w.get('windows_ms_summary') if isinstance(w, dict) else '')" $OUT/$name.json
}
for r in 0 1 2 3 4 5; do
  one head_$r --gpus 1 --steps 20 --warmup 5 || exit 1
  one graph_$r --gpus 1 --steps 20 --warmup 5 --stream-chunks 0 || exit 1
done
python tools/r06/distributions.py "head=$OUT/head_*.json" "graph=$OUT/graph_*.json"
