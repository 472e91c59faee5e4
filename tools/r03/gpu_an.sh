#!/usr/bin/env bash
# Round-3 call AN: run-to-run spread of the headline step with the runtime's
# SDMA copy engines (default) vs CU blit kernels for every copy
# (HSA_ENABLE_SDMA=0), alternating, 200- and 20-step regions.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/an
mkdir -p $O
one() {  # tag env steps warmup
  local tag=$1 e=$2 k=$3 w=$4
  env $e timeout -k 10 150 python3 bench.py --steps $k --warmup $w > $O/$tag.json 2> $O/$tag.err || { tail -3 $O/$tag.err; exit 1; }
  tail -1 $O/$tag.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'], 'loop', d['loop_only']['ms_per_step'], 'floor', d['copy_floor']['h2d_ms'], d['copy_floor']['d2h_ms'], 'lat', d['latency_ms'])" | tee -a $O/summary.txt
}
for r in 1 2 3; do
  one sdma_k200_$r HSA_ENABLE_SDMA=1 200 30
  one blit_k200_$r HSA_ENABLE_SDMA=0 200 30
  one sdma_k20_$r HSA_ENABLE_SDMA=1 20 5
  one blit_k20_$r HSA_ENABLE_SDMA=0 20 5
done
echo "call an done"
