#!/usr/bin/env bash
# Round-2 probe 42: the driver's N>1 command with the DEFAULT transport (RCCL)
# on a one-GPU box (two ranks share the GPU): the headline must still print;
# the RCCL halo_exchange measurement reports whatever RCCL does here.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe42
mkdir -p "$O"
rc=0
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29631 bench.py --gpus 2 --steps 20 --warmup 5 > "$O/bench2.json" 2> "$O/bench2.err" || rc=$?
echo "rc=$rc"
grep -c '^{' "$O/bench2.json" || true
python3 -c "
import json
d = [json.loads(l) for l in open('$O/bench2.json') if l.startswith('{')][-1]
print(d['ms_per_step'], d['n_gpus'], d.get('headline_transport'), json.dumps(d.get('halo_exchange'))[:300])"
