#!/usr/bin/env bash
# Round-2 probe 59: measured halo-mode selection in bench.py: multi-process
# rehearsals (ranks sharing the GPU, gloo-host halos), then the driver's N=2
# command with the default RCCL transport on this one-GPU box (the exchange
# check cannot build an RCCL communicator with two ranks on one GPU: the
# pre-loaded headline must still be printed, halo_select = preload).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe59
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multiproc.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --exchange-timeout 20 > "$O/bench_n2.json" 2> "$O/bench_n2.err" || echo "bench n2 rc=$?"
cut -c1-400 "$O/bench_n2.json"
python3 -c "
import json
d=json.loads([l for l in open('$O/bench_n2.json') if l.startswith('{')][0]); print(d['ms_per_step'], d.get('halo_select'), str(d.get('halo_exchange'))[:300])"
