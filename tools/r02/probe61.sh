#!/usr/bin/env bash
# Round-2 probe 61: exchange-mode images = upload, ONE whole-zone exchange,
# the repetitions as the engine's cached graph, download: halo / multiproc /
# engine suites (ranks sharing the GPU, gloo-host halos; RCCL self tests).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe61
mkdir -p "$O"
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_halo.py tests/test_gpu_multiproc.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 20 --warmup 5 --transport gloo-host --check > "$O/bench_n4_gloo.json" 2> "$O/bench_n4_gloo.err"
python3 -c "
import json
d=json.loads([l for l in open('$O/bench_n4_gloo.json') if l.startswith('{')][0]); print(d['ms_per_step'], d['mismatches'], d.get('halo_select'), str(d.get('halo_exchange'))[:300])"
