#!/usr/bin/env bash
# Round-3 call W: the driver's N=8 launch path rehearsed with 8 ranks sharing
# the one GPU (gloo-host halos; RCCL refuses two ranks on one device): every
# halo mode timed, bytes checked against the headline.  Then the headline at
# N=1 once more on this box.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/w
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 \
  --master-port 29617 bench.py --gpus 8 --steps 50 --warmup 5 --transport gloo-host --check > $O/rehearsal8.json 2> $O/rehearsal8.err \
  || { tail -20 $O/rehearsal8.err; exit 1; }
grep '^{' $O/rehearsal8.json | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('n', d['n_gpus'], 'ms', d['ms_per_step'], 'mismatches', d['mismatches'], 'per_rank', d['per_rank_ms_per_step'])
for m, r in d['halo_modes'].items(): print(' ', m, r['status'], r.get('ms_per_step'), r.get('mismatches_vs_headline'), r.get('exchanges_per_step'))
print('select', d['halo_select']['mode'], d['halo_select']['reason'])"
timeout -k 10 150 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -5 $O/bench_n1.err; exit 1; }
tail -1 $O/bench_n1.json | cut -c1-220
