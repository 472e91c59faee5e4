#!/usr/bin/env bash
# Round-3 call AG: 16-wave tall tiles ({4,12,16}, {4,16,16}: 192 / 256 rows,
# fewer halo rows per kept row) with the pair-sum step's lower VGPR counts
# (bin/conv_x16 = -DPCONV_EXTRA_SHAPES), forced shapes vs the production pick,
# CLI loop time, best of 3.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ag
mkdir -p $O
B=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin
one() {  # tag shape fuse args...
  local tag=$1 shape=$2 fuse=$3; shift 3
  local envs=""
  [ "$shape" != auto ] && envs="PCONV_SWAR_SHAPE=$shape PCONV_PREFETCH=0"
  env $envs timeout -k 10 120 $B/conv_x16 x.raw "$@" --fuse $fuse --synthetic 1 --json --quiet --out /tmp/ag.raw > /tmp/ag.json 2>$O/err.txt || { cat $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/ag.json')); print('$tag', '$shape', $fuse, round(d['loop_s']*1e3,4), d.get('mismatches'))" >> $O/ag.txt
}
for r in 1 2 3; do
  for sh in auto 4,20,8 4,12,16 4,16,16; do
    for f in 12 16; do one g32768 $sh $f 32768 32768 200 grey; done
    one rgb8192 $sh 8 8192 8192 100 rgb
    one grey1920 $sh 8 1920 2520 40 grey --check
    one rgb1920 $sh 8 1920 2520 40 rgb --check
  done
  echo "round $r"
done
rm -f /tmp/ag.raw
python3 - $O/ag.txt <<'PY'
import sys,collections
d=collections.defaultdict(list); bad=0
for l in open(sys.argv[1]):
    t,sh,f,v,m=l.split(); d[(t+' f'+f,sh)].append(float(v)); bad+=(m not in ('0','-1'))
rows=sorted({k for k,_ in d}); shapes=['auto','4,20,8','4,12,16','4,16,16']
print('config'.ljust(16)+''.join(s.rjust(10) for s in shapes))
for r in rows: print(r.ljust(16)+''.join((('%.4f'%min(d[(r,s)])) if (r,s) in d else '-').rjust(10) for s in shapes))
print('mismatching runs:', bad)
PY
