#!/usr/bin/env bash
# Round-3 call AC: A/B of CLI variants (BINS, default the step-order builds of
# tools/r03/build_variant.sh); loop time of each config, 3 alternating rounds.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/${TAG:-ac}
mkdir -p $O
B=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin
BINS=${BINS:-"conv conv_o1 conv_o2 conv_o3 conv_o4"}
one() {  # tag bin args...
  local tag=$1 bin=$2; shift 2
  timeout -k 10 120 $B/$bin x.raw "$@" --synthetic 1 --json --quiet --out /tmp/ab.raw > /tmp/ab.json 2>$O/err.txt || { cat $O/err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/ab.json')); print('$tag', '$bin', round(d['loop_s']*1e3,4), d.get('mismatches'))" >> $O/ab.txt
}
for r in 1 2 3; do
  for bin in $BINS; do
    one g32768 $bin 32768 32768 200 grey
    one rgb1920 $bin 1920 2520 40 rgb --check
    one grey1920 $bin 1920 2520 40 grey --check
    one rgb8192 $bin 8192 8192 100 rgb
    one band8 $bin 1920 395 40 rgb --check
    one g16384 $bin 16384 16384 40 grey
  done
  echo "round $r done"
done
rm -f /tmp/ab.raw
python3 - $O/ab.txt <<'PY'
import sys,collections
d=collections.defaultdict(list); bad=0
for l in open(sys.argv[1]):
    t,b,v,m=l.split(); d[(t,b)].append(float(v)); bad+= (m not in ('0','-1'))
tags=sorted({t for t,_ in d}); bins=[]
for _,b in d:
    if b not in bins: bins.append(b)
print('config'.ljust(10)+''.join(b.rjust(12) for b in bins))
for t in tags: print(t.ljust(10)+''.join(('%.4f'%min(d[(t,b)])).rjust(12) for b in bins))
print('mismatching runs:',bad)
PY
