#!/usr/bin/env bash
# Round-2 probe 18: where the HIP runtime start-up (hipInit 120-256 ms) goes.
# Fresh processes only; no kernels beyond the CLI's own.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe18
mkdir -p "$O"
{
  echo "dri: $(ls /dev/dri 2>&1 | tr '\n' ' ')"
  echo "kfd nodes: $(ls /sys/class/kfd/kfd/topology/nodes 2>&1 | tr '\n' ' ')"
  for n in /sys/class/kfd/kfd/topology/nodes/*; do
    echo "node $(basename $n): $(cat $n/name 2>/dev/null) simd=$(grep -m1 simd_count $n/properties 2>/dev/null | cut -d' ' -f2)"
  done
  echo "cpus online: $(cat /sys/devices/system/cpu/online)"
  grep -m1 MemTotal /proc/meminfo
  echo "env ROCR_VISIBLE_DEVICES=${ROCR_VISIBLE_DEVICES-unset} HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES-unset}"
} > "$O/system.txt" 2>&1
H=tools/ubench/hsa_cost
for i in 1 2 3; do timeout -k 5 60 $H >> "$O/hsa_default.jsonl"; done
for i in 1 2 3; do ROCR_VISIBLE_DEVICES=0 timeout -k 5 60 $H >> "$O/hsa_rocr0.jsonl"; done
CONV=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
wall() {  # external wall (ms) of one fresh conv process + its JSON line
  local t0 t1 line
  t0=$(date +%s%N)
  line=$(timeout -k 5 60 "$@" --synthetic 1 --json --out /tmp/p18.raw 2>/dev/null | tail -n 1)
  t1=$(date +%s%N)
  echo "{\"wall_ms\": $(( (t1 - t0) / 1000000 )), \"report\": $line}"
}
for i in 1 2 3; do wall $CONV x.raw 1920 630 10 grey >> "$O/conv_default.jsonl"; done
for i in 1 2 3; do ROCR_VISIBLE_DEVICES=0 wall $CONV x.raw 1920 630 10 grey >> "$O/conv_rocr0.jsonl"; done
for i in 1 2 3; do HIP_ENABLE_DEFERRED_LOADING=0 wall $CONV x.raw 1920 630 10 grey >> "$O/conv_nodefer.jsonl"; done
LD_DEBUG=statistics timeout -k 5 60 $CONV --help > "$O/ld_stats.txt" 2>&1 || true
cat "$O/system.txt"
cut -c1-200 "$O/hsa_default.jsonl" "$O/hsa_rocr0.jsonl"
for f in conv_default conv_rocr0 conv_nodefer; do python3 -c "
import json
for l in open('$O/$f.jsonl'):
    d = json.loads(l); r = d['report']
    print('$f', d['wall_ms'], r.get('since_exec_s'), r.get('e2e_s', r.get('total_s')), (r.get('phases_s') or {}).get('hip_init'))
"; done
