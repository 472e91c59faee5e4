#!/bin/bash
# Round 5: back-to-back start-up cost vs what the previous process did
# (tools/ubench/teardown_probe.hip).  For every mode: 5 pairs of
# (previous process, next process measuring its hipInit), no gap; and the
# idle baseline (2 s gap).
set -o pipefail
OUT=gpurun_out/r05/teardown
mkdir -p $OUT
B=/tmp/teardown_probe
hipcc --offload-arch=gfx950 -O2 tools/ubench/teardown_probe.hip -o $B || exit 1
for mode in idle init stream pinned dev kernel all all_free conv; do
  for i in 1 2 3 4 5; do
    if [ $mode = idle ]; then sleep 2;
    elif [ $mode = conv ]; then timeout -k 5 60 parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv s.raw 1920 630 10 grey --synthetic 1 --quiet --out /tmp/o.raw > /dev/null || exit 1;
    else timeout -k 5 60 $B $mode 15 >> $OUT/prev.jsonl || exit 1; fi
    r=$(timeout -k 5 60 $B measure) || exit 1
    echo "{\"prev\": \"$mode\", \"next\": $r}" | tee -a $OUT/next.jsonl
  done
done
