#!/bin/bash
# Round 4 (session 2): where a streamed single image's 0.56 ms goes (kernel +
# copy trace of the latency loop), and the CLI ring's download || write with
# SDMA vs CU-kernel copies and 32 vs 64 MB chunks.
set -o pipefail
OUT=gpurun_out/r04/lat_trace
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr -o run \
  -- python3 bench.py --gpus 1 --steps 4 --warmup 1 --no-check > $OUT/tr.json 2> $OUT/tr.err \
  || { echo "trace failed"; tail -5 $OUT/tr.err; exit 1; }
tail -1 $OUT/tr.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('latency', d['latency_ms'])"
python tools/r04/copy_kernel_timeline.py $OUT/tr --first 400 > $OUT/timeline.txt
C=parallel-image-convolution-using-mpi-openmp-and-cuda_amd/bin/conv
for v in "kernel 33554432" "sdma 33554432" "sdma 67108864" "kernel 67108864"; do
  set -- $v
  n=cli_32768_$1_$2
  PCONV_RING_CHUNK_BYTES=$2 timeout -k 10 300 $C /tmp/x.raw 32768 32768 200 grey --synthetic 7 --backend hip --copies $1 --json --quiet --out /tmp/o.raw > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['e2e_s'],4), d['phases_s'])" $OUT/$n.json
done
