set -e
B="timeout -k 5 120 python bench.py --steps 300 --warmup 40 --loop-steps 5 --trace 60"
$B --emulate 8:3 --slots 3 --graph-capture off --trace-out gpurun_out/tr_emu8_s3.json > gpurun_out/tr1.log 2>&1
$B --emulate 8:3 --slots 4 --graph-capture off --trace-out gpurun_out/tr_emu8_s4.json > gpurun_out/tr2.log 2>&1
$B --emulate 8:3 --slots 3 --step-graphs off --trace-out gpurun_out/tr_emu8_ev3.json > gpurun_out/tr3.log 2>&1
$B --slots 3 --graph-capture off --trace-out gpurun_out/tr_n1_s3.json > gpurun_out/tr4.log 2>&1
$B --slots 4 --graph-capture off --trace-out gpurun_out/tr_n1_s4.json > gpurun_out/tr5.log 2>&1
for f in gpurun_out/tr_*.json; do python tools/pipeline_trace.py $f; done > gpurun_out/trace_summary.txt
