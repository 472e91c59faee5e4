#!/usr/bin/env bash
# Round-2 probe 33: packed-row D2H (contiguous copy from a device staging
# buffer) against the pitched 2-D D2H, same box, interleaved; correctness.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/r02/probe33
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_multiproc.py -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
tail -n 2 "$O/pytest.log"
timeout -k 5 120 tools/ubench/copy_bw 2520 20 > "$O/copy_bw_2520.txt" 2>&1
timeout -k 5 120 tools/ubench/copy_bw 395 40 > "$O/copy_bw_395.txt" 2>&1
grep -E "pitched|contiguous  " "$O/copy_bw_2520.txt" | tail -n 4
for i in 1 2 3; do
  for m in on off; do
    timeout -k 10 120 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --check --packed-d2h $m >> "$O/bench_n1_$m.jsonl" 2>> "$O/bench.err"
    timeout -k 10 120 python3 -u bench.py --emulate 8:3 --steps 40 --warmup 5 --packed-d2h $m >> "$O/bench_e8_$m.jsonl" 2>> "$O/bench.err"
  done
done
python3 - <<'P'
import json
O = "gpurun_out/r02/probe33"
for f in ("bench_n1_on", "bench_n1_off", "bench_e8_on", "bench_e8_off"):
    rows = [json.loads(l) for l in open(f"{O}/{f}.jsonl") if l.startswith("{")]
    print(f, [r["ms_per_step"] for r in rows], "mism", [r.get("mismatches") for r in rows], "floor", [r["copy_floor"]["floor_ms"] for r in rows], "packed", [r["config"].get("packed_d2h") for r in rows])
P
