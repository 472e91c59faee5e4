#!/bin/bash
# Round 6, call T: the driver's SCALE command rehearsed on the final tree
# with N ranks sharing the one GPU of a gpurun box (N = 2, 4, 8):
#   python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... \
#     bench.py --gpus N --steps 20 --warmup 5
# (gloo-host transport for the RCCL halo modes — RCCL refuses two ranks on
# one device — HIP IPC for `ipc`), then the two large BASELINE configs at
# N = 8.  Records each line's wall time, the per-rank copy floors alone
# (pair_ms_solo) and all ranks at once (pair_ms_concurrent: N ranks on one
# link, so ~N x contention expected here), and the halo modes.
set -o pipefail
OUT=gpurun_out/r06/t
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
run() {  # name, nproc, timeout, bench args
  local name=$1 n=$2 lim=$3; shift 3
  local port=$((29500 + RANDOM % 2000))
  local t0=$(date +%s.%N)
  timeout -k 10 $lim python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 20 --warmup 5 --transport gloo-host "$@" \
    > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  local t1=$(date +%s.%N)
  python - "$OUT/$name.out" "$name" "$rc" "$t0" "$t1" <<'PY'
import json, sys
path, name, rc, t0, t1 = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4]), float(sys.argv[5])
lines = [l for l in open(path).read().splitlines() if l.startswith("{")]
rec = {"name": name, "rc": rc, "wall_s": round(t1 - t0, 1)}
if lines:
    d = json.loads(lines[-1])
    cf = d.get("copy_floor", {})
    rec.update(n_gpus=d["n_gpus"], ms_per_step=d["ms_per_step"], mismatches=d.get("mismatches"),
               per_rank=d["per_rank_ms_per_step"], pair_ms_solo=cf.get("pair_ms_solo"),
               pair_ms_concurrent=cf.get("pair_ms_concurrent"), latency_ms=d.get("latency_ms"),
               halo_select=d.get("halo_select", {}).get("mode"),
               modes={m: (r.get("status"), r.get("ms_per_step"), r.get("mismatches")) for m, r in
                      d.get("halo_modes", {}).items()},
               resident_loop=d.get("resident_loop"))
print(json.dumps(rec))
PY
  return $rc
}
run n2 2 300 | tee -a $OUT/summary.jsonl || exit 1
run n4 4 300 | tee -a $OUT/summary.jsonl || exit 1
run n8 8 400 | tee -a $OUT/summary.jsonl || exit 1
run n8_rgb8192 8 400 --width 8192 --height 8192 --channels rgb --reps 100 | tee -a $OUT/summary.jsonl || exit 1
run n8_grey32768 8 600 --width 32768 --height 32768 --channels grey --reps 200 | tee -a $OUT/summary.jsonl || exit 1
