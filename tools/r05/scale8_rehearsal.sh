#!/bin/bash
# Round 5: the driver's SCALE command at N = 8 on the
# final tree, rehearsed with 8 ranks sharing the one GPU of a gpurun box:
#   python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 ... \
#     bench.py --gpus 8 --steps 20 --warmup 5
# for the headline and the two large BASELINE configs, with every halo mode
# timed after the headline (gloo-host transport for the RCCL modes — RCCL
# refuses two ranks on one device — and HIP IPC for `ipc`) and the default
# oracle check.  Each line's wall time is recorded next to it.
set -o pipefail
OUT=${OUT:-gpurun_out/r05/scale8}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
run() {  # name, timeout, bench args
  local name=$1 lim=$2; shift 2
  local port=$((29500 + RANDOM % 2000))
  local t0=$(date +%s.%N)
  timeout -k 10 $lim python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 8 --steps 20 --warmup 5 --transport gloo-host "$@" \
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
    rec.update(n_gpus=d["n_gpus"], ms_per_step=d["ms_per_step"], mismatches=d.get("mismatches"),
               per_rank=len(d["per_rank_ms_per_step"]), h2d_bytes=d.get("h2d_bytes_per_step"),
               d2h_bytes=d.get("d2h_bytes_per_step"), halo_select=d.get("halo_select", {}).get("mode"),
               modes={m: (r.get("status"), r.get("ms_per_step"), r.get("mismatches")) for m, r in
                      d.get("halo_modes", {}).items()},
               resident_loop=d.get("resident_loop"))
print(json.dumps(rec))
PY
  return $rc
}
ONLY=${1:-all}  # one config name, or all
want() { [ "$ONLY" = all ] || [ "$ONLY" = "$1" ]; }
if want headline; then run headline 600 | tee -a $OUT/summary.jsonl || exit 1; fi
if want rgb8192; then run rgb8192 600 --width 8192 --height 8192 --channels rgb --reps 100 | tee -a $OUT/summary.jsonl || exit 1; fi
if want grey32768; then
  run grey32768 600 --width 32768 --height 32768 --channels grey --reps 200 | tee -a $OUT/summary.jsonl || exit 1
fi
