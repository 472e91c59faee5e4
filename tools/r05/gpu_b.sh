#!/bin/bash
# Round 5, second GPU call: stagger and stream-sync modes removed, IPC
# signalling through device-memory mailboxes, SWAR step form 2.  The whole
# GPU suite, smoke, the IPC pull probe, the driver's command, 200 images, the
# 8-way proxy (preload and every IPC pull form), the teardown probe and SQ
# counters.
set -o pipefail
OUT=gpurun_out/r05/b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
# plain test failures (rc 1) do not stop the measurements; a timeout, abort
# or crash of the test process does
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -1 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.txt | head -30; [ $rc -eq 1 ] || exit 1; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed"; cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 200 python -u tools/r05/ipc_probe.py --workgroups 0,8,16,32,64 > $OUT/ipc_probe.jsonl 2> $OUT/ipc_probe.err || { echo "probe failed"; tail -20 $OUT/ipc_probe.err; exit 1; }
cat $OUT/ipc_probe.jsonl
one() {  # name, -- bench args
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -5 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:14s} ms/step {d['ms_per_step']:.4f} latency {d['latency_ms']:.4f} pair {d['copy_floor']['pair_ms']} loop {d['loop_only']['ms_per_step']} mism {d.get('mismatches')} vs {d.get('vs_baseline')}")
PY
}
for i in a b c; do one bench_$i --gpus 1 --steps 20 --warmup 5 || exit 1; done
one s200 --steps 200 --warmup 5 || exit 1
one e8 --emulate 8:3 --steps 300 --warmup 10 || exit 1
for p in grid single sdma; do one e8_ipc_$p --emulate 8:3 --emulate-halo ipc --ipc-pull $p --steps 300 --warmup 10 || exit 1; done
one e8_rccl --emulate 8:3 --emulate-halo slot_exchange --steps 300 --warmup 10 || exit 1
bash tools/r05/teardown.sh > $OUT/teardown.txt 2>&1 || { echo "teardown probe failed"; tail -5 $OUT/teardown.txt; exit 1; }
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r05/teardown/next.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    by[r["prev"]].append(r["next"]["hip_init_ms"])
for k, v in by.items():
    v.sort()
    print(f"prev={k:9s} next hip_init ms median {v[len(v)//2]:7.1f} all {v}")
PY
O=gpurun_out/r05/pmc bash tools/r05/gpu_pmc.sh || exit 1
