#!/usr/bin/env bash
# Round-3 call AE: tuner picks with the pair-sum step and the updated launch
# model (DPP operand cost), default 6 candidates vs all 19 shapes.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03/ae
mkdir -p $O
timeout -k 10 240 python3 tools/r03/loop_probe.py --large > $O/default.jsonl 2> $O/default.err || { tail -5 $O/default.err; exit 1; }
PCONV_TUNE_CANDIDATES=19 timeout -k 10 400 python3 tools/r03/loop_probe.py --large > $O/all19.jsonl 2> $O/all19.err || { tail -5 $O/all19.err; exit 1; }
python3 - <<'PY'
import json
for f in ("default", "all19"):
    for l in open(f"gpurun_out/r03/ae/{f}.jsonl"):
        d = json.loads(l); print(f, d["frame"], d["world"], d["us_per_rep"], d["tuned"][-1][1] if d["tuned"] else None, d["tuned"][-1][0][4:] if d["tuned"] else None)
PY
