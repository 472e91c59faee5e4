#!/usr/bin/env python3
"""One line per bench JSON: the timed window, the replayed windows
(min / median / max), and per slot the mean completion delta of the steady
images (3rd to 17th) of the fastest and slowest marked windows — a slot whose
images are steadily slower than the copy floor is a per-stream effect, random
slow images are a dynamic one."""
import json
import statistics
import sys


def per_slot(w):
    acc = {}
    for i, (s, d) in enumerate(zip(w["slots"], w["deltas_ms"])):
        if 2 <= i < len(w["slots"]) - 3:
            acc.setdefault(s, []).append(d)
    return " ".join(f"s{s}:{statistics.mean(v):.3f}" for s, v in sorted(acc.items()))


for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f"{path}: unreadable ({e})")
        continue
    w = d.get("windows") or {}
    ws = sorted(w.get("ms_per_step") or [0])
    mk = sorted(w.get("marked_ms_per_step") or [0])
    line = (f"{path.split('/')[-1]:14s} timed {d['ms_per_step']:.4f} pair {d['copy_floor'].get('pair_ms')} "
            f"win {ws[0]:.4f}/{ws[len(ws) // 2]:.4f}/{ws[-1]:.4f} marked {mk[0]:.4f}/{mk[len(mk) // 2]:.4f}/{mk[-1]:.4f}")
    if "fastest_marked" in w:
        line += f" | fast {per_slot(w['fastest_marked'])} | slow {per_slot(w['slowest_marked'])}"
    print(line)
