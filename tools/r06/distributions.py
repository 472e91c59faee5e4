#!/usr/bin/env python3
"""Distributions behind docs/PERFORMANCE.md: for each named group of bench
JSON files, min / median / max and count of the timed window (ms/step), of
every replayed window (plain and marked), of latency_ms, loop_only and the
pair floor, and the share of windows above 1.15 x the line's own pair floor.

    python tools/r06/distributions.py 'final=profiles/r06/f/drv_*.json' ...
"""
import glob
import json
import statistics
import sys


def load(path):
    for line in reversed(open(path).read().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise ValueError(f"{path}: no JSON line")


def dist(v):
    if not v:
        return "—"
    v = sorted(v)
    return f"{v[0]:.4f} / {statistics.median(v):.4f} / {v[-1]:.4f} (n={len(v)})"


def main():
    for arg in sys.argv[1:]:
        name, pat = arg.split("=", 1)
        files = sorted(glob.glob(pat))
        timed, wins, lat, loop, pair, over = [], [], [], [], [], 0
        for f in files:
            d = load(f)
            timed.append(d["ms_per_step"])
            p = (d.get("copy_floor") or {}).get("pair_ms")
            if p:
                pair.append(p)
            if d.get("latency_ms"):
                lat.append(d["latency_ms"])
            lo = (d.get("loop_only") or {}).get("ms_per_step")
            if lo:
                loop.append(lo)
            w = d.get("windows") or {}
            ws = list(w.get("ms_per_step") or []) + list(w.get("marked_ms_per_step") or [])
            wins += ws
            if p:
                over += sum(1 for x in ws + [d["ms_per_step"]] if x > 1.15 * p)
        print(f"## {name}: {len(files)} lines ({pat})")
        print(f"  timed window ms/step  {dist(timed)}")
        print(f"  replayed windows      {dist(wins)}")
        print(f"  windows > 1.15 x pair {over} of {len(wins) + len(timed)}")
        print(f"  latency_ms            {dist(lat)}")
        print(f"  loop_only ms          {dist(loop)}")
        print(f"  pair floor ms         {dist(pair)}")


if __name__ == "__main__":
    main()
