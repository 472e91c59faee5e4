#!/usr/bin/env python3
"""Summarise a wave-image task timeline (PCONV_WAVE_TRACE=file, engine.cpp
enqueue_wave): one JSON line per traced image, every task as
[kind, level, a, b, part, tile, claimed, deps_met, done, wg | xcc << 32] with
wall-clock ticks (100 MHz).

Prints, per image: the span of the launch, the loads' effective H2D rate and
when the last one finished, the stores' D2H rate and the tail after the last
load, and per task kind / level the median and p90 of the time spent waiting
for dependencies and running.
"""
from __future__ import annotations

import argparse
import json
import statistics

TICK_US = 0.01  # wall_clock64 at 100 MHz


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else float("nan")


def summarise(rec) -> list[str]:
    tasks = rec["tasks"]
    rb = rec["row_bytes"]
    t0 = min(t[6] for t in tasks)
    us = lambda x: (x - t0) * TICK_US  # noqa: E731
    out = []
    end = max(us(t[8]) for t in tasks)
    loads = [t for t in tasks if t[0] == 0]
    stores = [t for t in tasks if t[0] == 2]
    comp = [t for t in tasks if t[0] == 1]
    lb = sum((t[3] - t[2]) * rb for t in loads)
    sb = sum((t[3] - t[2]) * rb for t in stores)
    l_first, l_last = min(us(t[7]) for t in loads), max(us(t[8]) for t in loads)
    s_first, s_last = min(us(t[7]) for t in stores), max(us(t[8]) for t in stores)
    wgs = {t[9] & 0xFFFFFFFF for t in tasks}
    out.append(f"span {end:.1f} us, {len(tasks)} tasks on {len(wgs)} workgroups")
    out.append(f"loads  {len(loads):4d}: {lb / 1e6:.2f} MB from {l_first:.1f} to {l_last:.1f} us = "
               f"{lb / max(l_last - l_first, 1e-9) / 1e3:.1f} GB/s; per task run p50 "
               f"{statistics.median(us(t[8]) - us(t[7]) for t in loads):.1f} us")
    out.append(f"stores {len(stores):4d}: {sb / 1e6:.2f} MB from {s_first:.1f} to {s_last:.1f} us = "
               f"{sb / max(s_last - s_first, 1e-9) / 1e3:.1f} GB/s; tail after the last load {s_last - l_last:.1f} us")
    levels = sorted({t[1] for t in comp})
    for j in levels:
        tj = [t for t in comp if t[1] == j]
        wait = [us(t[7]) - us(t[6]) for t in tj]
        run = [us(t[8]) - us(t[7]) for t in tj]
        out.append(f"level {j:2d} {len(tj):5d} tasks: wait p50 {pct(wait, .5):6.1f} p90 {pct(wait, .9):6.1f} us; "
                   f"run p50 {pct(run, .5):5.1f} p90 {pct(run, .9):5.1f} us; last done {max(us(t[8]) for t in tj):.1f} us")
    # front: the time each level finished its first / last row tile
    return out


def main():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("trace")
    p.add_argument("--image", type=int, default=-1, help="which traced image (default: the last)")
    a = p.parse_args()
    recs = [json.loads(l) for l in open(a.trace) if l.strip()]
    for line in summarise(recs[a.image]):
        print(line)


if __name__ == "__main__":
    main()
