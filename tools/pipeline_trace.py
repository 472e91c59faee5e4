#!/usr/bin/env python3
"""Summarise a pipeline stage trace written by `bench.py --trace N`.

Per image: H2D (start..end), reps (H2D end..reps end), D2H (reps end..D2H
end), and the interval between consecutive H2D starts (the pipeline period).
Prints medians and the first images' timeline."""
import json
import statistics
import sys


def main(path):
    d = json.load(open(path))
    ms = d["ms"]
    rows = []
    for i, (slot, a, b, c, e) in enumerate(ms):
        period = a - ms[i - 1][1] if i else float("nan")
        rows.append(dict(slot=int(slot), start=a, h2d=b - a, reps=c - b, d2h=e - c, latency=e - a, period=period))
    us = lambda v: f"{v * 1e3:7.1f}"
    print(f"{len(rows)} images; args: slots={d['args'].get('slots')} emulate={d['args'].get('emulate')} "
          f"graph_capture={d['args'].get('graph_capture')} step_graphs={d['args'].get('step_graphs')}")
    body = rows[len(rows) // 4:]
    for k in ("h2d", "reps", "d2h", "latency", "period"):
        vals = [r[k] for r in body if r[k] == r[k]]
        print(f"  median {k:8s} {us(statistics.median(vals))} us")
    slots = sorted({r["slot"] for r in body})
    if len(slots) > 1:
        print("  per slot median reps / latency (us): " + ", ".join(
            f"slot {k}: {us(statistics.median(r['reps'] for r in body if r['slot'] == k)).strip()} / "
            f"{us(statistics.median(r['latency'] for r in body if r['slot'] == k)).strip()}" for k in slots))
    total = ms[-1][4] - ms[0][1]
    print(f"  wall {us(total)} us for {len(ms)} images = {us(total / len(ms))} us/image")
    print("  img slot   start     h2d    reps     d2h  (us)")
    for i, r in enumerate(rows[:24]):
        print(f"  {i:3d} {r['slot']:4d} {us(r['start'])} {us(r['h2d'])} {us(r['reps'])} {us(r['d2h'])}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pipeline_trace.json")
