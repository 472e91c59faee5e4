#!/usr/bin/env python3
"""Timeline of the last head-streamed images of a latency_probe.py trace:
HIP API calls (host), SDMA copies and kernels (device) on one clock, in µs
from the image's first hipMemcpy2DAsync.  Answers: how long after the API
call that issued it does each chunk copy start, and how long after the
kernel / copy it waits for.

usage: latency_timeline.py TRACE_DIR [--images 2]
"""
import argparse
import csv
import glob
import os


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace_dir")
    p.add_argument("--images", type=int, default=2)
    a = p.parse_args()
    ev = []
    for r in rows(a.trace_dir, "*hip_api_trace.csv"):
        n = r.get("Function") or r.get("Operation") or r.get("Name")
        if n and any(k in n for k in ("Memcpy", "Launch", "EventRecord", "StreamWait", "GraphLaunch", "Synchronize")):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API", n))
    for r in rows(a.trace_dir, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY",
                   f'{r.get("Direction", "")} {int(r.get("Bytes", 0) or 0) / 1e6:.2f} MB'))
    for r in rows(a.trace_dir, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "KERN", r["Kernel_Name"][:40]))
    ev.sort()
    # image starts: a hipMemcpy2DAsync API call more than 0.3 ms after the previous one
    starts, last = [], None
    for b, e, k, n in ev:
        if k == "API" and "Memcpy2D" in n:
            if last is None or b - last > 300_000:
                starts.append(b)
            last = b
    for s0 in starts[-a.images:]:
        print(f"---- image at {s0}")
        for b, e, k, n in ev:
            if s0 - 50_000 <= b <= s0 + 900_000:
                print(f"{(b - s0) / 1e3:9.1f} {(e - s0) / 1e3:9.1f} {(e - b) / 1e3:7.1f}  {k:4s} {n}")


if __name__ == "__main__":
    main()
