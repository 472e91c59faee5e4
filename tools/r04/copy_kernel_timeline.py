#!/usr/bin/env python3
"""Merge a rocprofv3 kernel trace and memory-copy trace (csv) into one
timeline: consecutive kernels of a stream within 0.5 ms are folded into one
run; every copy is listed with its stream.  Used for the large-frame steady
state (profiles/r04/big/timeline.txt): which copies overlap which loops.

usage: copy_kernel_timeline.py TRACE_DIR [--first N] [--last N]
"""
import argparse
import csv
import glob
import os


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace_dir")
    p.add_argument("--first", type=int, default=80)
    p.add_argument("--last", type=int, default=0)
    a = p.parse_args()
    kf = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    cf = glob.glob(os.path.join(a.trace_dir, "**", "*memory_copy_trace.csv"), recursive=True)[0]
    ev = [("K", int(r["Stream_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:24])
          for r in csv.DictReader(open(kf))]
    ev += [("C", int(r["Stream_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"][12:])
           for r in csv.DictReader(open(cf))]
    ev.sort(key=lambda e: e[2])
    t0 = ev[0][2]
    runs = []
    for kind, s, b, e, name in ev:
        b, e = (b - t0) / 1e6, (e - t0) / 1e6  # ms
        if runs and kind == "K" and runs[-1][0] == "K" and runs[-1][1] == s and b - runs[-1][3] < 0.5:
            k, s0, b0, _, n0, cnt = runs[-1]
            runs[-1] = (k, s0, b0, e, n0, cnt + 1)
            continue
        runs.append((kind, s, b, e, name, 1))
    sel = runs[:a.first] + (runs[-a.last:] if a.last else [])
    print(f"{'start ms':>9} {'end ms':>9} kind stream {'dur ms':>7}  what")
    for kind, s, b, e, name, cnt in sel:
        what = f"{cnt} kernels ({name})" if kind == "K" else f"copy {name}"
        print(f"{b:9.2f} {e:9.2f} {kind:>4} {s:6d} {e - b:7.2f}  {what}")


if __name__ == "__main__":
    main()
