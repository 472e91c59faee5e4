#!/usr/bin/env python3
"""Where the time of a pipelined bench run goes, per hardware queue and per
stream, from a rocprofv3 --kernel-trace --memory-copy-trace (VERDICT r03
item 2: why 4+ images in flight collapse the 8-way per-rank step).

For the last --window fraction of the trace (the timed images) it reports:
  * per Queue_Id: stencil launches, their durations (p50 / p90), busy time;
  * copies: durations (p50 / p90), bytes-free busy time per stream;
  * the period (window / images) and how much of the window each engine
    class (stencil kernels, copies) is busy — a queue-scheduling stall shows
    as kernels stretched far beyond their solo duration while the device is
    otherwise idle, an SDMA-queue stall as copies stretched the same way.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import statistics


def union(iv):
    if not iv:
        return 0
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


def pct(v, q):
    if not v:
        return None
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def summarize(trace_dir, window=0.6, stencil=("k_swar", "k_binomial", "k_float")):
    kt = os.path.join(trace_dir, "run_kernel_trace.csv")
    ct = os.path.join(trace_dir, "run_memory_copy_trace.csv")
    ks = list(csv.DictReader(open(kt))) if os.path.exists(kt) else []
    cs = list(csv.DictReader(open(ct))) if os.path.exists(ct) else []
    ev = [int(k["Start_Timestamp"]) for k in ks] + [int(c["Start_Timestamp"]) for c in cs]
    if not ev:
        return {}
    t_end = max([int(k["End_Timestamp"]) for k in ks] + [int(c["End_Timestamp"]) for c in cs])
    t0 = t_end - (t_end - min(ev)) * window
    kern = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k.get("Queue_Id", "?"), k.get("Stream_Id", "?"),
             k["Kernel_Name"]) for k in ks if int(k["Start_Timestamp"]) >= t0]
    sten = [x for x in kern if any(s in x[4] for s in stencil)]
    cops = [(int(c["Start_Timestamp"]), int(c["End_Timestamp"]), c.get("Stream_Id", "?")) for c in cs
            if int(c["Start_Timestamp"]) >= t0]
    win = t_end - t0
    out = {"window_us": win / 1e3, "stencil_launches": len(sten), "copies": len(cops)}
    q = {}
    for s, e, qu, st, _ in sten:
        q.setdefault(qu, []).append((s, e))
    out["queues"] = {qu: {"launches": len(v), "p50_us": pct([(e - s) / 1e3 for s, e in v], 0.5),
                          "p90_us": pct([(e - s) / 1e3 for s, e in v], 0.9),
                          "busy_frac": union(v) / win} for qu, v in sorted(q.items())}
    d = [(e - s) / 1e3 for s, e, *_ in sten]
    out["stencil_p50_us"], out["stencil_p90_us"] = pct(d, 0.5), pct(d, 0.9)
    out["stencil_mean_us"] = statistics.mean(d) if d else None
    out["stencil_busy_frac"] = union([(s, e) for s, e, *_ in sten]) / win
    c = [(e - s) / 1e3 for s, e, _ in cops]
    out["copy_p50_us"], out["copy_p90_us"] = pct(c, 0.5), pct(c, 0.9)
    out["copy_busy_frac"] = union([(s, e) for s, e, _ in cops]) / win
    per = {}
    for s, e, st in cops:
        per.setdefault(st, []).append((s, e))
    out["copy_streams"] = {st: {"copies": len(v), "busy_frac": union(v) / win} for st, v in sorted(per.items())}
    other = [x for x in kern if x not in sten]
    out["other_kernels"] = sorted({x[4][:60] for x in other})
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace_dirs", nargs="+")
    ap.add_argument("--window", type=float, default=0.6, help="last fraction of the trace to summarise")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = {d: summarize(d, a.window) for d in a.trace_dirs}
    for d, r in res.items():
        if not r:
            print(f"{d}: no trace")
            continue
        print(f"{d}: window {r['window_us']:.0f} us, {r['stencil_launches']} stencil launches "
              f"p50 {r['stencil_p50_us']} p90 {r['stencil_p90_us']} us busy {r['stencil_busy_frac']:.2f}; "
              f"{r['copies']} copies p50 {r['copy_p50_us']} p90 {r['copy_p90_us']} us busy {r['copy_busy_frac']:.2f}")
        for qu, v in r["queues"].items():
            print(f"   queue {qu}: {v['launches']} launches p50 {v['p50_us']} p90 {v['p90_us']} busy {v['busy_frac']:.2f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
