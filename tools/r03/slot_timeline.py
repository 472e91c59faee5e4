#!/usr/bin/env python3
"""Busy fractions of a pipelined run from a rocprofv3 trace (CPU only).

Reads <dir>/run_kernel_trace.csv and run_memory_copy_trace.csv, keeps the
last --tail fraction of the pipelined burst (the timed steady state) and reports, per
class of work (H2D copies, D2H copies, stencil kernels, RCCL kernels), the
count, the mean duration and the fraction of the window in which at least one
was running, plus how much of the RCCL time overlapped a stencil kernel and
the mean gap between consecutive stencil launches of one stream.  Tells which
engine sets the period of the slot pipeline (docs/PERFORMANCE.md §2).
"""
from __future__ import annotations

import argparse
import csv
import os
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            t += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


def classify_kernel(name: str) -> str:
    low = name.lower()
    if "nccl" in low or "rccl" in low:
        return "rccl"
    if any(t in name for t in ("k_swar", "k_stream", "k_binomial", "k_float", "k_generic", "k_mfma")):
        return "stencil"
    return "other"


def analyse(d: str, tail: float):
    ev = []  # (start, end, class, stream)
    for k in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), classify_kernel(k["Kernel_Name"]),
                   k["Stream_Id"]))
    mc = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(mc):
        for c in csv.DictReader(open(mc)):
            kind = {"MEMORY_COPY_HOST_TO_DEVICE": "h2d", "MEMORY_COPY_DEVICE_TO_HOST": "d2h"}.get(c["Direction"], "d2d")
            ev.append((int(c["Start_Timestamp"]), int(c["End_Timestamp"]), kind, c["Stream_Id"]))
    ev.sort()
    # Copies between pinned host buffers and the device are traced as
    # DEVICE_TO_DEVICE: label them by their place in their stream (an upload
    # precedes that stream's next kernel, a download follows a kernel).
    per = defaultdict(list)
    for i, x in enumerate(ev):
        per[x[3]].append(i)
    for st, idx in per.items():
        for j, i in enumerate(idx):
            if ev[i][2] != "d2d":
                continue
            prev = ev[idx[j - 1]][2] if j else None
            nxt = ev[idx[j + 1]][2] if j + 1 < len(idx) else None
            if nxt in ("stencil", "rccl"):
                ev[i] = ev[i][:2] + ("h2d",) + ev[i][3:]
            elif prev in ("stencil", "rccl"):
                ev[i] = ev[i][:2] + ("d2h",) + ev[i][3:]
    # The pipelined run is the burst (events < 2 ms apart) holding the most
    # copies; its last `tail` fraction is the steady state.
    segs, cur = [], [ev[0]]
    for x in ev[1:]:
        if x[0] - cur[-1][0] > 2_000_000:
            segs.append(cur)
            cur = []
        cur.append(x)
    segs.append(cur)
    seg = max(segs, key=lambda g: sum(1 for x in g if x[2] in ("h2d", "d2h", "d2d")))
    t_end = max(e for _, e, _, _ in seg)
    t_beg = min(s for s, _, _, _ in seg)
    t0 = t_end - (t_end - t_beg) * tail
    win = [x for x in seg if x[0] >= t0]
    span = max(e for _, e, _, _ in win) - min(s for s, _, _, _ in win)
    by = defaultdict(list)
    for s, e, c, st in win:
        by[c].append((s, e, st))
    rows = []
    unions = {}
    for c in ("h2d", "d2h", "d2d", "stencil", "rccl", "other"):
        if not by[c]:
            continue
        u = union([(s, e) for s, e, _ in by[c]])
        unions[c] = u
        rows.append((c, len(by[c]), sum(e - s for s, e, _ in by[c]) / len(by[c]) / 1e3, total(u) / span))
    out = [f"# slot timeline: {d}", "", f"window: last {tail:.0%} of the run, {span / 1e3:.1f} us", "",
           "| class | count | mean us | busy fraction |", "|---|---|---|---|"]
    out += [f"| {c} | {n} | {m:.2f} | {f:.3f} |" for c, n, m, f in rows]
    if "stencil" in unions:
        comp = union(unions["stencil"] + unions.get("rccl", []))
        out += ["", f"compute busy (stencil or RCCL kernel running): {total(comp) / span:.3f}"]
        if "rccl" in unions:
            ov = intersect(unions["rccl"], unions["stencil"])
            out.append(f"RCCL time overlapping a stencil kernel: {ov / max(1, total(unions['rccl'])):.3f}")
        gaps = []
        per_stream = defaultdict(list)
        for s, e, st in by["stencil"]:
            per_stream[st].append((s, e))
        for st, iv in per_stream.items():
            iv.sort()
            gaps += [b[0] - a[1] for a, b in zip(iv, iv[1:]) if 0 <= b[0] - a[1] < 20_000]
        if gaps:
            out.append(f"gap between consecutive stencil launches of one stream (< 20 us): mean "
                       f"{sum(gaps) / len(gaps) / 1e3:.2f} us over {len(gaps)}")
    if by["h2d"]:
        out.append(f"period per H2D copy: {span / len(by['h2d']) / 1e3:.2f} us")
    return "\n".join(out)


def main():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("trace_dir")
    p.add_argument("--tail", type=float, default=0.5)
    p.add_argument("--md", default=None)
    a = p.parse_args()
    text = analyse(a.trace_dir, a.tail)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
