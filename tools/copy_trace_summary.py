#!/usr/bin/env python3
"""Per-direction PCIe utilisation of the serving pipeline from a rocprofv3
--kernel-trace --memory-copy-trace of bench.py.

Inside the whole-step hipGraphs every copy is reported as
MEMORY_COPY_DEVICE_TO_DEVICE with source = destination = the GPU agent: the
pinned host buffers (hipHostMalloc) are mapped into the GPU's address space
and the graph's memcpy nodes run as agent-local SDMA copies, so the tracer
cannot tell the direction.  It is recovered from stream order: every image
runs on its slot's stream as H2D -> stencil launches -> D2H, so a copy that
follows a stencil launch on its stream is the D2H, any other the H2D.

Reports, over the last --images images: each direction's busy fraction of
the window (union of its copies), copy durations and rates, same-direction
overlap, and the step period.
"""
from __future__ import annotations

import argparse
import csv
import os


def union(iv):
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace_dir")
    ap.add_argument("--images", type=int, default=20)
    ap.add_argument("--skip-images", type=int, default=None,
                    help="images to skip on the slot streams (bench.py: its --warmup count, so that the window is "
                         "exactly the timed images); default: take the last --images images of the trace")
    ap.add_argument("--bytes", type=int, default=1920 * 2520 * 3)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    cp = list(csv.DictReader(open(os.path.join(a.trace_dir, "run_memory_copy_trace.csv"))))
    ks = list(csv.DictReader(open(os.path.join(a.trace_dir, "run_kernel_trace.csv"))))
    ev = [(int(c["Start_Timestamp"]), int(c["End_Timestamp"]), "c", c["Stream_Id"], c["Direction"]) for c in cp]
    ev += [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "k", k["Stream_Id"], "")
           for k in ks if "k_swar" in k["Kernel_Name"] or "k_binomial" in k["Kernel_Name"]]
    ev.sort()
    last, copies = {}, []
    for s, e, t, st, lab in ev:
        if t == "c":
            copies.append((s, e, "D2H" if last.get(st) == "k" else "H2D", st, lab))
        last[st] = t
    # only the copies of streams that also ran stencil launches (the pipeline's
    # slot streams; bench.py's copy-floor probe runs on another stream)
    slot_streams = {st for _, _, t, st, _ in ev if t == "k"}
    copies = [c for c in copies if c[3] in slot_streams]
    if a.skip_images is not None:
        copies = copies[2 * a.skip_images:2 * (a.skip_images + a.images)]
    else:
        copies = copies[-2 * a.images:]
    t0, t1 = min(c[0] for c in copies), max(c[1] for c in copies)
    win = (t1 - t0) / 1e3
    out = [f"# Copy trace of the serving pipeline: {a.trace_dir}", "",
           f"Labels in the trace: {sorted({c[4] for c in copies})} (direction recovered from stream order).", "",
           f"Window of {a.images} images{' after ' + str(a.skip_images) + ' skipped' if a.skip_images is not None else ' (the last)'}: {win:.0f} us = {win / a.images / 1e3:.3f} ms per image.", "",
           "| direction | copies | busy % of window | mean us | min us | max us | mean GB/s | same-direction overlaps |",
           "|---|---|---|---|---|---|---|---|"]
    for d in ("H2D", "D2H"):
        iv = [(c[0], c[1]) for c in copies if c[2] == d]
        if not iv:
            continue
        du = [(e - s) / 1e3 for s, e in iv]
        srt = sorted(iv)
        ov = sum(1 for i in range(1, len(srt)) if srt[i][0] < srt[i - 1][1])
        mean = sum(du) / len(du)
        out.append(f"| {d} | {len(iv)} | {100.0 * union(iv) / (t1 - t0):.1f} | {mean:.0f} | {min(du):.0f} | "
                   f"{max(du):.0f} | {a.bytes / (mean * 1e-6) / 1e9:.1f} | {ov} |")
    both = [(c[0], c[1]) for c in copies]
    out += ["", f"Some copy in flight {100.0 * union(both) / (t1 - t0):.1f} % of the window."]
    text = "\n".join(out)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
