#!/usr/bin/env python3
"""Device loops for counter collection (run under rocprofv3 --pmc), round 5.

  headline  1920x2520 RGB, 40 reps, fuse 8 (the bench's loop_only)
  band8     rank 3 of an 8-way split of the same frame, 40-row ghost zones
  grey32768 32768x32768 grey, 24 reps, fuse 12 (two launches per run)

--pick: tune (no profiler) and print the chosen {shape, form, pf} as JSON.
Otherwise the choice given by --shape/--form/--pf is forced through the
kernel setters (no environment variables), so every counter pass counts the
same production kernel.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import pconv  # noqa: E402

CFG = {"headline": (1920, 2520, "rgb", 40, 8, 1, 0, 8), "band8": (1920, 2520, "rgb", 40, 8, 8, 3, 40),
       "grey32768": (32768, 32768, "grey", 24, 12, 1, 0, 12)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("which", choices=sorted(CFG))
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--pick", action="store_true")
    p.add_argument("--shape", default=None)
    p.add_argument("--form", type=int, default=-1)
    p.add_argument("--pf", type=int, default=-1)
    a = p.parse_args()
    n = pconv.native
    w, h, ch, reps, fuse, world, rank, halo = CFG[a.which]
    if not a.pick:
        if a.shape:
            n.set_swar_shape(*[int(x) for x in a.shape.split(",")])
        n.set_swar_alt(a.form)
        n.set_prefetch_mode(a.pf)
        n.set_autotune(False)
    eng = n.BandEngine(w, h, ch, "gaussian", rank, world, 0, halo=halo, fuse=fuse, graph=True)
    b = eng.band
    img = np.empty(w * h * (3 if ch == "rgb" else 1), np.uint8)
    n.synth_rows(img, w, h, ch, 7, 0, h)
    rows = img.reshape(h, -1)
    lo, hi = (-min(halo, b.y0), b.rows + min(halo, h - b.y0 - b.rows)) if world > 1 else (0, b.rows)
    eng.upload(np.ascontiguousarray(rows[b.y0 + lo:b.y0 + hi]).reshape(-1), lo, hi)
    for _ in range((1 if a.pick else a.iters) + 1):
        eng.set_halo_valid(world > 1)
        eng.run(reps)
    eng.synchronize()
    if a.pick:
        # the full-fuse launch's entry: the tuned key with steps == fuse
        t = [(k, s) for k, s in n.swar_tuned() if k[1] == fuse]
        k, s = max(t, key=lambda e: e[0][2])  # most rows: the main launch
        print(json.dumps({"shape": f"{s[0]},{s[1]},{s[2]}", "form": int(k[4]), "pf": int(k[5]),
                          "key": list(k)}), flush=True)
    else:
        print(a.which, "forced:", a.shape, a.form, a.pf, flush=True)


if __name__ == "__main__":
    main()
