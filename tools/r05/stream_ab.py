#!/usr/bin/env python3
"""Round 5: the row-streaming kernel (kernels/stencil_stream.hip) against the
tile kernels on the production loops (the per-step
barrier and the vertical halo).

For each loop the device time per repetition (best of --repeat) with:
  tiles    the tuner choosing among the tile kernels only (set_stream_mode 0);
  chained  the row-streaming kernel forced, levels chained per row;
  skewed   the row-streaming kernel forced, levels skewed by one row;
  tuned    the tuner choosing among all of them (the default), with its pick.
One JSON line per (loop, variant).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import pconv  # noqa: E402

CFG = {"headline": (1920, 2520, "rgb", 40, 8, 1, 0, 8), "band8": (1920, 2520, "rgb", 40, 8, 8, 3, 40),
       "rgb8192": (8192, 8192, "rgb", 24, 8, 1, 0, 8), "grey32768": (32768, 32768, "grey", 24, 12, 1, 0, 12)}
MODES = {"tiles": 0, "chained": 1, "skewed": 2, "tuned": -1}


def loop_us(n, which, iters, repeat):
    import torch

    w, h, ch, reps, fuse, world, rank, halo = CFG[which]
    eng = n.BandEngine(w, h, ch, "gaussian", rank, world, 0, halo=halo, fuse=fuse, graph=True)
    b = eng.band
    img = np.empty(w * h * (3 if ch == "rgb" else 1), np.uint8)
    n.synth_rows(img, w, h, ch, 7, 0, h)
    rows = img.reshape(h, -1)
    lo, hi = (-min(halo, b.y0), b.rows + min(halo, h - b.y0 - b.rows)) if world > 1 else (0, b.rows)
    eng.upload(np.ascontiguousarray(rows[b.y0 + lo:b.y0 + hi]).reshape(-1), lo, hi)
    best = 1e30
    for r in range(repeat + 1):
        eng.synchronize()
        t = time.perf_counter()
        for _ in range(iters):
            eng.set_halo_valid(world > 1)
            eng.run(reps)
        eng.synchronize()
        torch.cuda.synchronize()
        if r:
            best = min(best, (time.perf_counter() - t) / iters / reps * 1e6)
    del eng
    return best


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--which", default="headline,band8,rgb8192,grey32768")
    p.add_argument("--variants", default="tiles,chained,skewed,tuned")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--repeat", type=int, default=3)
    a = p.parse_args()
    n = pconv.native
    try:
        for which in a.which.split(","):
            iters = a.iters if which in ("headline", "band8") else 3
            for v in a.variants.split(","):
                n.clear_swar_tuning()
                n.set_stream_mode(MODES[v])
                us = loop_us(n, which, iters, a.repeat)
                rec = {"loop": which, "variant": v, "us_per_rep": round(us, 3)}
                if v in ("tiles", "tuned"):
                    fuse = CFG[which][4]
                    t = [(k, s) for k, s in n.swar_tuned() if k[1] == fuse]
                    if t:
                        k, s = max(t, key=lambda e: e[0][2])
                        rec["pick"] = {"shape": list(s), "form": int(k[4]), "kernel": int(k[5])}
                print(json.dumps(rec), flush=True)
    finally:
        n.set_stream_mode(-1)
        n.clear_swar_tuning()


if __name__ == "__main__":
    main()
