#!/usr/bin/env python3
"""Round 5: the SWAR step forms timed against each other on the production
launch geometries (one barrier per step pair).

For each loop (headline 1920x2520 RGB x40, rank 3 of the 8-way split,
32768^2 grey x24) the tuner's pick (shape, kernel) is taken, then the loop is
timed with each step form forced on that pick:
  form 0: one barrier per step, truncating every step;
  form 1: steps in pairs with a x16 intermediate (2 barriers per pair);
Prints one JSON line per (loop, form): us per repetition (best of --repeat).
A third form (ONE barrier per pair: two boundary rows per side, ghost rows
recomputed) was timed too (profiles/r05/d/form_ab.jsonl), never won, and was
removed from the kernels; set_swar_alt now clamps to 0 / 1.
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
       "grey32768": (32768, 32768, "grey", 24, 12, 1, 0, 12)}


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
    p.add_argument("--which", default="headline,band8,grey32768")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--repeat", type=int, default=3)
    a = p.parse_args()
    n = pconv.native
    for which in a.which.split(","):
        n.clear_swar_tuning()
        n.set_autotune(True)
        n.set_swar_alt(-1)
        n.set_prefetch_mode(-1)
        n.set_swar_shape(0, 0, 0)
        tuned_us = loop_us(n, which, a.iters if which != "grey32768" else 3, a.repeat)
        fuse = CFG[which][4]
        t = [(k, s) for k, s in n.swar_tuned() if k[1] == fuse]
        k, s = max(t, key=lambda e: e[0][2])
        print(json.dumps({"loop": which, "form": "tuned", "pick": {"shape": list(s), "form": int(k[4]),
                          "pf": int(k[5])}, "us_per_rep": round(tuned_us, 3)}), flush=True)
        n.set_autotune(False)
        n.set_swar_shape(*s)
        n.set_prefetch_mode(int(k[5]))
        for form in (0, 1):
            n.set_swar_alt(form)
            us = loop_us(n, which, a.iters if which != "grey32768" else 3, a.repeat)
            print(json.dumps({"loop": which, "form": form, "shape": list(s), "pf": int(k[5]),
                              "us_per_rep": round(us, 3)}), flush=True)
    n.set_swar_alt(-1)
    n.set_prefetch_mode(-1)
    n.set_swar_shape(0, 0, 0)
    n.set_autotune(True)


if __name__ == "__main__":
    main()
