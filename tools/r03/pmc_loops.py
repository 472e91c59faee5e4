#!/usr/bin/env python3
"""Device loops for counter collection (run under rocprofv3 --pmc).

  headline  1920x2520 RGB, 40 reps, fuse 8: the bench's loop_only
  band8     rank 3 of an 8-way split of the same frame, 40-row ghost zones
            (halo 40): the per-rank loop of the N=8 pipeline
  grey32768 32768x32768 grey, 24 reps, fuse 12 (two launches per run): the
            large-frame loop of the BASELINE 32768^2 config

The first run tunes (its candidate launches show up as other kernels); the
production kernel is the one launched `iters` x 5 times afterwards.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import pconv  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("which", choices=["headline", "band8", "grey32768"])
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args()
    n = pconv.native
    w, h, ch, reps, fuse = 1920, 2520, "rgb", 40, 8
    world, rank, halo = (1, 0, 8) if a.which == "headline" else (8, 3, 40)
    if a.which == "grey32768":
        w, h, ch, reps, fuse, halo, world, rank = 32768, 32768, "grey", 24, 12, 12, 1, 0
    eng = n.BandEngine(w, h, ch, "gaussian", rank, world, 0, halo=halo, fuse=fuse, graph=True)
    b = eng.band
    img = np.empty(w * h * (3 if ch == "rgb" else 1), np.uint8)
    n.synth_rows(img, w, h, ch, 7, 0, h)
    rows = img.reshape(h, -1)
    lo, hi = (-min(halo, b.y0), b.rows + min(halo, h - b.y0 - b.rows)) if world > 1 else (0, b.rows)
    eng.upload(np.ascontiguousarray(rows[b.y0 + lo:b.y0 + hi]).reshape(-1), lo, hi)
    for _ in range(a.iters + 1):
        eng.set_halo_valid(world > 1)
        eng.run(reps)
    eng.synchronize()
    print(a.which, "tuned:", n.swar_tuned(), flush=True)


if __name__ == "__main__":
    main()
