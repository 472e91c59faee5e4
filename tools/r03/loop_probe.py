#!/usr/bin/env python3
"""Device loop of the headline frame and of an emulated 8-way band: the
tuner's pick and the loop time per repetition (rep-loop graph, 40 reps per
run).  Run with and without PCONV_TUNE_CANDIDATES to A/B the model's
candidate ranking."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import pconv  # noqa: E402

n = pconv.native
reps = 40
# default: the headline frame, its 8-way band and its 2-way band; --large adds
# the large BASELINE frames (1 GPU: 8192^2 RGB, 16384^2 and 32768^2 grey at
# their auto fuse)
CONFIGS = [(1920, 2520, "rgb", 1, 0, 8), (1920, 2520, "rgb", 8, 3, 8), (1920, 2520, "rgb", 2, 0, 8)]
if "--large" in sys.argv:
    CONFIGS += [(8192, 8192, "rgb", 1, 0, 8), (16384, 16384, "grey", 1, 0, 12), (32768, 32768, "grey", 1, 0, 12)]
for (w, h, ch, world, rank, fuse) in CONFIGS:
    n.clear_swar_tuning()
    halo = fuse if world == 1 else 40
    eng = n.BandEngine(w, h, ch, "gaussian", rank, world, 0, halo=halo, fuse=fuse, graph=True)
    b = eng.band
    img = np.empty(w * h * (3 if ch == "rgb" else 1), np.uint8)
    n.synth_rows(img, w, h, ch, 7, 0, h)
    rows = img.reshape(h, -1)
    lo, hi = (-min(halo, b.y0), b.rows + min(halo, h - b.y0 - b.rows)) if world > 1 else (0, b.rows)
    eng.upload(np.ascontiguousarray(rows[b.y0 + lo:b.y0 + hi]).reshape(-1), lo, hi)
    for _ in range(3):
        eng.set_halo_valid(world > 1)
        eng.run(reps)
    eng.synchronize()
    k = max(3, min(200, int(2e11 // (w * h * (3 if ch == "rgb" else 1) * reps))))
    t0 = time.perf_counter()
    for _ in range(k):
        eng.set_halo_valid(world > 1)
        eng.run(reps)
    eng.synchronize()
    us = (time.perf_counter() - t0) / k * 1e6
    print(json.dumps({"frame": f"{w}x{h} {ch}", "world": world, "rank": rank,
                      "candidates": os.environ.get("PCONV_TUNE_CANDIDATES", "6 (default)"),
                      "loop_us": round(us, 2), "us_per_rep": round(us / reps, 3),
                      "tuned": [[list(k_), list(s)] for k_, s in n.swar_tuned()]}), flush=True)
