#!/usr/bin/env python3
"""Float temporal kernel sweep: tile shape (PCONV_FLOAT_SHAPE) x repetitions per
launch for the float filters on the BASELINE frames; device loop time per
repetition (rep-loop graph, 40 reps per run), every configuration checked
against the native OpenMP oracle once.  One JSON line per point."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import pconv  # noqa: E402

n = pconv.native
frames = [(1920, 2520, "rgb"), (1920, 2520, "grey"), (8192, 8192, "rgb")]
if len(sys.argv) > 1 and sys.argv[1] == "quick":
    frames = frames[:1]
shapes = ["16,8", "8,8", "16,4", "8,4", "4,8", ""]
reps = 40
for (w, h, ch) in frames:
    c = {"grey": 1, "rgb": 3}[ch]
    img = np.empty(w * h * c, np.uint8)
    n.synth_rows(img, w, h, ch, 5, 0, h)
    for filt in ("box", "edge"):
        ref = np.empty_like(img)
        n.cpu_convolve(img, ref, w, h, ch, reps, pconv.get_filter(filt).to_native(), True, 0)
        for fuse in (2, 3, 4, 6, 8):
            for sh in shapes:
                if sh:
                    os.environ["PCONV_FLOAT_SHAPE"] = sh
                else:
                    os.environ.pop("PCONV_FLOAT_SHAPE", None)
                eng = n.BandEngine(w, h, ch, filt, 0, 1, 0, halo=fuse, fuse=fuse, graph=True)
                eng.upload(img, 0, h)
                eng.run(reps)
                eng.synchronize()
                out = np.empty_like(img)
                eng.download(out, 0, h)
                eng.synchronize()
                bad = int(np.count_nonzero(out != ref))
                k = 10 if w * h < 10_000_000 else 3
                eng.synchronize()
                t0 = time.perf_counter()
                for _ in range(k):
                    eng.run(reps)
                eng.synchronize()
                us = (time.perf_counter() - t0) / (k * reps) * 1e6
                print(json.dumps({"w": w, "h": h, "ch": ch, "filter": filt, "fuse": fuse, "shape": sh or "auto",
                                  "us_per_rep": round(us, 3), "mismatches": bad}), flush=True)
                del eng
