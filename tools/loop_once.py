#!/usr/bin/env python3
"""Run one device-resident loop (for profilers): W H channels reps fuse iters.
Environment knobs of the kernels apply (PCONV_SWAR_SHAPE, PCONV_PREFETCH, ...)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pconv  # noqa: E402

w, h, ch, reps, fuse, iters = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5]),
                               int(sys.argv[6]))
img = pconv.synthetic_image(w, h, ch, seed=1)
eng = pconv.Engine(w, h, ch, fuse=fuse)
eng._eng.upload(np.ascontiguousarray(img).reshape(-1), 0, h)
for _ in range(iters):
    eng._eng.run(reps)
eng._eng.synchronize()
print("tuned:", pconv.native.swar_tuned())
