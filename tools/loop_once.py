#!/usr/bin/env python3
"""Run one device-resident loop (for profilers): W H channels reps fuse iters.
The kernel choice is the tuner's; force one through the kernel setters
(pconv.native.set_swar_shape / set_prefetch_mode / set_swar_alt) in a copy
of this script (no environment variable changes the kernels)."""
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
