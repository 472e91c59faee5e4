#!/usr/bin/env python3
"""One gaussian step on a 32768^2 grey frame: the MFMA prototype
(kernels/stencil_mfma.hip) against the single-step VALU kernel (k_binomial)
and the SWAR kernel (1 step, and 12 fused steps per launch = the production
per-repetition cost).  Device time per step from hipEvents on the stream;
`--iters` launches per variant (rocprofv3 counter passes use few)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pconv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=32768)
p.add_argument("--iters", type=int, default=20)
p.add_argument("--variants", default="mfma,binomial,temporal1,temporal12")
a = p.parse_args()
n = pconv.native
w = h = a.size
halo = 12
lay = n.frame_layout(w, h, halo)
src = torch.zeros(lay["bytes"], dtype=torch.uint8, device="cuda")
dst = torch.zeros_like(src)
v = src.view(h + 2 * halo, lay["pitch"])
v[halo:halo + h, 16:16 + w] = torch.randint(0, 256, (h, w), dtype=torch.uint8, device="cuda")
base = lay["pitch"] * halo + 16
s = torch.cuda.current_stream()


def launch(variant, steps):
    n.launch_stencil("gaussian", "grey", src.data_ptr() + base, dst.data_ptr() + base, lay["pitch"], w, 0, h, -halo,
                     h + halo, steps, 0, h, s.cuda_stream, variant)


ref = None
for name in a.variants.split(","):
    variant, steps = {"mfma": ("mfma", 1), "binomial": ("binomial", 1), "temporal1": ("temporal", 1),
                      "temporal12": ("temporal", 12)}[name]
    launch(variant, steps)  # warm (+ tuning)
    torch.cuda.synchronize()
    if steps == 1:
        out = dst.view(h + 2 * halo, lay["pitch"])[halo:halo + h, 16:16 + w].clone()
        if ref is None:
            ref = out
        bad = int((out != ref).sum().item())
    else:
        bad = None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        launch(variant, steps)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    print(json.dumps({"variant": name, "size": a.size, "us_per_launch": round(us, 2),
                      "us_per_step": round(us / steps, 2), "mismatches_vs_first": bad}), flush=True)
