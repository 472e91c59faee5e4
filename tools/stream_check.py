#!/usr/bin/env python3
"""Row-streaming temporal kernel: bit-exactness against the NumPy oracle and
loop timing against the tile kernel (run on the GPU box).

  python tools/stream_check.py [--check-only] [--time-only]
Correctness: stream mode forced (every launch with 8/16 steps uses it), both
step forms, grey/RGB/RGBA, odd sizes, multi-launch schedules.  Timing: device
loop of the same schedule with the streaming kernel off / forced / tuned.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def check(n, pconv, np):
    rng = np.random.default_rng(7)
    cases = [((300, 500), "grey", 8, 8), ((257, 1000), "rgb", 20, 8), ((190, 333), "rgba", 16, 8),
             ((64, 64), "grey", 24, 8), ((513, 700), "grey", 32, 16), ((200, 901), "rgb", 16, 16),
             ((1, 77), "grey", 8, 8), ((37, 5), "rgb", 8, 8), ((600, 1920), "rgb", 40, 8)]
    bad_total = 0
    for (h, w), ch, reps, fuse in cases:
        c = {"grey": 1, "rgb": 3, "rgba": 4}[ch]
        img = rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)
        ref = pconv.numpy_convolve(img, reps)
        for alt in (0, 1):
            n.set_swar_alt(alt)
            n.clear_swar_tuning()
            eng = pconv.Engine(w, h, ch, fuse=fuse)
            out = eng.run_numpy(img, reps)
            bad = int(np.count_nonzero(out != ref))
            tuned = n.swar_tuned()
            streamed = any(k[5] > 0 for k, _ in tuned)
            print(json.dumps({"check": f"{h}x{w}x{c}", "reps": reps, "fuse": fuse, "alt": alt, "bad": bad,
                              "stream_used": streamed, "tuned": [list(k) for k, _ in tuned]}), flush=True)
            bad_total += bad
    n.set_swar_alt(-1)
    return bad_total


def timing(n, pconv, np, w, h, ch, reps, iters):
    img = pconv.synthetic_image(w, h, ch, seed=1)
    res = {}
    for label, mode in (("tile", 0), ("stream", 1), ("tuned", -1)):
        n.set_stream_mode(mode)
        n.clear_swar_tuning()
        eng = pconv.Engine(w, h, ch, fuse=8)
        eng._eng.upload(np.ascontiguousarray(img).reshape(-1), 0, h)
        eng._eng.run(reps)
        eng._eng.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            eng._eng.run(reps)
        eng._eng.synchronize()
        dt = (time.perf_counter() - t0) / iters
        res[label] = round(dt / reps * 1e6, 2)
        res[label + "_tuned"] = [list(k) + list(v) for k, v in n.swar_tuned()]
        del eng
    n.set_stream_mode(-1)
    print(json.dumps({"time": f"{w}x{h} {ch}", "reps": reps, "us_per_rep": res}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--check-only", action="store_true")
    p.add_argument("--time-only", action="store_true")
    a = p.parse_args()
    import numpy as np

    import pconv

    n = pconv.native
    if not a.time_only:
        n.set_stream_mode(1)
        bad = check(n, pconv, np)
        n.set_stream_mode(-1)
        print(json.dumps({"check_total_bad": bad}), flush=True)
        if bad:
            return 1
    if not a.check_only:
        timing(n, pconv, np, 32768, 32768, "grey", 16, 5)
        timing(n, pconv, np, 16384, 16384, "grey", 16, 10)
        timing(n, pconv, np, 8192, 8192, "rgb", 16, 10)
        timing(n, pconv, np, 1920, 2520, "rgb", 40, 50)
    return 0


if __name__ == "__main__":
    sys.exit(main())
