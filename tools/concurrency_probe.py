"""Do independent small-band rep loops overlap on one GPU?

K BandEngines (each with its own compute stream) run `reps` repetitions of a
HxW image back to back; reports aggregate us per image for K = 1..4.  If the
aggregate time per image falls with K, small bands leave the GPU idle and
images in flight should compute concurrently.
python tools/concurrency_probe.py [--height 315] [--iters 50]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=315)
    p.add_argument("--channels", default="rgb")
    p.add_argument("--reps", type=int, default=40)
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--kmax", type=int, default=4)
    a = p.parse_args()
    import numpy as np

    import pconv

    n = pconv.native
    img = pconv.synthetic_image(a.width, a.height, a.channels, seed=2)
    engines = []
    for _ in range(a.kmax):
        e = n.BandEngine(a.width, a.height, a.channels, "gaussian", 0, 1, 0, halo=8, fuse=8)
        e.upload(np.ascontiguousarray(img).reshape(-1), 0, a.height)
        e.synchronize()
        engines.append(e)
    for k in range(1, a.kmax + 1):
        es = engines[:k]
        for e in es:
            e.run(a.reps)
        for e in es:
            e.synchronize()
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(a.iters):
                for e in es:
                    e.run(a.reps)
            for e in es:
                e.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"h": a.height, "k": k, "us_per_image": round(best / (a.iters * k) * 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
