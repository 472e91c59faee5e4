"""Device-resident loop timing sweep over kernel variants / fuse depths.

python tools/kernel_sweep.py [--width W --height H --channels C --reps R]
Prints one JSON line per configuration: us per repetition (host wall clock
around `iters` back-to-back runs of `reps` repetitions, device synchronised).
Interleaves configurations round-robin so DVFS / noise hits all of them.
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
    p.add_argument("--height", type=int, default=2520)
    p.add_argument("--channels", default="rgb")
    p.add_argument("--reps", type=int, default=40)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--fuse", default="1,2,4,8,12,16")
    p.add_argument("--graph", action="store_true")
    a = p.parse_args()
    import numpy as np

    import pconv

    n = pconv.native
    img = pconv.synthetic_image(a.width, a.height, a.channels, seed=3)
    ref = None
    engines = {}
    for f in [int(x) for x in a.fuse.split(",")]:
        e = n.BandEngine(a.width, a.height, a.channels, "gaussian", 0, 1, 0, halo=f, fuse=f, graph=a.graph)
        e.upload(img.reshape(-1), 0, a.height)
        e.run(a.reps)
        out = np.empty_like(img)
        e.download(out.reshape(-1), 0, a.height)
        e.synchronize()
        if ref is None:
            ref = pconv.numpy_convolve(img, a.reps) if a.width * a.height <= 1 << 23 else out
        ok = bool(np.array_equal(out, ref))
        engines[f] = (e, ok)
    res = {f: [] for f in engines}
    for _ in range(a.rounds):
        for f, (e, _) in engines.items():
            e.run(a.reps)
            e.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                e.run(a.reps)
            e.synchronize()
            res[f].append((time.perf_counter() - t0) / a.iters)
    for f, (e, ok) in engines.items():
        best = min(res[f])
        print(json.dumps({"w": a.width, "h": a.height, "ch": a.channels, "reps": a.reps, "fuse": f,
                          "graph": a.graph, "launches": e.stats.launches, "us_per_rep": round(best / a.reps * 1e6, 3),
                          "ms_per_run": round(best * 1e3, 4),
                          "gpix_per_s": round(a.width * a.height * a.reps / best / 1e9, 2), "correct": ok}),
              flush=True)


if __name__ == "__main__":
    main()
