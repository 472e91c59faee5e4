"""Device-resident loop timing sweep over kernel variants / fuse depths.

python tools/kernel_sweep.py [--width W --height H --channels C --reps R]
                             [--fuse 1,4,8] [--variants auto,temporal_pk]
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
    p.add_argument("--variants", default="auto")
    p.add_argument("--world", type=int, default=1, help="time the band of rank --rank of a WORLD-way split")
    p.add_argument("--rank", type=int, default=0)
    a = p.parse_args()
    import numpy as np

    import pconv

    n = pconv.native
    img = pconv.synthetic_image(a.width, a.height, a.channels, seed=3)
    small = a.width * a.height <= 1 << 23 and a.world == 1
    ref = pconv.numpy_convolve(img, a.reps) if small else None
    engines = {}
    for v in a.variants.split(","):
        for f in [int(x) for x in a.fuse.split(",")]:
            if f > 1 and not n.supports_fusion("gaussian", v):
                continue
            halo = max(f, min(a.reps, 64, a.height // a.world)) if a.world > 1 else f
            e = n.BandEngine(a.width, a.height, a.channels, "gaussian", a.rank, a.world, 0, halo=halo, fuse=f,
                             graph=a.graph, variant=v)
            if a.world > 1:
                e.attach_null_transport()  # timing only: the band's compute schedule without peers
            b = e.band
            rows = img.reshape(a.height, -1)[b.y0 : b.y0 + b.rows]
            e.upload(np.ascontiguousarray(rows).reshape(-1), 0, b.rows)
            ok = None
            if ref is not None:
                e.run(a.reps)
                out = np.empty_like(img)
                e.download(out.reshape(-1), 0, a.height)
                e.synchronize()
                ok = bool(np.array_equal(out, ref))
            engines[(v, f)] = (e, ok)
    res = {k: [] for k in engines}
    for _ in range(a.rounds):
        for k, (e, _) in engines.items():
            e.run(a.reps)
            e.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                e.run(a.reps)
            e.synchronize()
            res[k].append((time.perf_counter() - t0) / a.iters)
    for (v, f), (e, ok) in engines.items():
        best = min(res[(v, f)])
        px = e.band.rows * a.width
        print(json.dumps({"w": a.width, "h": a.height, "band_rows": e.band.rows, "ch": a.channels, "reps": a.reps,
                          "variant": v, "fuse": f, "graph": a.graph, "launches": e.stats.launches,
                          "us_per_rep": round(best / a.reps * 1e6, 3), "ms_per_run": round(best * 1e3, 4),
                          "gpix_per_s": round(px * a.reps / best / 1e9, 2), "correct": ok}), flush=True)


if __name__ == "__main__":
    main()
