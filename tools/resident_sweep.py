#!/usr/bin/env python3
"""Device-resident loop time of the register-resident kernel against the tile
kernel (tuned shapes, `fuse` steps per launch) on single-band frames.

python tools/resident_sweep.py [--frames 1920x2520:rgb,1920x2520:grey] [--reps 40]
One JSON line per (frame, path): us_per_rep (best of rounds), launches.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", default="1920x2520:rgb,1920x2520:grey,1920x630:grey,1920x1260:rgb,1920x5040:grey")
    p.add_argument("--reps", default="40", help="comma-separated repetition counts")
    p.add_argument("--paths", default="tile,resident")
    p.add_argument("--fuse", type=int, default=8)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    import pconv

    n = pconv.native
    for spec in a.frames.split(","):
        dims, ch = spec.split(":")
        w, h = (int(x) for x in dims.split("x"))
        img = pconv.synthetic_image(w, h, ch, seed=9)
        for resident, reps in [(r, int(x)) for r in (False, True) if ("resident" if r else "tile") in a.paths
                               for x in a.reps.split(",")]:
            e = n.BandEngine(w, h, ch, "gaussian", 0, 1, 0, halo=a.fuse, fuse=a.fuse, variant="temporal",
                             resident=resident)
            e.upload(img.reshape(-1), 0, h)
            e.run(reps)  # warm: code objects, tuning
            e.synchronize()
            best = 1e9
            for _ in range(a.rounds):
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    e.run(reps)
                e.synchronize()
                best = min(best, (time.perf_counter() - t0) / a.iters)
            print(json.dumps({"frame": spec, "reps": reps, "fuse": a.fuse, "path": "resident" if resident else "tile",
                              "launches": e.stats.launches, "us_per_rep": round(best / reps * 1e6, 3),
                              "ms_per_loop": round(best * 1e3, 4)}), flush=True)


if __name__ == "__main__":
    main()
