"""Tile-shape x fuse sweep of the SWAR temporal kernel on the row band one
rank of a WORLD-way split computes (null transport: the band's own schedule,
timed on one GPU).  One process; shapes switched with set_swar_shape.

python tools/band_sweep.py [--worlds 1,2,4,8] [--fuse 4,8,12,16] [--channels rgb]
Prints one JSON line per (world, fuse, shape) with us_per_rep (best of rounds)
and the shape the latency model would pick ("auto").
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
    p.add_argument("--worlds", default="1,2,4,8")
    p.add_argument("--fuse", default="4,8,12,16")
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--shapes", default="all", help="all | auto | list of lw,m,nw separated by ';'")
    a = p.parse_args()
    import numpy as np

    import pconv

    n = pconv.native
    shapes = [tuple(s) if isinstance(s, (tuple, list)) else (s.lw, s.m, s.nw) for s in n.swar_shapes()]
    for world in [int(x) for x in a.worlds.split(",")]:
        rank = 1 if world > 1 else 0
        for f in [int(x) for x in a.fuse.split(",")]:
            halo = max(f, min(a.reps, 64, a.height // world)) if world > 1 else f
            e = n.BandEngine(a.width, a.height, a.channels, "gaussian", rank, world, 0, halo=halo, fuse=f,
                             variant="temporal")
            if world > 1:
                e.attach_null_transport()
            b = e.band
            img = pconv.synthetic_image(a.width, a.height, a.channels, seed=5)
            rows = img.reshape(a.height, -1)[b.y0:b.y0 + b.rows]
            e.upload(np.ascontiguousarray(rows).reshape(-1), 0, b.rows)
            e.synchronize()
            res = {}
            todo = [None] + shapes if a.shapes == "all" else [None] if a.shapes == "auto" else \
                [tuple(int(v) for v in x.split(",")) for x in a.shapes.split(";")]
            for sh in todo:
                try:
                    n.set_swar_shape(*(sh or (0, 0, 0)))
                    e.run(a.reps)
                    e.synchronize()
                except Exception as ex:  # shape cannot hold this fuse depth
                    res[sh] = None
                    continue
                best = 1e9
                for _ in range(a.rounds):
                    t0 = time.perf_counter()
                    for _ in range(a.iters):
                        e.run(a.reps)
                    e.synchronize()
                    best = min(best, (time.perf_counter() - t0) / a.iters)
                res[sh] = best
            n.set_swar_shape(0, 0, 0)
            tuned = [list(k) + list(sh) for k, sh in n.swar_tuned() if k[1] == f and k[2] == b.rows + 0]
            for sh, t in res.items():
                print(json.dumps({"world": world, "band_rows": b.rows, "halo": halo, "fuse": f, "ch": a.channels,
                                  "shape": "auto" if sh is None else "%d,%d,%d" % sh,
                                  "launches": e.stats.launches,
                                  "tuned_keys": tuned,
                                  "us_per_rep": None if t is None else round(t / a.reps * 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
