#!/usr/bin/env python3
"""Round 5: head streaming against whole-image step graphs, per band size and
burst length (the streamed head's copies on the slots'
streams vs the burst behind it; the stream_min_bytes threshold).

For the headline image (1920x2520 RGB, 40 reps) as one band (N=1) and as the
pre-loaded bands of a 2-, 4- and 8-way split, one pipeline of 4 slots per
mode:
  graph       stream_chunks 0 (every image one step graph);
  head_slots  stream_chunks 4, the head's copies on the slots' streams;
  head_pool   stream_chunks 4, the head's copies on two pool streams.
Each burst (B images submitted to an idle pipeline, then drained) is timed
R times; one JSON line per (band, mode, B) with the median and the spread in
ms.  B = 1 is the single-image latency.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

MODES = {"graph": dict(stream_chunks=0), "head_slots": dict(stream_chunks=4, head_on_slot_streams=True),
         "head_pool": dict(stream_chunks=4, head_on_slot_streams=False)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--bands", default="1:0,2:0,4:1,8:3")
    p.add_argument("--modes", default="graph,head_slots,head_pool")
    p.add_argument("--bursts", default="1,4,8")
    p.add_argument("--repeat", type=int, default=25)
    p.add_argument("--slots", type=int, default=4)
    a = p.parse_args()
    import pconv  # noqa: F401
    from pconv.parallel.dist_engine import DistributedBlur

    w, h, reps = 1920, 2520, 40
    img = np.random.default_rng(5).integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    for band in a.bands.split(","):
        world, rank = (int(x) for x in band.split(":"))
        for mode in a.modes.split(","):
            kw = dict(MODES[mode])
            if world > 1:
                kw.update(rank=rank, world=world, preload_halo=True, transport="none")
            b = DistributedBlur(w, h, "rgb", "gaussian", reps, device=0, slots=a.slots, **kw)
            b.load_image(img)
            for _ in range(3):  # warm: captures, tuning
                for _ in range(a.slots):
                    b.submit(reps)
                b.drain()
            for burst in (int(x) for x in a.bursts.split(",")):
                t = []
                for _ in range(a.repeat):
                    t0 = time.perf_counter()
                    for _ in range(burst):
                        b.submit(reps)
                    b.drain()
                    t.append((time.perf_counter() - t0) * 1e3)
                print(json.dumps({"band": band, "mode": mode, "burst": burst, "slots": a.slots,
                                  "h2d_bytes": b.h2d_bytes_per_image, "median_ms": round(statistics.median(t), 4),
                                  "min_ms": round(min(t), 4), "max_ms": round(max(t), 4)}), flush=True)
            del b


if __name__ == "__main__":
    main()
