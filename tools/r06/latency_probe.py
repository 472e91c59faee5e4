#!/usr/bin/env python3
"""One head-streamed headline image at a time (the `latency_ms` scope of
bench.py: submit to an idle pipeline, drain), N times, with a host
timestamp per image — run under rocprofv3 (kernel + memory-copy + HIP API
traces) to see where one image's 0.53 ms goes: each chunk copy's start
against the API call that issued it and the event it waited for.

    rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace \
        --output-format csv -d OUT -o lat -- python3 tools/r06/latency_probe.py
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=30)
    p.add_argument("--chunks", type=int, default=4)
    p.add_argument("--weights", default=None, help="streamed chunk weights, e.g. 3,4,4,5,5 (sets --chunks)")
    p.add_argument("--tune-candidates", type=int, default=None, help="shapes timed per launch geometry")
    p.add_argument("--fuse", type=int, default=None, help="reps per launch (default: the engine's pick)")
    p.add_argument("--trace", type=int, default=0, help="then this many images with chunk timing events")
    a = p.parse_args()
    import torch

    from pconv.parallel.dist_engine import DistributedBlur

    torch.cuda.set_device(0)
    if a.tune_candidates:
        import pconv
        pconv.native.set_tune_candidates(a.tune_candidates)
    blur = DistributedBlur(1920, 2520, "rgb", "gaussian", 40, rank=0, world=1, device=0, slots=4,
                           stream_chunks=a.chunks, fuse=a.fuse,
                           stream_weights=[int(x) for x in a.weights.split(",")] if a.weights else None)
    blur.load_synthetic(1234)
    for _ in range(5):
        blur.submit(40)
    blur.drain()
    lat = []
    for _ in range(a.images):
        t = time.perf_counter()
        blur.step(40)
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    out = {"latency_ms_median": round(lat[len(lat) // 2], 4), "min": round(lat[0], 4), "max": round(lat[-1], 4),
           "streamed_heads": int(blur.pipe.streamed_heads), "chunks": a.chunks, "fuse": a.fuse,
           "weights": a.weights,
           "tune_candidates": a.tune_candidates}
    if a.trace:
        # the same single images with chunk timing events (their own timing shifts slightly)
        for k in range(blur.slots):
            blur.pipe.slot(k).set_stream_trace(True)
        traces, lat2 = [], []
        for _ in range(a.trace):
            k = blur._next
            t = time.perf_counter()
            blur.step(40)
            lat2.append((time.perf_counter() - t) * 1e3)
            traces.append([[round(x, 4) for x in r] for r in blur.pipe.slot(k).stream_trace()])
        out["traced_latency_ms"] = sorted(lat2)[len(lat2) // 2]
        # per chunk: [chunk, upload end, launch wait passed, launches end, download wait passed, download end]
        out["chunk_trace_ms"] = traces[-3:]
    import pconv
    # the tuner's pick per launch key: [ch, steps, rows, row bytes, form, pf, lanes, rows/wave, waves]
    out["tuned"] = [list(k) + list(sh) for k, sh in pconv.native.swar_tuned()]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
