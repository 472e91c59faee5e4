"""Host-side cost of enqueueing one image into the serving pipeline.

Times N back-to-back submit() calls (host wall, no drain) vs the time until
the GPU has drained them: if enqueue time ~ total, the pipeline is host-bound.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import pconv  # noqa: F401
    from pconv.parallel.dist_engine import DistributedBlur

    for h in (315, 2520):
        blur = DistributedBlur(1920, h, "rgb", "gaussian", 40, rank=0, world=1, device=0, slots=3, concurrent=0)
        blur.load_synthetic(1)
        for _ in range(20):
            blur.submit(40)
        blur.drain()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            blur.submit(40)
        t1 = time.perf_counter()
        blur.drain()
        t2 = time.perf_counter()
        eng = blur.engine
        t3 = time.perf_counter()
        for _ in range(n):
            eng.run(40)
        t4 = time.perf_counter()
        eng.synchronize()
        t5 = time.perf_counter()
        print(json.dumps({"height": h, "submit_us": round((t1 - t0) / n * 1e6, 2),
                          "submit_to_drain_us": round((t2 - t0) / n * 1e6, 2),
                          "run_enqueue_us": round((t4 - t3) / n * 1e6, 2),
                          "run_total_us": round((t5 - t3) / n * 1e6, 2),
                          "launches_per_run": blur.stats.launches}), flush=True)


if __name__ == "__main__":
    main()
