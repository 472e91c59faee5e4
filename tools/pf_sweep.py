"""Prefetching persistent tile kernel (k_swar_pf) against the relaunching
tile kernel on one frame: us per repetition of a fused-launch loop
(BandEngine, one GPU, whole frame), for
  * the tuned default without the prefetch kernel (PCONV_PREFETCH=0 path),
  * every prefetch shape x step form, forced,
  * the tuned choice with the prefetch kernel among the candidates.
python tools/pf_sweep.py --width 32768 --height 32768 --channels grey --fuse 8 --reps 240
One JSON line per configuration.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--width", type=int, default=32768)
    p.add_argument("--height", type=int, default=32768)
    p.add_argument("--channels", default="grey")
    p.add_argument("--reps", type=int, default=240)
    p.add_argument("--fuse", type=int, default=8)
    p.add_argument("--iters", type=int, default=2)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--check", action="store_true", help="compare every configuration's result with the first")
    a = p.parse_args()
    import numpy as np

    import pconv

    n = pconv.native
    e = n.BandEngine(a.width, a.height, a.channels, "gaussian", 0, 1, 0, halo=a.fuse, fuse=a.fuse,
                     variant="temporal")
    img = pconv.synthetic_image(a.width, a.height, a.channels, seed=5)
    flat = np.ascontiguousarray(img.reshape(a.height, -1)).reshape(-1)

    def timed():
        e.upload(flat, 0, a.height)
        e.run(a.reps)  # warm + tune
        e.synchronize()
        best = 1e9
        for _ in range(a.rounds):
            t = time.perf_counter()
            for _ in range(a.iters):
                e.run(a.reps)
            e.synchronize()
            best = min(best, (time.perf_counter() - t) / a.iters)
        return best / a.reps * 1e6

    def result():
        e.upload(flat, 0, a.height)
        e.run(a.reps)
        e.synchronize()
        out = np.empty_like(flat)
        e.download(out, 0, a.height)
        e.synchronize()
        return out

    ref = None
    # (name, prefetch mode, grid cap, shape, form): tile = relaunching k_swar
    # forced to the shape; pf = persistent prefetching; buf = the prefetch
    # kernel's buffer-op code with one workgroup per tile (no persistence)
    configs = [("tuned_no_prefetch", 0, 0, None, -1), ("tuned_with_prefetch", -1, 0, None, -1)]
    for sh in n.swar_prefetch_shapes():
        for form in (0, 1):
            tag = f"{sh[0]}_{sh[1]}_{sh[2]}_alt{form}"
            configs += [(f"tile_{tag}", 0, 0, sh, form), (f"pf_{tag}", 1, -1, sh, form), (f"buf_{tag}", 1, 0, sh, form)]
    for name, mode, cap, sh, form in configs:
        n.clear_swar_tuning()
        n.set_prefetch_mode(mode, cap)
        n.set_swar_shape(*(sh or (0, 0, 0)))
        n.set_swar_alt(form)
        rec = {"config": name, "width": a.width, "height": a.height, "channels": a.channels, "fuse": a.fuse,
               "reps": a.reps}
        try:
            rec["us_per_rep"] = round(timed(), 3)
            rec["tuned"] = [list(k) + [list(v)] for k, v in n.swar_tuned()]
            if a.check:
                r = result()
                if ref is None:
                    ref = r
                rec["mismatches_vs_first"] = int(np.count_nonzero(r != ref))
        except Exception as ex:
            rec["error"] = str(ex)[:200]
        print(json.dumps(rec), flush=True)
    n.set_prefetch_mode(-1, 0)
    n.set_swar_shape(0, 0, 0)
    n.set_swar_alt(-1)


if __name__ == "__main__":
    main()
