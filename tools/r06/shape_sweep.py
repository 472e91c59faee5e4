#!/usr/bin/env python3
"""Round 6: tile shapes forced on the large-frame loop (32768^2 grey, 24
reps at fuse 12) — the tuner's pick first, then every (kernel, shape, form)
listed, each timed as us per repetition (best of --repeat), and the tuner
again with the widened candidate set.  One JSON line per configuration."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "r05"))
import pconv  # noqa: E402
from form_ab import CFG, loop_us  # noqa: E402

SHAPES = [(1, 4, 20, 8), (1, 4, 24, 8), (1, 4, 16, 16), (1, 4, 20, 16), (0, 4, 20, 8), (0, 4, 24, 8),
          (0, 4, 16, 16), (0, 4, 20, 16)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--which", default="grey32768")
    p.add_argument("--repeat", type=int, default=3)
    p.add_argument("--candidates", type=int, default=8)
    a = p.parse_args()
    n = pconv.native
    for which in a.which.split(","):
        iters = 3 if which == "grey32768" else 20
        fuse = CFG[which][4]
        for cands in (6, a.candidates):
            n.clear_swar_tuning()
            n.set_autotune(True)
            n.set_tune_candidates(cands)
            n.set_swar_alt(-1)
            n.set_prefetch_mode(-1)
            n.set_swar_shape(0, 0, 0)
            us = loop_us(n, which, iters, a.repeat)
            t = [(k, s) for k, s in n.swar_tuned() if k[1] == fuse]
            k, s = max(t, key=lambda e: e[0][2])
            print(json.dumps({"loop": which, "config": f"tuned({cands})", "pick": {"shape": list(s), "form": int(k[4]),
                              "pf": int(k[5])}, "us_per_rep": round(us, 3)}), flush=True)
        n.set_tune_candidates(6)
        n.set_autotune(False)
        for pf, lw, m, nw in SHAPES:
            for form in (0, 1):
                n.set_swar_shape(lw, m, nw)
                n.set_prefetch_mode(pf)
                n.set_swar_alt(form)
                try:
                    us = loop_us(n, which, iters, a.repeat)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"loop": which, "shape": [lw, m, nw], "pf": pf, "form": form,
                                      "error": str(e)[:200]}), flush=True)
                    continue
                print(json.dumps({"loop": which, "shape": [lw, m, nw], "pf": pf, "form": form,
                                  "us_per_rep": round(us, 3)}), flush=True)
    n.set_swar_alt(-1)
    n.set_prefetch_mode(-1)
    n.set_swar_shape(0, 0, 0)
    n.set_autotune(True)


if __name__ == "__main__":
    main()
