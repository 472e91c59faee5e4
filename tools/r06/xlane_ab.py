#!/usr/bin/env python3
"""Round 6: the SWAR step's lane-crossing operand read with DPP (the add's
DPP source, ~1.8 issue slots) or with an LDS permute (ds_bpermute: off the
VALU, the add a plain VOP2) — the tuned loops of the headline, the 8-way band
and 32768^2 grey x24, us per repetition (best of --repeat), for whichever
native build is loaded (the caller swaps the .so between runs)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "r05"))
import pconv  # noqa: E402
from form_ab import loop_us  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", required=True)
    p.add_argument("--repeat", type=int, default=3)
    a = p.parse_args()
    n = pconv.native
    for which in ("headline", "band8", "grey32768"):
        n.clear_swar_tuning()
        n.set_autotune(True)
        us = loop_us(n, which, 3 if which == "grey32768" else 20, a.repeat)
        picks = [list(k) + list(s) for k, s in n.swar_tuned()]
        print(json.dumps({"variant": a.variant, "loop": which, "us_per_rep": round(us, 3), "tuned": picks}), flush=True)


if __name__ == "__main__":
    main()
