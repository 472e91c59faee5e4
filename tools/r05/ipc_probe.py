#!/usr/bin/env python3
"""Round 5: cost of one IPC halo exchange per pull form (ipc_halo.hpp).

Each form pulls the 8-way headline rank's ghost zone (2 sides x 40 rows x
5,760 B = 460 KB) through the self-neighbour flag protocol, from this GPU's
HBM and from pinned HOST memory — the stand-in for a peer GPU's HBM behind
xGMI (every load a fabric round trip of microseconds, as a remote pull is).
Prints one JSON line per (form, workgroups, source): ms per exchange, best of
`--repeat` runs of `--iters` back-to-back exchanges.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--bytes", type=int, default=40 * 5760, help="bytes per side")
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--repeat", type=int, default=3)
    p.add_argument("--workgroups", default="0,8,16,32,64,128")
    a = p.parse_args()
    import pconv

    n = pconv.native
    cases = [("single", 0), ("sdma", 0)] + [("grid", int(g)) for g in a.workgroups.split(",")]
    for host in (False, True):
        for form, wg in cases:
            ms = min(n.ipc_pull_probe(form, a.bytes, host, a.iters, 0, wg) for _ in range(a.repeat))
            eff = wg if wg else (n.ipc_grid_workgroups(a.bytes) if form == "grid" else (1 if form == "single" else 0))
            print(json.dumps({"form": form, "workgroups": eff, "source": "pinned_host" if host else "hbm",
                              "bytes_per_side": a.bytes, "ms_per_exchange": round(ms, 5),
                              "gb_per_s": round(2 * a.bytes / ms / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
