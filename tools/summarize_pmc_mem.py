#!/usr/bin/env python3
"""Summarise tools/r02/pmc_mem.sh passes into a markdown roofline table.

For every stencil-kernel dispatch of the timed loop (the tuned kernel; the
tuning candidates are reported separately) it joins the counter passes by
dispatch order and reports, per launch:
  * duration (kernel trace of each pass, median),
  * FETCH_SIZE / WRITE_SIZE (KB) against the ideal bytes of one fused launch
    (read the source frame rows the launch touches once, write the output
    rows once),
  * TCC_EA0_RDREQ / WRREQ (fabric requests: L2 misses going to the Infinity
    Cache / HBM) and TCC hit rate,
  * LDS bank conflicts per LDS instruction, VALU instructions per wave.
Caveat (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE = RDREQ x 64 B
and reports 1/2 of the bytes of 128-B streaming requests; both readings are
given.  Usage: summarize_pmc_mem.py DIR --rows R --row-bytes B --steps S
"""
from __future__ import annotations

import argparse
import csv
import os
import statistics
from collections import defaultdict


def load(pass_dir):
    p = os.path.join(pass_dir, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    per = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(p)):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                   int(r["Grid_Size"]), int(r["Workgroup_Size"]), int(r["VGPR_Count"]), int(r["LDS_Block_Size"]))
    return {d: (meta[d], per[d]) for d in per}


def short(name):
    import re

    m = re.search(r"(k_\w+<[^>]*>)", name)
    return m.group(1) if m else name.split("(")[0]


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("dir")
    ap.add_argument("--rows", type=int, required=True, help="rows per launch (output)")
    ap.add_argument("--row-bytes", type=int, required=True)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--title", default="")
    ap.add_argument("--last", type=int, default=0, help="only the last N stencil dispatches (the timed loop)")
    a = ap.parse_args()
    passes = {k: load(os.path.join(a.dir, k)) for k in ("fetch", "write_l2", "sq", "ea")}
    # kernel -> list of merged counter dicts (dispatch order within each pass)
    merged = defaultdict(list)
    for name, data in passes.items():
        seq = [(d, m, c) for d, (m, c) in sorted(data.items()) if "k_swar" in m[0] or "k_stream" in m[0]
               or "k_binomial" in m[0] or "k_temporal" in m[0]]
        if a.last:
            seq = seq[-a.last:]
        bykern = defaultdict(list)
        for d, m, c in seq:
            bykern[(short(m[0]), m[2], m[3], m[4], m[5])].append((m[1], c))
        for k, lst in bykern.items():
            cur = merged[k]
            while len(cur) < len(lst):
                cur.append({"dur_us": []})
            for i, (dur, c) in enumerate(lst):
                cur[i]["dur_us"].append(dur)
                cur[i].update(c)
    ideal_in = (a.rows + 2 * a.steps) * a.row_bytes
    ideal_out = a.rows * a.row_bytes
    out = []
    if a.title:
        out.append(f"## {a.title}\n")
    out.append(f"Ideal bytes per launch: read {ideal_in / 1024:.0f} KB (rows + 2x{a.steps} halo rows), "
               f"write {ideal_out / 1024:.0f} KB.\n")
    out.append("| kernel (grid, wg, vgpr, lds) | launches | us | FETCH_SIZE KB (x2 for 128-B req.) | fetch / ideal "
               "| WRITE_SIZE KB | write / ideal | EA rd req | EA wr req | TCC hit % | LDS conflicts / LDS inst "
               "| VALU inst / wave |")
    out.append("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for (kname, grid, wg, vgpr, lds), lst in sorted(merged.items(), key=lambda kv: -len(kv[1])):
        def med(key):
            v = [x[key] for x in lst if key in x]
            return statistics.median(v) if v else float("nan")
        dur = statistics.median([d for x in lst for d in x["dur_us"]])
        fetch = med("FETCH_SIZE")
        write = med("WRITE_SIZE")
        hit, miss = med("TCC_HIT_sum"), med("TCC_MISS_sum")
        hr = 100.0 * hit / (hit + miss) if hit + miss > 0 else float("nan")
        conf, ldsi = med("SQ_LDS_BANK_CONFLICT"), med("SQ_ACTIVE_INST_LDS")
        valu, waves = med("SQ_INSTS_VALU"), med("SQ_WAVES")
        out.append(f"| {kname} ({grid}, {wg}, {vgpr}, {lds}) | {len(lst)} | {dur:.1f} | {fetch:.0f} ({2 * fetch:.0f}) | "
                   f"{fetch * 1024 / ideal_in:.2f}-{2 * fetch * 1024 / ideal_in:.2f} | {write:.0f} | "
                   f"{write * 1024 / ideal_out:.2f} | {med('TCC_EA0_RDREQ_sum'):.0f} | {med('TCC_EA0_WRREQ_sum'):.0f} | "
                   f"{hr:.1f} | {conf / ldsi if ldsi else float('nan'):.3f} | "
                   f"{valu / waves if waves else float('nan'):.0f} |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
