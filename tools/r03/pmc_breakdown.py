#!/usr/bin/env python3
"""Where a fused launch's time goes, from rocprofv3 --pmc passes (CPU only).

python tools/r03/pmc_breakdown.py DIR [DIR ...] [--md out.md]
Each DIR holds one pass's run_counter_collection.csv.  The kernel launched
most often (the production kernel of tools/r03/pmc_loops.py) is summarised:
mean duration, counters per launch, and the shares of the waves' lifetime
(SQ_WAVE_CYCLES) spent issuing VALU, waiting on a dependency (s_waitcnt /
barrier: SQ_WAIT_ANY) and waiting for an issue slot (SQ_WAIT_INST_ANY), plus
the VALU issue rate per SIMD against the measured gfx950 limit (~0.35
wave-instructions per SIMD per clock with 2+ waves per SIMD).
"""
import argparse
import collections
import csv
import glob
import os


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, dur


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dirs", nargs="+")
    p.add_argument("--cus", type=int, default=256)
    p.add_argument("--ghz", type=float, default=2.4)
    p.add_argument("--md", default=None)
    p.add_argument("--title", default="")
    a = p.parse_args()
    tot = collections.defaultdict(float)
    launches = us = 0.0
    name = None
    for d in a.dirs:
        per, dur = load(d)
        k = max(dur, key=lambda x: len(dur[x]))
        name = name or k
        n = len(dur[k])
        for c, v in per[k].items():
            tot[c] = v / n
        launches = n
        us = sum(dur[k].values()) / n / 1e3
    lines = [f"# {a.title or 'fused launch breakdown'}", "", f"kernel `{name}`, {launches:.0f} launches per pass, "
             f"mean {us:.2f} us per launch", "", "| counter | per launch |", "|---|---|"]
    lines += [f"| {c} | {v:.4g} |" for c, v in sorted(tot.items())]
    wc = tot.get("SQ_WAVE_CYCLES", 0)
    if wc:
        lines += ["", "| share of wave lifetime (SQ_WAVE_CYCLES) | |", "|---|---|"]
        for c, label in (("SQ_ACTIVE_INST_VALU", "issuing VALU"), ("SQ_ACTIVE_INST_LDS", "issuing LDS"),
                         ("SQ_ACTIVE_INST_ANY", "issuing any instruction"),
                         ("SQ_WAIT_ANY", "waiting on a dependency (waitcnt / barrier)"),
                         ("SQ_WAIT_INST_ANY", "waiting for an issue slot"),
                         ("SQ_WAIT_INST_LDS", "waiting to issue LDS")):
            if c in tot:
                lines.append(f"| {label} ({c}) | {tot[c] / wc:.3f} |")
    if "SQ_INSTS_VALU" in tot and us:
        ipc = tot["SQ_INSTS_VALU"] / (us * 1e3 * a.ghz * a.cus * 4)
        lines += ["", f"VALU issue rate: {ipc:.3f} wave-instructions per SIMD per clock "
                      f"({ipc / 0.35:.0%} of the ~0.35 measured limit); "
                      f"{tot['SQ_INSTS_VALU'] / max(1.0, tot.get('SQ_WAVES', 1)):.0f} VALU per wave, "
                      f"{tot.get('SQ_WAVES', 0) / (a.cus * 4):.2f} waves per SIMD per launch"]
    text = "\n".join(lines)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
