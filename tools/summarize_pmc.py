"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel.

python tools/summarize_pmc.py gpurun_out/pmc_sq/run_counter_collection.csv [--cus 256]
Prints a markdown table: dispatches, mean duration, counters summed per
dispatch, and derived issue rates:
  valu_per_wave   = SQ_INSTS_VALU / SQ_WAVES
  valu_ipc_simd   = SQ_INSTS_VALU / (duration * clock * CUs * 4)  (wave-instr / SIMD / clock;
                    measured gfx950 issue limit ~0.36 with >= 3 waves/SIMD, 0.17 with one)
  lds_per_wave    = SQ_INSTS_LDS / SQ_WAVES
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("pconv::(anonymous namespace)::", "").replace("void ", "")
    if name.endswith(")"):  # drop the argument list (last balanced parenthesis)
        depth = 0
        for i in range(len(name) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(name[i], 0)
            if depth == 0:
                return name[:i]
    return name


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--cus", type=int, default=256)
    p.add_argument("--ghz", type=float, default=2.4)
    a = p.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(a.csv)):
        k = short(r["Kernel_Name"])
        d = r["Dispatch_Id"]
        per[k][(d, r["Counter_Name"])] += float(r["Counter_Value"])
        dur[k][d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["SGPR_Count"])
    print("| kernel | dispatches | grid | wg | LDS B | VGPR | mean us | waves | VALU/wave | LDS/wave | "
          "waves/SIMD | VALU IPC/SIMD |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k, cnt in per.items():
        ds = sorted(dur[k])
        tot = collections.defaultdict(float)
        for (d, c), v in cnt.items():
            tot[c] += v
        n = len(ds)
        waves = tot["SQ_WAVES"] / n if n else 0
        valu = tot["SQ_INSTS_VALU"] / n if n else 0
        lds = tot["SQ_INSTS_LDS"] / n if n else 0
        gui = tot["GRBM_GUI_ACTIVE"] / n if n else 0
        busy = tot["SQ_BUSY_CYCLES"] / n if n else 0
        us = sum(dur[k].values()) / n / 1e3 if n else 0
        ipc = valu / (us * 1e3 * a.ghz * a.cus * 4) if us else 0
        g, wg, ldsb, vg, sg = meta[k]
        print(f"| `{k}` | {n} | {g} | {wg} | {ldsb} | {vg} | {us:.1f} | {waves:.0f} | {valu / waves if waves else 0:.0f} "
              f"| {lds / waves if waves else 0:.1f} | {waves / (a.cus * 4):.2f} | {ipc:.3f} |")


if __name__ == "__main__":
    main()
