#!/usr/bin/env python3
"""Interior || halo overlap on the device, for a rocprofv3 trace.

  run   (GPU, under rocprofv3 --kernel-trace --memory-copy-trace):
          rccl-self   one band whose up/down neighbour is itself, RCCL
                      ncclSend/ncclRecv on the comm stream every exchange
                      phase, interior launch on the compute stream — the
                      production per-rank path of a multi-GPU run;
          local-async N bands on one device, D2D halo copies on each band's
                      comm stream (LocalCluster device_async).
  analyse (CPU): read the trace CSVs and report, per exchange, whether an
          interior stencil kernel ran concurrently with the halo transfer
          (RCCL kernel or copy), and by how much.

The reference overlaps MPI_Isend/Irecv with an "inner" compute pass
(mpi/mpi_convolution.c:156-240; in fact its inner pass covers the whole
block).
"""
from __future__ import annotations

import argparse
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(a):
    sys.path.insert(0, ROOT)
    import numpy as np

    import pconv

    n = pconv.native
    w, h, reps = a.width, a.height, a.reps
    img = np.random.default_rng(1).integers(0, 256, size=(h, w * 3), dtype=np.uint8)
    if a.mode == "rccl-self":
        b = n.Band()
        b.rank, b.world, b.y0, b.rows, b.up, b.down = 0, 1, 0, h, 0, 0
        comm = n.RcclComm(n.rccl_unique_id(), 0, 1, 0)
        eng = n.BandEngine.for_band(w, h, "rgb", "gaussian", b, 0, a.halo, a.fuse, True, "auto")
        eng.attach_rccl(comm)
        for _ in range(a.iters):
            eng.upload(img.reshape(-1), 0, h)
            eng.run(reps)
            comm.wait(eng.comm_stream, 60.0)
            comm.wait(eng.compute_stream, 60.0)
            eng.synchronize()
        out = np.empty_like(img)
        eng.download(out.reshape(-1), 0, h)
        eng.synchronize()
        ok = np.array_equal(out.reshape(h, w, 3), pconv.numpy_convolve(img.reshape(h, w, 3), reps))
    else:
        cl = n.LocalCluster(w, h, "rgb", "gaussian", a.bands, 0, a.halo, a.fuse, "auto", True)
        for _ in range(a.iters):
            cl.upload(img.reshape(-1), False)
            cl.run(reps, True)
        out = np.empty_like(img)
        cl.download(out.reshape(-1))
        ok = np.array_equal(out.reshape(h, w, 3), pconv.numpy_convolve(img.reshape(h, w, 3), reps))
    print(f"{a.mode}: exact={ok}")
    if not ok:
        sys.exit(1)


def analyse(a):
    d = a.trace_dir
    ks = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    halo = []  # (start, end, what, stream)
    interior = []
    stencil_streams = {k["Stream_Id"] for k in ks if "k_swar" in k["Kernel_Name"] or "k_binomial" in k["Kernel_Name"]}
    blits = []
    for k in ks:
        name = k["Kernel_Name"]
        s, e, st = int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Stream_Id"]
        if any(t in name.lower() for t in ("rccl", "ncclkernel", "nccldevkernel")):
            if a.kinds == "rccl":
                halo.append((s, e, "rccl:" + name.split("(")[0].replace("void ", "")[:30], st))
        elif "k_swar" in name or "k_binomial" in name or "k_stream" in name:
            interior.append((s, e, name.split("(")[0][-40:], st))
        elif "copyBuffer" in name and st not in stencil_streams:
            blits.append((s, e, "D2D halo copy (blit)", st))
    if a.kinds == "blit":
        # halo copies = blit copies on streams that run no stencil kernel
        # (the bands' comm streams); uploads run on the compute streams
        halo = blits
    halo.sort()
    lines = [f"# overlap trace: {d}", "",
             f"{len(halo)} halo transfers (RCCL kernels / copies), {len(interior)} stencil launches", "",
             "| transfer | stream | us | overlapping stencil launches (other stream) | overlap us |",
             "|---|---|---|---|---|"]
    n_ov = 0
    tot = 0.0
    for s, e, what, st in halo:
        ov = [(max(s, ks_), min(e, ke)) for ks_, ke, _, kst in interior if kst != st and ks_ < e and ke > s]
        us = sum(b - a_ for a_, b in ov) / 1e3
        n_ov += bool(ov)
        tot += us
        lines.append(f"| {what} | {st} | {(e - s) / 1e3:.1f} | {len(ov)} | {us:.1f} |")
    lines += ["", f"**{n_ov} of {len(halo)} halo transfers overlapped a stencil launch on another stream "
                  f"(total overlap {tot:.1f} us).**"]
    text = "\n".join(lines[:6 + min(len(halo), a.max_rows)] + lines[-2:])
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


def main():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("mode", choices=["rccl-self", "local-async"])
    r.add_argument("--width", type=int, default=1920)
    r.add_argument("--height", type=int, default=2520)
    r.add_argument("--reps", type=int, default=40)
    r.add_argument("--halo", type=int, default=8)
    r.add_argument("--fuse", type=int, default=8)
    r.add_argument("--bands", type=int, default=4)
    r.add_argument("--iters", type=int, default=3)
    an = sub.add_parser("analyse")
    an.add_argument("trace_dir")
    an.add_argument("--md", default=None)
    an.add_argument("--max-rows", type=int, default=40)
    an.add_argument("--kinds", choices=["rccl", "blit"], default="rccl",
                    help="which transfers are halo exchanges: RCCL kernels, or D2D blit copies on comm streams")
    a = p.parse_args()
    run(a) if a.cmd == "run" else analyse(a)


if __name__ == "__main__":
    main()
