#!/usr/bin/env python3
"""Reproduce the reference's published timing tables (README.pdf pp.5-7,
transcribed in BASELINE.md) with MATCHING timer semantics.

  cuda     CUDA table: `conv image.raw 1920 H reps {grey,rgb}` on one GPU,
           END-TO-END time after argument parsing (HIP init, file read, H2D,
           loop, D2H, output write) -- the reference's cuda/main.c:20-49
           timer.  4 sizes x grey/RGB x reps 10..100, a real raw file per
           size (synthetic random bytes), median of --runs fresh processes.
  mpi-gpu  MPI table semantics (20 reps, loop only: mpi_convolution.c:151-154,
           242) on one GPU: `conv ... 20 ch` loop time.
  mpi-cpu  MPI / MPI+OpenMP tables on the CPU: torch.distributed.run with n
           ranks of `pconv.parallel.run --backend cpu|omp` (gloo halos), loop
           time max over ranks (the reference's Send/Recv max-gather).
  report   Render the JSONL results as markdown tables next to the published
           numbers (BASELINE.md "MI355X results").

Every run appends one JSON line to --out.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONV = os.path.join(ROOT, "parallel-image-convolution-using-mpi-openmp-and-cuda_amd", "bin", "conv")
SIZES = [630, 1260, 2520, 5040]
NAMES = {630: "1920×630 (x/4)", 1260: "1920×1260 (x/2)", 2520: "1920×2520 (x)", 5040: "1920×5040 (2x)"}
REPS = [10, 20, 40, 60, 80, 100]
NS = [1, 2, 4, 9, 16, 25]

# BASELINE.md wide tables (seconds).  CUDA: end-to-end on a GTX 970.
CUDA_REF = {
    ("grey", 630): [0.062, 0.068, 0.076, 0.089, 0.103, 0.118],
    ("grey", 1260): [0.077, 0.086, 0.116, 0.141, 0.168, 0.191],
    ("grey", 2520): [0.085, 0.123, 0.172, 0.221, 0.283, 0.326],
    ("grey", 5040): [0.113, 0.141, 0.189, 0.272, 0.332, 0.39],
    ("rgb", 630): [0.13, 0.183, 0.307, 0.426, 0.547, 0.67],
    ("rgb", 1260): [0.188, 0.296, 0.537, 0.78, 1.015, 1.254],
    ("rgb", 2520): [0.311, 0.546, 1.017, 1.503, 1.272, 2.448],
    ("rgb", 5040): [0.562, 1.021, 1.837, 2.308, 3.2, 4.428],
}
# MPI / MPI+OpenMP (20 reps, loop only), n = 1, 2, 4, 9, 16, 25.
MPI_REF = {
    ("grey", 630): [0.22, 0.09, 0.09, 0.08, 0.08, 0.1],
    ("grey", 1260): [0.69, 0.36, 0.3, 0.09, 0.1, 0.18],
    ("grey", 2520): [2.73, 1.28, 0.59, 0.31, 0.17, 0.24],
    ("grey", 5040): [10.71, 5.09, 2.3, 1.15, 0.56, 0.63],
    ("rgb", 630): [0.37, 0.14, 0.14, 0.1, 0.1, 0.2],
    ("rgb", 1260): [1.35, 0.68, 0.3, 0.17, 0.1, 0.2],
    ("rgb", 2520): [5.27, 2.55, 1.07, 0.59, 0.32, 0.37],
    ("rgb", 5040): [21.09, 10.08, 4.2, 2.19, 1.11, 1.18],
}
OMP_REF = {
    ("grey", 630): [0.12, 0.05, 0.05, 0.04, 0.04, 0.07],
    ("grey", 1260): [0.45, 0.23, 0.19, 0.05, 0.07, 0.14],
    ("grey", 2520): [1.7, 0.84, 0.37, 0.2, 0.1, 0.15],
    ("grey", 5040): [6.87, 3.26, 1.35, 0.75, 0.39, 0.46],
    ("rgb", 630): [0.25, 0.09, 0.08, 0.06, 0.06, 0.15],
    ("rgb", 1260): [0.91, 0.45, 0.2, 0.12, 0.61, 0.14],
    ("rgb", 2520): [3.41, 1.63, 0.68, 0.37, 0.19, 0.25],
    ("rgb", 5040): [13.47, 6.49, 2.68, 1.41, 0.7, 0.74],
}


def emit(path, rec):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
    print(json.dumps(rec)[:300], flush=True)


def make_image(d, ch, h, w=1920, seed=7):
    import numpy as np

    c = 3 if ch == "rgb" else 1
    p = os.path.join(d, f"img_{ch}_{w}_{h}.raw")
    if not os.path.exists(p) or os.path.getsize(p) != w * h * c:
        np.random.default_rng(seed + h + c).integers(0, 256, size=w * h * c, dtype=np.uint8).tofile(p)
    return p


def run_conv(args, timeout=120):
    t = time.perf_counter()
    r = subprocess.run([CONV] + args, capture_output=True, text=True, timeout=timeout)
    wall = time.perf_counter() - t
    if r.returncode != 0:
        raise RuntimeError(f"conv {' '.join(args)} failed: {r.stderr[-500:]}")
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    meta["process_wall_s"] = wall
    return meta


def start_server(d):
    sock = os.path.join(d, "pconv.sock")
    # stderr to a file, never an undrained pipe (a full pipe would block the server)
    log = open(os.path.join(d, "pconv_serve.stderr"), "w+")
    p = subprocess.Popen([CONV, "--serve", sock, "--device", "0", "--idle-timeout", "600"], stderr=log, text=True)
    for _ in range(1200):
        if os.path.exists(sock):
            return p, sock
        if p.poll() is not None:
            log.seek(0)
            raise RuntimeError(log.read()[-2000:])
        time.sleep(0.05)
    raise RuntimeError("server did not start")


def stop_server(p, sock):
    import struct

    s = socket.socket(socket.AF_UNIX)
    s.connect(sock)
    s.sendall(struct.pack("I", 1) + struct.pack("I", 12) + b"__shutdown__")
    s.recv(4096)
    s.close()
    p.wait(timeout=60)


def cmd_cuda(a):
    d = a.tmp
    os.makedirs(d, exist_ok=True)
    srv = start_server(d) if a.service else None
    extra = list(a.extra) + (["--server", srv[1]] if srv else [])
    for ch in ("grey", "rgb"):
        for h in SIZES:
            img = make_image(d, ch, h)
            for i, reps in enumerate(REPS):
                runs = []
                for _ in range(a.runs):
                    if a.gap > 0:  # let the previous process's KFD teardown finish (tools/ubench/hsa_cost.cpp)
                        time.sleep(a.gap)
                    m = run_conv([img, "1920", str(h), str(reps), ch, "--json", "--quiet",
                                  "--out", os.path.join(d, "out.raw")] + extra)
                    if srv:  # the client's clock (after its argument parsing -> answer), IPC included
                        m["server_e2e_s"], m["e2e_s"] = m["e2e_s"], m["client_e2e_s"]
                    runs.append(m)
                runs.sort(key=lambda m: m["e2e_s"])
                med = runs[len(runs) // 2]
                table = "cuda-service" if srv else ("cuda-idle" if a.gap > 0 else "cuda")
                emit(a.out, {"table": table, "gap_s": a.gap, "channels": ch, "height": h, "reps": reps,
                             "ref_s": CUDA_REF[(ch, h)][i],
                             "e2e_s": med["e2e_s"], "e2e_all_s": [m["e2e_s"] for m in runs],
                             "loop_s": med["loop_s"], "process_wall_s": med["process_wall_s"],
                             "since_exec_s": med.get("since_exec_s"), "phases_s": med.get("phases_s"),
                             "rccl_loaded": med.get("rccl_loaded"), "extra": extra})
    if srv:
        stop_server(*srv)


def cmd_mpi_gpu(a):
    d = a.tmp
    os.makedirs(d, exist_ok=True)
    for ch in ("grey", "rgb"):
        for h in SIZES:
            img = make_image(d, ch, h)
            runs = [run_conv([img, "1920", str(h), "20", ch, "--json", "--quiet", "--warmup", "1",
                              "--out", os.path.join(d, "out.raw")]) for _ in range(a.runs)]
            loops = sorted(m["loop_s"] for m in runs)
            emit(a.out, {"table": "mpi-gpu", "channels": ch, "height": h, "reps": 20, "gpus": 1,
                         "loop_s": loops[len(loops) // 2], "loop_all_s": loops,
                         "ref_mpi_best_s": min(MPI_REF[(ch, h)]), "ref_omp_best_s": min(OMP_REF[(ch, h)])})


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cmd_mpi_cpu(a):
    d = a.tmp
    os.makedirs(d, exist_ok=True)
    if not a.cpus:  # the CPUs this process may use: affinity capped by the cgroup quota (native helper)
        sys.path.insert(0, ROOT)
        import pconv

        a.cpus = pconv.native.default_cpu_threads() + 1
    ncpu = a.cpus
    for backend in a.backends.split(","):
        for ch in a.channels.split(","):
            for h in ([int(x) for x in a.sizes.split(",")] if a.sizes else SIZES):
                img = make_image(d, ch, h)
                for n in [int(x) for x in a.ranks.split(",")]:
                    env = dict(os.environ, PYTHONPATH=ROOT)
                    extra = []
                    threads = None
                    if a.unbound:  # round-2 policy (A/B): unbound ranks, team = CPUs // ranks
                        threads = max(1, ncpu // n) if backend == "omp" else 1
                        env.update(OMP_NUM_THREADS=str(threads))
                        extra = ["--threads", str(threads)] if backend == "omp" else []
                    if a.bind == "on" and not a.unbound:  # run.py --cpu-bind (default: unbound teams)
                        extra.append("--cpu-bind")
                    if a.wait:
                        env["OMP_WAIT_POLICY"] = a.wait
                    if a.spin is not None:
                        env["GOMP_SPINCOUNT"] = str(a.spin)
                        env.setdefault("OMP_WAIT_POLICY", "active")  # the spin count decides (libgomp)
                    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "pconv.parallel.run",
                           img, "1920", str(h), "20", ch, "--backend", backend, "--json", "--quiet",
                           "--out", os.path.join(d, f"out_{n}.raw")] + extra
                    loops, meta = [], {}
                    for _ in range(a.runs):
                        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
                        if r.returncode != 0:
                            raise RuntimeError(r.stderr[-800:])
                        meta = json.loads(r.stdout.strip().splitlines()[-1])
                        loops.append(meta["loop_s"])
                    loops.sort()
                    ref = (MPI_REF if backend == "cpu" else OMP_REF)[(ch, h)]
                    emit(a.out, {"table": "mpi-cpu", "backend": backend, "channels": ch, "height": h, "reps": 20,
                                 "ranks": n, "omp_threads": meta.get("omp_threads", threads),
                                 "rank0_cpus": meta.get("rank0_cpus"), "bound": meta.get("rank0_cpus") is not None,
                                 "wait_policy": a.wait or "runner default", "spin": a.spin,
                                 "loop_s": loops[len(loops) // 2],
                                 "loop_all_s": loops, "ref_s": ref[NS.index(n)] if n in NS else None,
                                 "cpus": ncpu})


def _load(paths):
    recs = []
    for p in paths:
        with open(p) as f:
            recs += [json.loads(l) for l in f if l.strip()]
    return recs


def _cuda_table(recs, table, title, out):
    cuda = {(r["channels"], r["height"], r["reps"]): r for r in recs if r["table"] == table}
    if not cuda:
        return
    out.append(title)
    out.append("Each cell: MI355X e2e (median of fresh processes) / reference; **bold** = MI355X faster.\n")
    out.append("| image | " + " | ".join(f"{r} reps" for r in REPS) + " |")
    out.append("|---" * (len(REPS) + 1) + "|")
    wins = total = 0
    for ch in ("grey", "rgb"):
        for h in SIZES:
            cells = []
            for i, reps in enumerate(REPS):
                r = cuda.get((ch, h, reps))
                if r is None:
                    cells.append("—")
                    continue
                ref = CUDA_REF[(ch, h)][i]
                total += 1
                win = r["e2e_s"] < ref
                wins += win
                v = f"{r['e2e_s']:.3f} / {ref}"
                cells.append(f"**{v}**" if win else v)
            out.append(f"| {'Grey' if ch == 'grey' else 'RGB'} {NAMES[h]} | " + " | ".join(cells) + " |")
    out.append(f"\nMI355X faster in {wins} of {total} cells.\n")
    ph = [r for r in cuda.values() if r.get("phases_s")]
    if ph:
        keys = list(ph[0]["phases_s"].keys())
        out.append("Median phase breakdown over all cells (ms): " + ", ".join(
            f"{k} {statistics.median(r['phases_s'].get(k, 0) for r in ph) * 1e3:.2f}" for k in keys) + "\n")


def cmd_report(a):
    recs = _load(a.inputs)
    out = []
    for table, title in (("cuda", "### CUDA table semantics: `conv` end-to-end (s), cold process, one MI355X vs "
                                   "GTX 970, processes back to back\n"),
                         ("cuda-idle", "### CUDA table semantics: `conv` end-to-end (s), one cold process on an idle GPU "
                                       "(idle gap before each process), one MI355X vs GTX 970\n"),
                         ("cuda-service", "### CUDA table semantics through the resident service: `conv --server` "
                                          "end-to-end (s, client clock), one MI355X vs GTX 970\n")):
        _cuda_table(recs, table, title, out)
    mg = [r for r in recs if r["table"] == "mpi-gpu"]
    if mg:
        out.append("### MPI table semantics (20 reps, loop only, s): one MI355X vs the reference's best n\n")
        out.append("| image | MI355X 1 GPU loop | ref MPI best (any n) | ref MPI+OpenMP best | speed-up vs best |")
        out.append("|---|---|---|---|---|")
        for r in sorted(mg, key=lambda r: (r["channels"], r["height"])):
            best = min(r["ref_mpi_best_s"], r["ref_omp_best_s"])
            out.append(f"| {'Grey' if r['channels'] == 'grey' else 'RGB'} {NAMES[r['height']]} | {r['loop_s']:.6f} | "
                       f"{r['ref_mpi_best_s']} | {r['ref_omp_best_s']} | {best / r['loop_s']:.0f}× |")
        out.append("")
    mc = [r for r in recs if r["table"] == "mpi-cpu"]
    for backend, title, ref in (("cpu", "MPI (CPU ranks, gloo halos)", MPI_REF), ("omp", "MPI+OpenMP", OMP_REF)):
        rows = [r for r in mc if r["backend"] == backend]
        if not rows:
            continue
        ns = sorted({r["ranks"] for r in rows})
        cpus = rows[0].get("cpus")
        out.append(f"### {title}, 20 reps, loop only, max over ranks (s): this CPU ({cpus} cores) / reference\n")
        out.append("| image | " + " | ".join(f"n={n}" for n in ns) + " |")
        out.append("|---" * (len(ns) + 1) + "|")
        for ch in ("grey", "rgb"):
            for h in SIZES:
                cells = []
                for n in ns:
                    r = next((x for x in rows if x["channels"] == ch and x["height"] == h and x["ranks"] == n), None)
                    if r is None:
                        cells.append("—")
                        continue
                    refv = ref[(ch, h)][NS.index(n)] if n in NS else None
                    v = f"{r['loop_s']:.3f} / {refv}"
                    cells.append(f"**{v}**" if refv is not None and r["loop_s"] < refv else v)
                out.append(f"| {'Grey' if ch == 'grey' else 'RGB'} {NAMES[h]} | " + " | ".join(cells) + " |")
        out.append("")
    text = "\n".join(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")
    print(text)


def main():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = p.add_subparsers(dest="cmd", required=True)
    for name in ("cuda", "mpi-gpu", "mpi-cpu"):
        s = sub.add_parser(name)
        s.add_argument("--out", default=f"gpurun_out/ref_tables/{name}.jsonl")
        s.add_argument("--tmp", default="/tmp/pconv_ref_tables")
        s.add_argument("--runs", type=int, default=3)
        if name == "cuda":
            s.add_argument("--service", action="store_true",
                           help="run every job through one resident `conv --serve` (warm GPU context)")
            s.add_argument("--gap", type=float, default=0.0,
                           help="idle seconds before each fresh process: a process started right after another "
                                "waits 85-206 ms in open(/dev/kfd) for the previous one's driver teardown")
            s.add_argument("--extra", nargs=argparse.REMAINDER, default=[])
        if name == "mpi-cpu":
            s.add_argument("--backends", default="cpu,omp")
            s.add_argument("--ranks", default="1,2,4,9,16")
            s.add_argument("--cpus", type=int, default=0)
            s.add_argument("--sizes", default=None, help="comma list of heights (default: all four)")
            s.add_argument("--channels", default="grey,rgb")
            s.add_argument("--unbound", action="store_true",
                           help="A/B: the round-2 policy (no CPU binding, team = CPUs // ranks)")
            s.add_argument("--bind", choices=["default", "on", "off"], default="default",
                           help="A/B: CPU slices per rank (default: the runner's choice, off)")
            s.add_argument("--wait", choices=["passive", "active"], default=None,
                           help="A/B: OMP_WAIT_POLICY of the ranks (default: the runner's choice)")
            s.add_argument("--spin", type=int, default=None, help="A/B: GOMP_SPINCOUNT of the ranks")
    s = sub.add_parser("report")
    s.add_argument("inputs", nargs="+")
    s.add_argument("--md", default=None)
    a = p.parse_args()
    {"cuda": cmd_cuda, "mpi-gpu": cmd_mpi_gpu, "mpi-cpu": cmd_mpi_cpu, "report": cmd_report}[a.cmd](a)


if __name__ == "__main__":
    main()
