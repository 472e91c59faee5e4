"""CPU tests of the evidence tooling (tools/): the analyses that turn
rocprofv3 traces and sweep JSONL into the tables under profiles/ are checked
on small synthetic inputs with known answers."""
from __future__ import annotations

import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")


def _run(*args):
    r = subprocess.run([sys.executable] + list(args), cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def _write_csv(path, fields, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _kernel_rows(spec):
    return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e, "Stream_Id": st} for n, s, e, st in spec]


def test_copy_trace_direction_from_stream_order(tmp_path):
    """Copies before a stencil launch on their stream are H2D, after it D2H
    (whole-step graphs report every copy as device-to-device)."""
    copies, kernels = [], []
    t = 0
    for img in range(4):
        st = str(img % 2 + 1)  # two slot streams
        copies.append({"Start_Timestamp": t, "End_Timestamp": t + 300_000, "Stream_Id": st,
                       "Direction": "MEMORY_COPY_DEVICE_TO_DEVICE"})
        kernels.append(("void pconv::k_swar<3, 4, 8, 8, true>(...)", t + 300_000, t + 400_000, st))
        copies.append({"Start_Timestamp": t + 400_000, "End_Timestamp": t + 700_000, "Stream_Id": st,
                       "Direction": "MEMORY_COPY_DEVICE_TO_DEVICE"})
        t += 350_000
    _write_csv(tmp_path / "run_memory_copy_trace.csv", ["Start_Timestamp", "End_Timestamp", "Stream_Id", "Direction"],
               copies)
    _write_csv(tmp_path / "run_kernel_trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id"],
               _kernel_rows(kernels))
    md = tmp_path / "out.md"
    out = _run(os.path.join(TOOLS, "copy_trace_summary.py"), str(tmp_path), "--images", "4", "--md", str(md),
               "--bytes", str(300 * 1000))
    rows = {l.split("|")[1].strip(): l for l in out.splitlines() if l.startswith("| H2D") or l.startswith("| D2H")}
    assert set(rows) == {"H2D", "D2H"}
    assert rows["H2D"].split("|")[2].strip() == "4" and rows["D2H"].split("|")[2].strip() == "4"
    # every copy lasts 300 us
    assert rows["H2D"].split("|")[4].strip() == "300"
    assert md.read_text().startswith("# Copy trace")


def test_overlap_trace_counts_concurrent_interior(tmp_path):
    """An RCCL transfer on the comm stream overlapping a stencil launch on
    the compute stream counts; one with nothing concurrent does not."""
    ks = _kernel_rows([
        ("void pconv::k_swar<1, 4, 8, 8, false>(...)", 0, 10_000, "1"),
        ("ncclDevKernel_Generic_1(...)", 2_000, 6_000, "2"),           # under the interior launch
        ("void rcclGenericKernel<1, false>(...)", 20_000, 25_000, "2"),  # alone
        ("void pconv::k_swar<1, 4, 8, 8, false>(...)", 26_000, 30_000, "1"),
    ])
    _write_csv(tmp_path / "run_kernel_trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id"], ks)
    out = _run(os.path.join(TOOLS, "overlap_trace.py"), "analyse", str(tmp_path))
    assert "1 of 2 halo transfers overlapped" in out
    assert "total overlap 4.0 us" in out


def test_ref_tables_report_counts_wins(tmp_path):
    """The CUDA-table renderer bolds and counts exactly the cells below the
    reference; MPI rows render from their own records."""
    recs = []
    for table, e2e in (("cuda", 0.5), ("cuda-idle", 0.07)):
        for reps, ref in zip((10, 20, 40, 60, 80, 100), (0.062, 0.068, 0.076, 0.089, 0.103, 0.118)):
            recs.append({"table": table, "channels": "grey", "height": 630, "reps": reps, "ref_s": ref, "e2e_s": e2e,
                         "phases_s": {"hip_init": 0.05, "queue": 0.02}})
    recs.append({"table": "mpi-gpu", "channels": "rgb", "height": 2520, "reps": 20, "gpus": 1, "loop_s": 0.0001,
                 "ref_mpi_best_s": 0.32, "ref_omp_best_s": 0.19})
    recs.append({"table": "mpi-cpu", "backend": "cpu", "channels": "rgb", "height": 2520, "reps": 20, "ranks": 4,
                 "omp_threads": 1, "loop_s": 0.5, "ref_s": 1.07, "cpus": 16})
    src = tmp_path / "recs.jsonl"
    src.write_text("".join(json.dumps(r) + "\n" for r in recs))
    md = tmp_path / "t.md"
    out = _run(os.path.join(TOOLS, "ref_tables.py"), "report", str(src), "--md", str(md))
    counts = [l for l in out.splitlines() if "faster in" in l]
    assert counts == ["MI355X faster in 0 of 6 cells.", "MI355X faster in 4 of 6 cells."]
    assert "**0.070 / 0.076**" in out and "| 0.070 / 0.068 |" in out
    assert "1900×" in out  # 0.19 / 0.0001
    assert "**0.500 / 1.07**" in out
    assert md.read_text() == out
