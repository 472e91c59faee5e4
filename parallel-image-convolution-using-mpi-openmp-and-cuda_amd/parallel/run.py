"""Per-rank program for ``torch.distributed.run`` — the ``mpiexec -n P
./mpi_convolution image W H reps {grey,rgb}`` of this framework.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 -m pconv.parallel.run image.raw W H reps rgb [options]

Reference flow (``mpi/mpi_convolution.c``): every rank parses argv
(``Usage`` ``:328-348``; the 6 ``MPI_Bcast`` of ``:65-70`` are unnecessary
because every rank sees the same argv), computes its block (``:72-73``),
reads only that block with MPI-IO (``:126-140``), runs the halo-exchange loop
between ``MPI_Barrier`` + ``MPI_Wtime`` (``:151-242``), writes its block into
``blur_<image>`` (``:244-262``) and rank 0 prints the max loop time over
ranks as ``"%f\\n"`` (``:264-275``).

Here a rank owns a contiguous row band (any H >= N, remainders to the first
ranks), ``pread``s only its rows (plus, by default, its ghost rows — a free
read that removes the first exchange; ``--exchange-halo`` reads owned rows
only), runs the band on its GPU (``--backend hip``: native ``BandEngine``,
RCCL halos over xGMI, interior compute overlapped with the exchange) or on
the CPU (``--backend omp``: the same C++ schedule on NumPy frames with gloo
halos — the reference's MPI+OpenMP hybrid), ``pwrite``s its band into the
pre-sized output (created with ``O_TRUNC`` by rank 0) and reports the max loop
time.  ``--check`` compares the written file with the CPU oracle on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List, Optional

import numpy as np

from .._native import require_native
from ..models.filters import get_filter, list_filters
from ..utils.raw_io import output_path_for

_CH = {"grey": 1, "rgb": 3, "rgba": 4}


def omp_team_size(threads: int, cpus, default_threads: int, local_world: int, env=None) -> int:
    """OpenMP team of one CPU rank (the OpenMP program's threads per MPI
    process, open-mp/omp_convolution.c:292,297).  Precedence: --threads; an
    explicit OMP_NUM_THREADS; the CPUs the rank is bound to; the node's budget
    split over the local ranks.  torch.distributed.run exports
    OMP_NUM_THREADS=1 to every worker of a multi-process launch when the user
    did not set it, so "1" under such a launch is taken as injected (and the
    override reported on stderr); any other value is the user's and wins."""
    env = os.environ if env is None else env
    if threads:
        return int(threads)
    v = env.get("OMP_NUM_THREADS", "")
    injected = v.strip() == "1" and local_world > 1 and "TORCHELASTIC_RUN_ID" in env
    if v.strip().isdigit() and int(v) > 0 and not injected:
        return int(v)
    n = len(cpus) if cpus else max(1, default_threads // max(1, local_world))
    if injected and n != 1:
        print(f"pconv: OMP_NUM_THREADS=1 set by torch.distributed.run ignored: {n} OpenMP threads per rank "
              "(--threads sets the team)", file=sys.stderr)
    return n


def usage(prog: str) -> str:
    # Same text as the reference (mpi/mpi_convolution.c:344) and the native CLI.
    return f"Error Input!\n{prog} image_name width height repetitions [rgb/grey].\n"


def parse(argv: List[str]) -> argparse.Namespace:
    prog = "pconv.parallel.run"
    if len(argv) < 5 or argv[4] not in _CH:
        sys.stderr.write(usage(prog))
        raise SystemExit(1)
    p = argparse.ArgumentParser(prog=prog, description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("image")
    p.add_argument("width", type=int)
    p.add_argument("height", type=int)
    p.add_argument("reps", type=int)
    p.add_argument("channels", choices=sorted(_CH))
    p.add_argument("--backend", choices=["hip", "omp", "cpu"], default="hip")
    p.add_argument("--filter", default="gaussian", choices=list_filters())
    p.add_argument("--halo", type=int, default=None, help="ghost rows exchanged at once (default: auto)")
    p.add_argument("--fuse", type=int, default=None, help="repetitions per kernel launch (default: auto)")
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--transport", choices=["rccl", "gloo-host"], default="rccl")
    p.add_argument("--threads", type=int, default=0,
                   help="--backend omp: OpenMP threads per rank (default: the rank's CPU slice, i.e. the node's "
                        "CPU budget / ranks on the node)")
    p.add_argument("--exchange-halo", action="store_true", help="read owned rows only; ghost rows from neighbours")
    p.add_argument("--out", default=None)
    p.add_argument("--synthetic", type=int, default=None, metavar="SEED")
    p.add_argument("--check", action="store_true")
    p.add_argument("--json", action="store_true")
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--timeout", type=float, default=600.0, help="RCCL watchdog (seconds) on the halo waits")
    p.add_argument("--checkpoint-every", type=int, default=0, metavar="K",
                   help="every K repetitions write the whole image to <out>.rep<N> (each rank pwrites its band); "
                        "resume = rerun on that file with the remaining repetitions")
    p.add_argument("--cpu-bind", action="store_true",
                   help="--backend cpu/omp: bind each rank to its own CPU slice (off by default: unbound teams "
                        "were steadier on a shared host, profiles/r03/hybrid/)")
    p.add_argument("--no-numa-bind", action="store_true",
                   help="--backend hip: leave each rank's CPU affinity alone (default: the GPU's NUMA node)")
    a = p.parse_args(argv)
    if a.width < 1 or a.height < 1 or a.reps < 0 or a.checkpoint_every < 0:
        sys.stderr.write(usage(prog))
        raise SystemExit(1)
    return a


class _HipBand:
    """One band on this rank's GPU (native BandEngine + RCCL / gloo-host halos)."""

    def __init__(self, a, rank, world, device):
        n = require_native()
        from .dist_engine import auto_halo

        nf = get_filter(a.filter).to_native()
        frame = a.width * _CH[a.channels] * (a.height // max(1, world))
        fuse = a.fuse if a.fuse is not None else n.auto_fuse(nf, "auto", frame, _CH[a.channels])
        halo = a.halo if a.halo is not None else auto_halo(a.height, world, a.reps, fuse)
        self.eng = n.BandEngine(a.width, a.height, a.channels, nf, rank, world, device, halo=int(halo),
                                fuse=int(fuse), overlap=not a.no_overlap)
        self.band, self.halo, self.fuse = self.eng.band, self.eng.halo, self.eng.fuse
        self.comm = self.transport = None
        self.timeout_s = float(a.timeout)
        if world > 1:
            if a.transport == "rccl":
                from .bootstrap import make_rccl_comm

                self.comm = make_rccl_comm(device)
                self.eng.attach_rccl(self.comm)
            else:
                from .transports import GlooHostTransport

                self.transport = GlooHostTransport()
                self.eng.attach_transport(self.transport)

    def load(self, rows: np.ndarray, r0: int, r1: int, halo_valid: bool) -> None:
        self.eng.upload(rows.reshape(-1), r0, r1)
        self.eng.set_halo_valid(halo_valid)
        self.eng.synchronize()

    def run(self, reps: int) -> None:
        self.eng.run(reps)
        if self.comm is not None:  # poll RCCL errors; abort + raise instead of hanging on a dead peer
            self.comm.wait(self.eng.comm_stream, self.timeout_s)
            self.comm.wait(self.eng.compute_stream, self.timeout_s)
        self.eng.synchronize()

    def result(self, out: np.ndarray) -> None:
        self.eng.download(out.reshape(-1), 0, self.band.rows)
        self.eng.synchronize()

    @property
    def counts(self):
        """(launches, exchanges) of the LAST run() (the caller sums chunks)."""
        s = self.eng.stats
        return int(s.launches), int(s.exchanges)


class _CpuBand:
    """One band on the CPU (MPI+OpenMP analog): the same C++ schedule, gloo halos."""

    def __init__(self, a, rank, world, omp):
        from .cpu_dist import CpuBandRunner
        from .dist_engine import auto_halo

        fuse = a.fuse if a.fuse is not None else 1
        halo = a.halo if a.halo is not None else auto_halo(a.height, world, a.reps, fuse)
        self.r = CpuBandRunner(a.width, a.height, a.channels, a.filter, rank=rank, world=world, halo=halo, fuse=fuse,
                               overlap=not a.no_overlap, omp=omp)
        self.band, self.halo, self.fuse = self.r.band, self.r.halo, self.r.fuse
        self._preloaded = False

    def load(self, rows: np.ndarray, r0: int, r1: int, halo_valid: bool) -> None:
        b = self.band
        rows = rows.reshape(r1 - r0, -1)
        self.r.load(rows[-r0 : -r0 + b.rows])
        if r0 < 0:
            self.r._rows_view(self.r.frames[0], r0, 0)[:] = rows[: -r0]
        if r1 > b.rows:
            self.r._rows_view(self.r.frames[0], b.rows, r1)[:] = rows[-r0 + b.rows :]
        self._preloaded = halo_valid

    def run(self, reps: int) -> None:
        before = self.r.exchanges
        self.r.run(reps, halo_preloaded=self._preloaded)
        self._last_exchanges = self.r.exchanges - before
        self._preloaded = False  # a later run (after a checkpoint) exchanges its ghost rows

    def result(self, out: np.ndarray) -> None:
        out.reshape(self.band.rows, -1)[:] = self.r.result()

    @property
    def counts(self):
        """(launches, exchanges) of the LAST run() (the caller sums chunks)."""
        return 0, int(getattr(self, "_last_exchanges", 0))


def main(argv: Optional[List[str]] = None) -> int:
    a = parse(list(sys.argv[1:] if argv is None else argv))
    from .bootstrap import barrier, init_distributed, max_over_ranks, shutdown, sum_over_ranks

    n = require_native()
    ctx = init_distributed("gloo")
    rank, world = ctx.rank, ctx.world
    try:
        if a.height < world:
            raise SystemExit(f"image has fewer rows ({a.height}) than ranks ({world})")
        cpus = None
        if a.backend == "hip":
            device = ctx.local_rank % max(1, n.device_count())
            n.set_device(device)
            if world > 1 and not a.no_numa_bind:
                n.bind_to_device_numa(device)
            runner = _HipBand(a, rank, world, device)
        else:
            # the node's CPU budget split between the ranks on it (MPI+OpenMP
            # hybrid): each rank bound to its own slice, its team = the slice
            from .bootstrap import bind_cpu_rank

            local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
            cpus = bind_cpu_rank(ctx.local_rank, local_world, a.cpu_bind)
            if a.backend == "omp":
                n.set_cpu_threads(omp_team_size(a.threads, cpus, n.default_cpu_threads(), local_world))
            runner = _CpuBand(a, rank, world, omp=a.backend == "omp")
        b = runner.band
        rb = a.width * _CH[a.channels]
        preload = world > 1 and not a.exchange_halo
        above = min(runner.halo, b.y0) if preload else 0
        below = min(runner.halo, a.height - (b.y0 + b.rows)) if preload else 0
        rows = np.empty((b.rows + above + below) * rb, np.uint8)
        if a.synthetic is not None:
            n.synth_rows(rows, a.width, a.height, a.channels, int(a.synthetic), b.y0 - above, b.rows + above + below)
        else:
            n.read_raw_rows(a.image, rows, a.width, a.height, a.channels, b.y0 - above, b.rows + above + below)
        out_path = a.out or output_path_for(a.image)
        if rank == 0:
            n.create_output(out_path, a.width, a.height, a.channels)
        runner.load(rows, -above, b.rows + below, preload)

        # Checkpoints: the iteration is Markov in the image, so a checkpoint
        # is just the whole image after `done` repetitions (every rank pwrites
        # its band into <out>.rep<done>, pre-sized by rank 0).
        ce = a.checkpoint_every
        ck = [d for d in range(ce, a.reps, ce)] if ce > 0 else []
        if rank == 0:
            for d in ck:
                n.create_output(f"{out_path}.rep{d}", a.width, a.height, a.channels)
        res = np.empty(b.rows * rb, np.uint8)
        barrier()  # MPI_Barrier before MPI_Wtime (mpi_convolution.c:151-154)
        t0 = time.perf_counter()
        done = 0
        launches = exchanges = 0  # summed over checkpoint chunks (each run() reports its own)
        while done < a.reps or (done == 0 and a.reps == 0):
            k = min(ce, a.reps - done) if ce > 0 else a.reps
            runner.run(k)
            cl, cx = runner.counts
            launches += cl
            exchanges += cx
            done += k
            if done in ck:
                runner.result(res)
                n.write_raw_rows(f"{out_path}.rep{done}", res, a.width, a.height, a.channels, b.y0, b.rows)
            if a.reps == 0:
                break
        loop_s = time.perf_counter() - t0

        barrier()  # output file exists before any pwrite
        runner.result(res)
        n.write_raw_rows(out_path, res, a.width, a.height, a.channels, b.y0, b.rows)
        t_max = max_over_ranks(loop_s)
        barrier()
        mismatches = None
        if a.check:
            bad = 0
            if rank == 0:
                src = np.empty(a.height * rb, np.uint8)
                if a.synthetic is not None:
                    n.synth_rows(src, a.width, a.height, a.channels, int(a.synthetic), 0, a.height)
                else:
                    n.read_raw(a.image, src, a.width, a.height, a.channels)
                ref = np.empty_like(src)
                n.cpu_convolve(src, ref, a.width, a.height, a.channels, a.reps, get_filter(a.filter).to_native(),
                               True, 0)
                got = np.empty_like(src)
                n.read_raw(out_path, got, a.width, a.height, a.channels)
                bad = int(np.count_nonzero(got != ref))
            mismatches = sum_over_ranks(bad)
        if rank == 0:
            if not a.quiet:
                print(f"{t_max:f}", flush=True)  # reference format (mpi_convolution.c:274)
            if a.json:
                px = a.width * a.height * a.reps
                print(json.dumps({
                    "backend": a.backend, "ranks": world, "width": a.width, "height": a.height,
                    "channels": a.channels, "reps": a.reps, "filter": a.filter, "loop_s": t_max,
                    "mpix_per_s": px / t_max / 1e6 if t_max > 0 else 0.0, "halo": int(runner.halo),
                    "fuse": int(runner.fuse), "transport": (a.transport if a.backend == "hip" else "gloo") if world > 1 else None,
                    "preload_halo": preload, "launches": launches, "exchanges": exchanges, "output": out_path,
                    "mismatches": mismatches,
                    "rank0_cpus": len(cpus) if cpus is not None else None,
                    "omp_threads": n.cpu_threads() if a.backend == "omp" else None,
                }), flush=True)
        return 0 if not mismatches else 2
    finally:
        shutdown(ctx)


if __name__ == "__main__":
    sys.exit(main())
