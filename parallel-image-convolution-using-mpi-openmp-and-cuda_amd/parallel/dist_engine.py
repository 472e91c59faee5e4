"""Per-rank distributed engine: one row band on one GPU, RCCL halos.

The MPI rank of the reference (``mpi/mpi_convolution.c:72-240``) owns a 2-D
block, reads it with MPI-IO, exchanges depth-1 halos with <=4 neighbours per
rep and times the loop.  Here a rank owns a contiguous row band
(``native.row_band``), its input rows arrive in pinned host memory (from the
image, a file band read, or the synthetic generator), and the native
``BandPipeline`` runs ``upload -> reps -> download`` per image without
returning to Python, with halo rows moved by the native RCCL transport on a
communication stream, overlapped with interior compute.  With ``slots > 1``
consecutive images overlap (H2D of the next, compute of the current, D2H of
the previous: a serving pipeline).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .._native import require_native
from ..models.filters import get_filter
from .bootstrap import env_context, make_rccl_comm

AUTO_HALO_CAP = 64


def auto_halo(height: int, world: int, reps: Optional[int], fuse: int, preload: bool = False) -> int:
    """Deep ghost zone: one exchange per `halo` reps, capped so the redundant
    ghost-row compute stays small and the band can supply it.

    preload: the ghost rows are uploaded with the band and never exchanged,
    so the zone must cover ALL `reps` (a 200-rep run needs 200 ghost rows per
    side; the redundant compute is the shrinking trapezoid, ~reps^2/fuse rows
    per image — 5 % of a 4096-row band at 200 reps).  Bands shorter than
    `reps` cannot supply that: they get the exchange cap and need a transport.
    """
    if world <= 1:
        return fuse
    band = height // world
    if preload and reps and int(reps) <= band:
        return max(int(reps), fuse, 1)
    d = min(AUTO_HALO_CAP, band)
    if reps:
        d = min(d, int(reps))
    return max(d, fuse, 1)


def preload_is_exchange_free(height: int, world: int, reps: int) -> bool:
    """True when pre-loaded ghost rows can carry all `reps` (every band is at
    least `reps` rows tall), so a run needs no halo transport at all."""
    return world <= 1 or int(reps) <= height // world


def pcie_bytes_per_image(width: int, height: int, channels: str, world: int, rank: int, halo: int,
                         preload: bool) -> tuple:
    """(H2D, D2H) bytes one rank moves per image: its band plus, when the
    ghost rows are pre-loaded, `halo` rows per side clipped at the image
    edges in; its owned rows out.  The bench JSON reports them per rank
    (h2d_bytes_per_step / d2h_bytes_per_step): at N = 8 pre-loading 40 ghost
    rows per side makes an interior rank's H2D 25 % larger than its band."""
    rb = int(width) * {"grey": 1, "rgb": 3, "rgba": 4}[channels]
    base, rem = divmod(int(height), int(world))
    rows = base + (1 if rank < rem else 0)
    y0 = rank * base + min(rank, rem)
    above = min(int(halo), y0) if preload and world > 1 else 0
    below = min(int(halo), int(height) - (y0 + rows)) if preload and world > 1 else 0
    return (rows + above + below) * rb, rows * rb


class DistributedBlur:
    def __init__(self, width: int, height: int, channels: str = "grey", filter="gaussian",
                 reps: Optional[int] = None, *, rank: Optional[int] = None, world: Optional[int] = None,
                 device: Optional[int] = None, halo: Optional[int] = None, fuse: Optional[int] = None,
                 overlap: bool = True, preload_halo: bool = False, comm=None, slots: int = 2,
                 variant: str = "auto", graph: bool = False, transport: str = "rccl", concurrent: int = -1,
                 step_graphs: Optional[bool] = None, graph_capture: bool = True, slot_exchange: bool = False,
                 self_neighbours: bool = False, slot_comm: bool = False, stream_chunks: int = 0,
                 ipc_timeout_s: float = 30.0, ipc_pull: str = "grid", cu_mask_queues: bool = True,
                 head_on_slot_streams: bool = True, stream_min_bytes: Optional[int] = None,
                 head_alt_uploads: bool = True, qualify_staging: bool = True, flush_staging: bool = True,
                 stream_weights: Optional[Sequence[int]] = None, lazy_head: Optional[bool] = None):
        """Pipeline policy (native EngineOptions, echoed by bench.py's JSON
        config): `cu_mask_queues` puts every slot stream on its own hardware
        queue; `head_on_slot_streams` runs a streamed head image's copies on
        the next slots' streams and `head_alt_uploads` alternates its chunk
        uploads over two of them (>= 4 slots); `stream_min_bytes` (None: the
        native default, 8 MiB) is the smallest input head-streamed;
        `stream_weights` (one per chunk; sets the chunk count) sizes the
        streamed chunks (None: the native default, schedule.hpp stream_cuts);
        `lazy_head` holds a burst's first image back until the next submit
        (then a step graph) or drain (then row-streamed) (None: native default);
        `ipc_pull` is the IPC transport's pull form (grid | single | sdma,
        ipc_halo.hpp).  `qualify_staging`: time every slot's pinned staging
        buffers through the copy engines once and replace any that copies
        slower than the best (see _qualify_staging).  `flush_staging`: after
        the CPU writes input rows into the pinned buffers (load_*), clflush
        them out of every CPU cache — the copy engines' reads of lines left
        dirty in the caches of the cores that wrote them (the OpenMP writers
        of load_synthetic) ran that buffer's uploads 5-15 % slower for the
        life of the process (profiles/r06/e/)."""
        n = require_native()
        ctx = env_context()
        self.rank = ctx.rank if rank is None else int(rank)
        self.world = ctx.world if world is None else int(world)
        self.device = ctx.local_rank if device is None else int(device)
        self.width, self.height, self.channels = int(width), int(height), channels
        nf = get_filter(filter).to_native()
        if fuse is None:
            ch = {"grey": 1, "rgb": 3, "rgba": 4}[channels]
            fuse = n.auto_fuse(nf, variant, self.width * ch * (self.height // max(1, self.world)), ch)
        if halo is None:
            halo = auto_halo(self.height, self.world, reps, fuse, preload=bool(preload_halo) and not slot_exchange)
        # stream_chunks > 1: each exchange-free image's rows are uploaded in
        # that many chunks and its levels advance behind them (H2D, launches
        # and D2H of ONE image overlap; schedule.hpp plan_streamed)
        if stream_weights:
            stream_chunks = len(stream_weights)
        kw = dict(halo=int(halo), fuse=int(fuse), overlap=bool(overlap), variant=variant, slots=int(slots),
                  concurrent=int(concurrent), stream_chunks=int(stream_chunks),
                  cu_mask_queues=bool(cu_mask_queues), head_on_slot_streams=bool(head_on_slot_streams),
                  head_alt_uploads=bool(head_alt_uploads),
                  stream_weights=[int(w) for w in (stream_weights or [])],
                  **({} if lazy_head is None else {"lazy_head": bool(lazy_head)}),
                  **({} if stream_min_bytes is None else {"stream_min_bytes": int(stream_min_bytes)}))
        if self_neighbours:
            # One-GPU emulation of rank `rank` of a `world`-way split whose halos
            # really move: its neighbours are replaced by itself (a 1-rank
            # communicator, RCCL send/recv to self), so every exchange costs
            # what it costs (kernels, latency, host calls) while the ghost
            # CONTENT is not its neighbours' (timing only; bytes not checked).
            b = n.row_band(self.height, self.world, self.rank)
            b.up = 0 if b.up >= 0 else -1
            b.down = 0 if b.down >= 0 else -1
            b.rank, b.world = 0, 1
            kw["band"] = b
        self.pipe = n.BandPipeline(self.width, self.height, channels, nf, self.rank, self.world, self.device, **kw)
        self.preload_halo = bool(preload_halo) and self.world > 1
        # Whole-step graphs (one host call per image, slots on their own
        # streams) whenever the images need no halo exchange: one band, or
        # ghost rows pre-loaded deep enough for all `reps`.
        free = reps is not None and self.pipe.slot(0).exchange_free(int(reps), self.preload_halo)
        if self.world > 1 and transport == "none" and not free:
            raise ValueError(f"transport 'none' needs exchange-free images: {reps} reps with a "
                             f"{self.pipe.slot(0).halo}-row ghost zone (preload_halo={self.preload_halo}) exchange "
                             "halos; use transport rccl/gloo-host")
        if step_graphs and not free and not slot_exchange:
            raise ValueError("step_graphs needs exchange-free images (world 1, or preload_halo with halo >= reps)")
        # slot_exchange: images that DO exchange halos, each on its slot's own
        # stream with its own transport (one RCCL communicator per slot), the
        # exchange in stream order between upload and launches — slots overlap
        # each other instead of the exchange overlapping its own image.
        self.slot_exchange = bool(slot_exchange) and self.world > 1
        if transport == "ipc" and self.world > 1 and not free and not self.slot_exchange:
            raise ValueError("transport 'ipc' exchanges per slot: use slot_exchange=True (one transport per slot)")
        if self.slot_exchange and transport not in ("rccl", "ipc"):
            graph_capture = False  # host-staged transports synchronise: they cannot be captured
        # With RCCL, an exchange image is ONE captured graph (upload, ncclSend/
        # ncclRecv of the ghost zone, launches, download): one host call per
        # image instead of the transport's group calls + launches + copies.
        # stream_chunks > 1 with step_graphs=False: EVERY image row-streamed,
        # issued directly on shared H2D / compute / D2H streams (the
        # event-ordered pipeline; captured as one graph with fork/join
        # branches a streamed image measured 1.4-4.3x slower,
        # profiles/r04/stream_a/).  Otherwise (step graphs): only an image
        # submitted to an idle pipeline is streamed — the head of a burst,
        # every single image — and the rest run as one graph each.
        streamed = int(stream_chunks) > 1 and free and not self.slot_exchange and step_graphs is False
        if not streamed and (self.slot_exchange or (free if step_graphs is None else bool(step_graphs))):
            del self.pipe
            # slot_comm (exchange images): each slot also gets a communication
            # stream, so an exchange phase runs beside the interior launch and
            # the edges follow the halo event — captured, the reference's per-
            # phase loop becomes ONE graph per image.
            self.pipe = n.BandPipeline(self.width, self.height, channels, nf, self.rank, self.world, self.device,
                                       graphs=True, step_graphs=bool(graph_capture),
                                       slot_comm=bool(slot_comm) and self.slot_exchange, **kw)
        self.engine = self.pipe.slot(0)
        self.band = self.engine.band
        self.row_bytes = self.engine.row_bytes
        d = self.engine.halo
        b = self.band
        self.above = min(d, b.y0) if self.preload_halo else 0
        self.below = min(d, self.height - (b.y0 + b.rows)) if self.preload_halo else 0
        in_rows = b.rows + self.above + self.below
        self.slots = int(slots)
        # one pinned input/output buffer per slot (in-flight images never share)
        self._in = [n.PinnedBuffer(in_rows * self.row_bytes) for _ in range(self.slots)]
        self._out = [n.PinnedBuffer(b.rows * self.row_bytes) for _ in range(self.slots)]
        self.staging = None
        if qualify_staging:
            self.staging = self._qualify_staging(in_rows)
        self.inputs = [np.asarray(x).reshape(in_rows, self.row_bytes) for x in self._in]
        self.outputs = [np.asarray(x).reshape(b.rows, self.row_bytes) for x in self._out]
        self.input, self.output = self.inputs[0], self.outputs[0]
        self.flush_staging = bool(flush_staging)
        self._next = 0
        self._pending = False  # submitted images not yet drained
        self.comm = None
        self.transport = None
        self.slot_comms = []
        self.slot_transports = []
        self.ipc = []
        if self.slot_exchange and transport == "ipc":
            # device-side pulls of the neighbours' rows through HIP IPC, ordered
            # by flag kernels (ipc_halo.hpp); one transport per slot
            from .bootstrap import make_ipc_transports

            self.ipc = make_ipc_transports([self.pipe.slot(k) for k in range(self.slots)], ipc_timeout_s,
                                           pull=ipc_pull)
            for k, t in enumerate(self.ipc):
                self.pipe.attach_slot_transport(k, t)
        elif self.slot_exchange:
            for k in range(self.slots):
                if transport == "rccl":
                    c = make_rccl_comm(self.device)
                    self.slot_comms.append(c)
                    self.pipe.attach_slot_rccl(k, c)
                elif transport == "gloo-host":
                    from .transports import GlooHostTransport

                    t = GlooHostTransport()
                    self.slot_transports.append(t)
                    self.pipe.attach_slot_transport(k, t)
                else:
                    raise ValueError(f"slot_exchange needs transport rccl, ipc or gloo-host, not {transport!r}")
            self.comm = self.slot_comms[0] if self.slot_comms else None
        elif self.world > 1 and transport not in ("none", "ipc"):  # exchange-free images need none
            if transport == "rccl":
                self.comm = comm if comm is not None else make_rccl_comm(self.device)
                self.pipe.attach_rccl(self.comm)
            elif transport == "gloo-host":
                from .transports import GlooHostTransport

                self.transport = GlooHostTransport()
                self.pipe.attach_transport(self.transport)
            else:
                raise ValueError(f"unknown transport {transport!r} (rccl|ipc|gloo-host|none)")

    def _qualify_staging(self, in_rows: int, tolerance: float = 1.05, attempts: int = 3) -> dict:
        """Pinned staging buffers are not all equal: measured on MI355X
        boxes, in some processes ONE slot's input buffer uploaded at ~42
        instead of ~55 GB/s (0.342 vs 0.263 ms for the headline image, alone
        on the link) and that slot's images paced the whole pipeline —
        the slow mode of the driver's 20-image window (profiles/r06/).  So
        every slot's buffers go through the copy engines once (H2D alone,
        D2H alone: copy_floor_on), and a buffer more than `tolerance` slower
        than the best of its direction — over the slots AND a freshly
        allocated pair, since in one process every slot's output buffer ran
        D2H at 0.41 ms against 0.26 for fresh buffers (profiles/r06/aa/
        drv_0.json) — is replaced by a fresh allocation —
        the rejected ones stay allocated until the search ends, so the
        allocator cannot hand the same pages back — up to `attempts` rounds.
        Set-up only (before any image is loaded); returns what it measured."""
        n = require_native()
        rb, out_rows = self.row_bytes, self.band.rows

        def rates():
            return [n.copy_floor_on(self.device, self._in[k].ptr, self._out[k].ptr, rb, in_rows, out_rows, 4)
                    for k in range(self.slots)]

        held, first, replaced = [], rates(), 0
        fresh = n.copy_floor_on(self.device, 0, 0, rb, in_rows, out_rows, 4)
        now = first
        for _ in range(attempts):
            best_h, best_d = min([fresh[0]] + [r[0] for r in now]), min([fresh[1]] + [r[1] for r in now])
            bad_in = [k for k, r in enumerate(now) if r[0] > tolerance * best_h]
            bad_out = [k for k, r in enumerate(now) if r[1] > tolerance * best_d]
            if not bad_in and not bad_out:
                break
            for k in bad_in:
                held.append(self._in[k])
                self._in[k] = n.PinnedBuffer(in_rows * rb)
            for k in bad_out:
                held.append(self._out[k])
                self._out[k] = n.PinnedBuffer(out_rows * rb)
            replaced += len(bad_in) + len(bad_out)
            now = rates()
        del held
        r4 = lambda v: [[round(x, 4) for x in r] for r in v]  # noqa: E731
        return {"h2d_d2h_pair_ms_first": r4(first), "h2d_d2h_pair_ms": r4(now), "fresh_ms": r4([fresh])[0],
                "replaced": replaced}

    # ------------------------------------------------------------ inputs
    @property
    def h2d_bytes_per_image(self) -> int:
        """Host-to-device bytes this rank moves per image: its band plus the
        pre-loaded ghost rows (exchange modes upload only the band)."""
        a, b = self.input_rows
        return (b - a) * self.row_bytes

    @property
    def d2h_bytes_per_image(self) -> int:
        """Device-to-host bytes per image: the owned rows."""
        return self.band.rows * self.row_bytes

    @property
    def input_rows(self):
        """Global rows [first, last) held by the pinned input buffers."""
        return self.band.y0 - self.above, self.band.y0 + self.band.rows + self.below

    def _quiesce(self) -> None:
        # Images in flight read the pinned inputs asynchronously: never
        # rewrite an input buffer under them.
        if self._pending:
            self.drain()

    def _flushed(self, slots) -> None:
        """flush_staging: the input rows the CPU just wrote leave every CPU
        cache, so the copy engines' reads of them never fetch dirty lines from
        the cores that wrote them."""
        if self.flush_staging:
            n = require_native()
            for i in slots:
                n.flush_host_cache(self._in[i].ptr, len(self._in[i]))

    def load_image(self, image: np.ndarray, slot: Optional[int] = None) -> None:
        self._quiesce()
        a, b = self.input_rows
        rows = np.ascontiguousarray(image, dtype=np.uint8).reshape(self.height, self.row_bytes)[a:b]
        for i in ([slot] if slot is not None else range(self.slots)):
            self.inputs[i][:] = rows
        self._flushed([slot] if slot is not None else range(self.slots))

    def load_file(self, path: str) -> None:
        self._quiesce()
        a, b = self.input_rows
        require_native().read_raw_rows(path, self.inputs[0].reshape(-1), self.width, self.height, self.channels, a,
                                       b - a)
        for i in range(1, self.slots):
            self.inputs[i][:] = self.inputs[0]
        self._flushed(range(self.slots))

    def load_synthetic(self, seed: int = 0) -> None:
        self._quiesce()
        a, b = self.input_rows
        require_native().synth_rows(self.inputs[0].reshape(-1), self.width, self.height, self.channels, int(seed),
                                    a, b - a)
        for i in range(1, self.slots):
            self.inputs[i][:] = self.inputs[0]
        self._flushed(range(self.slots))

    # ------------------------------------------------------------ compute
    def submit(self, reps: int) -> int:
        """Enqueue one image (slot round-robin); returns the slot whose output
        buffer will hold the result after drain()."""
        k = self._next
        # An IPC wait that timed out (a stalled or vanished neighbour) is final:
        # no further image — no graph replay whose copies might read a gone
        # neighbour's frames (the sdma form) — is issued once it is set.  A
        # read of host-mapped memory, no device synchronisation.
        for t in self.ipc:
            t.check()
        self.pipe.submit(self._in[k].ptr, -self.above, self.band.rows + self.below, self._out[k].ptr, int(reps))
        self._next = (k + 1) % self.slots
        self._pending = True
        return k

    def drain(self, timeout_s: Optional[float] = None) -> None:
        """Wait for every submitted image.  With per-slot RCCL communicators
        and a timeout, each slot's stream is polled for RCCL asynchronous
        errors and the communicator aborted (raising) if it does not finish."""
        if timeout_s is not None and self.slot_comms:
            for k, c in enumerate(self.slot_comms):
                c.wait(self.pipe.slot(k).compute_stream, float(timeout_s))
        self.pipe.drain()
        for t in self.ipc:
            t.check()  # a timed-out device-side wait (a stalled neighbour) raises here
        self._pending = False

    def step(self, reps: int) -> np.ndarray:
        """Synchronous: one image through H2D + reps + D2H; returns its rows."""
        k = self.submit(reps)
        self.drain()
        self.output = self.outputs[k]
        return self.output

    @property
    def stats(self):
        return self.engine.stats

    def plan(self, reps: int):
        return self.engine.plan(reps)

    def write_band(self, path: str, slot: int = 0) -> None:
        """pwrite the owned rows into an existing, pre-sized output file."""
        require_native().write_raw_rows(path, self.outputs[slot].reshape(-1), self.width, self.height,
                                        self.channels, self.band.y0, self.band.rows)
