#!/usr/bin/env python3
"""Headline benchmark: 1920x2520 RGB, 40 repetitions of the 3x3 gaussian.

BASELINE.json metric: "Mpixels/sec (and wall-time) for 1920x2520 RGB, 40 reps
at 1/2/4/8 MI355X".  The reference's headline number is the CUDA program's
end-to-end time for that run on a GTX 970, 1.017 s = 190.3 Mpix/s
(README.pdf p.7); its GPU work is GPU_convolution()
(cuda/cuda_convolution.cu:49-102): H2D of the image, `reps` kernels, D2H.

One benchmark STEP here is that same unit of work for one image: H2D of the
image (pinned host memory), 40 repetitions, D2H of the result.  With N GPUs
(one process per GPU, launched by torch.distributed.run) the image is split
into N row bands (strong scaling: the image and the total work are fixed);
each rank uploads only its band and downloads only its band.  Ghost rows:
  --halo-mode preload (default): each rank also uploads `reps` ghost rows per
      side with its band (communication-avoiding: the ghost zone is deep
      enough for all 40 repetitions, no exchange at all), and every image is
      ONE hipGraph (H2D + 5 fused launches + D2H) on its slot's own stream;
  --halo-mode exchange: ghost rows move GPU-to-GPU with RCCL ncclSend/Recv
      over xGMI on a communication stream, overlapped with interior compute
      (event-ordered streams; the reference's MPI_Isend/Irecv loop).
For N>1 the JSON line also carries "halo_modes": after the headline's timed
region, the same images run through each halo mode that moves ghost rows
GPU-to-GPU (RCCL over xGMI; see HALO_MODES below: slot_exchange, event, and
overlap = the reference's Isend/Irecv + inner compute + Wait + edges loop),
each timed with the same K steps, barriers and syncs as the headline, with
its bytes compared against the headline's result.  The halo mode is then
chosen by measurement (--halo-select auto): the fastest bit-exact mode is
reported as the headline when it is at least 3 % faster than the pre-loaded
pipeline ("halo_select" names the choice and every candidate's ms/step).
The measurement is bounded by --exchange-timeout per drain and a watchdog,
so a stalled peer can never take the headline line down with it.
Measured on one GPU (tools: --emulate), preload is the faster per-rank step:
the 40-row ghost zone costs ~25% more H2D at N=8, the exchange path costs
more host API calls and RCCL latency per image.  In preload mode the headline
pipeline holds no communicator at all (its images are exchange-free); the
elapsed time is reduced with a gloo all-reduce (max over ranks, the
reference's MPI_Send/Recv max-gather).
The JSON names the runtime actually loaded ("runtime": HIP runtime version
and library path, RCCL version and library path): under torch, librccl and
the HIP runtime resolve to torch's bundled copies.
value = W*H*reps*steps / max-over-ranks elapsed / 1e6 (whole-job Mpix/s).
Extra fields report the device-resident loop alone (no PCIe copies) and the
box's PCIe floor: each copy alone and, as `copy_floor.pair_ms`, one pitched
H2D + one pitched D2H of a step issued together — what a PCIe-bound step
converges to (e.g. 0.309 ms per pair vs a 0.318 ms step at N=1).

Data: synthetic random bytes (no image ships with the reference).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_MPIX = 190.3  # CUDA 1920x2520 RGB 40 reps end-to-end, GTX 970
METRIC = "Mpixels/sec (and wall-time) for 1920x2520 RGB, 40 reps at 1/2/4/8 MI355X"
HEADLINE = (1920, 2520, "rgb", 40)


def metric_for(a) -> str:
    """BASELINE.json's metric string for the headline config; the same form
    with this run's geometry otherwise (never a mislabelled headline)."""
    if (a.width, a.height, a.channels, a.reps) == HEADLINE and a.filter == "gaussian":
        return METRIC
    f = "" if a.filter == "gaussian" else f" {a.filter}"
    return f"Mpixels/sec (and wall-time) for {a.width}x{a.height} {a.channels.upper()}, {a.reps} reps{f} " \
           "at 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=2520)
    p.add_argument("--channels", default="rgb")
    p.add_argument("--reps", type=int, default=40)
    p.add_argument("--filter", default="gaussian")
    p.add_argument("--fuse", type=int, default=None)
    p.add_argument("--halo", type=int, default=None)
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--halo-mode", choices=["preload", "exchange"], default="preload",
                   help="N>1 ghost rows: uploaded with the band (preload) or exchanged with RCCL (exchange)")
    p.add_argument("--preload-halo", action="store_true", help="alias of --halo-mode preload")
    p.add_argument("--loop-steps", type=int, default=None, help="timed device-resident loops (default = --steps)")
    p.add_argument("--variant", default="auto")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--slots", type=int, default=None,
                   help="images in flight (default 4: slot streams on CU-masked queues; 4 beat 3 on the 8-way "
                        "per-rank proxy in every halo mode and tie at N=1, profiles/r04/e2/, final_b/)")
    p.add_argument("--concurrent", choices=["auto", "on", "off"], default="off",
                   help="one compute stream per image in flight (default: one shared compute stream)")
    p.add_argument("--transport", choices=["rccl", "gloo-host"], default="rccl",
                   help="halo transport (gloo-host: host-staged, lets several ranks share one GPU for rehearsals)")
    p.add_argument("--step-graphs", choices=["auto", "on", "off"], default="auto",
                   help="one hipGraph per image (H2D + reps + D2H) on per-slot streams (auto: when exchange-free)")
    p.add_argument("--graph-capture", choices=["on", "off"], default="on",
                   help="slot-stream pipeline: capture each image as a hipGraph (on) or issue directly (off)")
    p.add_argument("--stream-chunks", type=int, default=4,
                   help="rows streamed within each image: upload in this many row chunks, advance every level behind "
                        "them, download finished rows meanwhile (H2D, reps and D2H of ONE image overlap; 0 = off). "
                        "With step graphs only an image submitted to an idle pipeline is streamed, and with "
                        "--lazy-head (default) only when no second image follows before the drain: every single "
                        "image (latency_ms 0.53 vs 0.69 ms whole-image)")
    p.add_argument("--stream-weights", default=None, metavar="W1,W2,...",
                   help="relative rows of each streamed chunk (sets the chunk count; default 5,...,5,6)")
    p.add_argument("--lazy-head", choices=["on", "off"], default=None,
                   help="hold a burst's first image until the next submit (step graph) or drain (row-streamed); "
                        "default (native) on: window 0.3290 vs 0.3315 ms/step median, profiles/r06/z/")
    p.add_argument("--head-one-upload-stream", dest="head_alt_uploads", action="store_false", default=True,
                   help="streamed head image: all chunk uploads on one slot's stream (default with >= 4 slots: "
                        "alternating over two, one image 0.546-0.549 vs 0.559-0.568 ms, profiles/r05/l/)")
    p.add_argument("--stream-min-mb", type=float, default=8.0,
                   help="head-stream only images of at least this many MiB of input: below it the hand-offs of a "
                        "streamed image cost more than they hide (N=4 band 0.32 vs 0.23 ms as one graph, N=8 0.28 "
                        "vs 0.15; N=1 0.58 vs 0.68: profiles/r05/e/burst.jsonl)")
    p.add_argument("--emulate", default=None, metavar="WORLD:RANK",
                   help="time ONE rank of a WORLD-way split on this GPU (pre-loaded halos, no peers): a "
                        "single-GPU proxy of the per-rank step; reported as emulated, never as the headline")
    p.add_argument("--emulate-halo", default="preload", choices=("preload",) + HALO_MODES,
                   help="with --emulate: the halo mode of the emulated rank; an exchange mode replaces the rank's "
                        "neighbours by itself (1-rank RCCL communicator, send/recv to self: real exchange costs, "
                        "ghost contents not checked)")
    p.add_argument("--emulate-rccl", action="store_true",
                   help="with --emulate: also hold a 1-rank RCCL communicator during the timed region (its "
                        "streams and queues, as a real N>1 rank has)")
    p.add_argument("--exchange-check", choices=["auto", "on", "off"], default="auto",
                   help="N>1: after the headline timing, also time the halo modes of --halo-modes (ghost rows "
                        "moved GPU-to-GPU) with the same K steps, and compare their bytes with the headline "
                        "result; reported under 'halo_modes' (auto: on for N>1)")
    p.add_argument("--halo-modes", default=",".join(HALO_MODES),
                   help="comma list of the halo modes timed after the headline at N>1: " + ", ".join(HALO_MODES))
    p.add_argument("--exchange-timeout", type=float, default=30.0, help="seconds before a mode's drain aborts")
    p.add_argument("--resident-loop", choices=["on", "off"], default="on",
                   help="N>1, halo modes 'event' and 'ipc': also time the reference's MPI loop on the resident bands "
                        "(reps with the ghost rows exchanged every halo-depth reps through RCCL / HIP-IPC, no PCIe), "
                        "reported as halo_modes.<mode>.resident_loop, resident_loop and resident_loop_ipc")
    p.add_argument("--resident-overlap", choices=["on", "off"], default="off",
                   help="resident loop: split each exchange phase into the interior launch beside the exchange and "
                        "the edge strips after it, captured as ONE graph with a fork/join (on), or exchange then "
                        "launches in stream order (off, default: the forked graph measured 4-5x slower on this "
                        "runtime, 0.33-0.42 vs 0.04-0.10 ms per image, profiles/r06/b/)")
    p.add_argument("--resident-images", type=int, default=2,
                   help="resident loop: this many independent images' loops concurrently (own engines, streams and "
                        "transports) — one image's exchange overlaps another's launches; ms_per_image = elapsed / "
                        "images; with more than one, 'one_image' holds the single-image loop too")
    p.add_argument("--halo-select", choices=["auto", "off", "exchange"] + list(HALO_MODES), default="auto",
                   help="N>1: report as the headline the fastest bit-exact halo mode when it is at least 3 %% faster "
                        "than the pre-loaded pipeline (auto; the halo mode chosen by measurement, like the kernel "
                        "tuner), or a given mode whenever it is bit-exact (tests; exchange = slot_exchange); every "
                        "mode's timing stays in 'halo_modes'")
    p.add_argument("--watchdog", type=float, default=None,
                   help="seconds the whole halo-mode measurement may take, communicator set-up included, before "
                        "every rank exits with the line as it stands printed (default modes x (timeout + 10) + 30)")
    p.add_argument("--stall-exchange", action="store_true", help=argparse.SUPPRESS)  # tests: a hung peer
    p.add_argument("--hw-queues", type=int, default=0,
                   help="GPU_MAX_HW_QUEUES for this process (default: 4 with CU-masked slot queues, else "
                        "max(8, slots + 3))")
    p.add_argument("--trace", type=int, default=0, metavar="IMAGES",
                   help="after the timed region, time the stages of IMAGES more images (needs a directly issued "
                        "pipeline: --graph-capture off or --step-graphs off) and write them to --trace-out")
    p.add_argument("--trace-out", default="gpurun_out/pipeline_trace.json")
    p.add_argument("--check", dest="check", action="store_true", default=True,
                   help="after timing (outside the timed region), compare every rank's newest image, and every halo "
                        "mode's at N>1, with the CPU oracle; 'mismatches' in the JSON line (default on)")
    p.add_argument("--no-check", dest="check", action="store_false", help="skip the oracle check (sweeps)")
    p.add_argument("--pool-queues", dest="cu_mask_queues", action="store_false", default=True,
                   help="slot streams from the runtime's queue pool (default: each on its own CU-masked hardware "
                        "queue, profiles/r04/slots_c/)")
    p.add_argument("--head-pool-streams", dest="head_on_slot_streams", action="store_false", default=True,
                   help="a streamed head image's copies on two pool streams (default: the next two slots' streams)")
    p.add_argument("--ipc-pull", choices=["grid", "single", "sdma"], default="grid",
                   help="halo mode ipc: how a rank pulls its neighbours' rows (grid: one dispatch of many "
                        "workgroups; single: one workgroup; sdma: flag kernels around SDMA peer copies)")
    p.add_argument("--numa-bind", choices=["on", "off"], default="on",
                   help="restrict each rank to its GPU's NUMA node (default on)")
    p.add_argument("--diag-windows", type=int, default=8, metavar="W",
                   help="after the timed region, replay the identical K-image window W times unmarked and W times "
                        "with per-image completion marks; reported under 'windows' (0 = off)")
    p.add_argument("--mark-timed", action="store_true",
                   help="diagnostics: completion marks in the TIMED window too (adds one event per image; the "
                        "line is flagged 'timed_window_marked')")
    p.add_argument("--qualify-staging", choices=["on", "off"], default="on",
                   help="time every slot's pinned staging buffers through the copy engines at set-up and replace any "
                        "that copies >5%% slower than the best (DistributedBlur._qualify_staging); 'staging' in the "
                        "JSON line")
    p.add_argument("--flush-staging", choices=["on", "off"], default="on",
                   help="after the input images are written into the pinned staging buffers, clflush them out of "
                        "every CPU cache (DistributedBlur(flush_staging=True)): rows left dirty in the caches of the "
                        "cores that wrote them made that buffer's uploads ~5-15%% slower for the whole process "
                        "(profiles/r06/e/)")
    p.add_argument("--native", action="store_true",
                   help="run the same serving step on the native stack: the in-tree `conv --bench` (ROCm's HIP "
                        "runtime, no torch; its fork launcher for N > 1) and print its JSON line")
    return p.parse_args()


def oracle_rows(a, band):
    """The CPU oracle (native OpenMP stencil, bit-exact with the reference's
    float32) for this rank's owned rows: the synthetic image rows of the
    band's dependency cone [y0 - reps, y0 + rows + reps) (clipped to the
    image) convolved `reps` times; an artificial edge of the cone moves one
    row per repetition, so the owned rows are exact without convolving the
    whole image on every rank."""
    import numpy as np

    from pconv._native import require_native
    from pconv.models.filters import get_filter

    n = require_native()
    c = {"grey": 1, "rgb": 3, "rgba": 4}[a.channels]
    lo, hi = max(0, band.y0 - a.reps), min(a.height, band.y0 + band.rows + a.reps)
    sub = np.empty((hi - lo) * a.width * c, np.uint8)
    n.synth_rows(sub, a.width, a.height, a.channels, int(a.seed), lo, hi - lo)
    ref = np.empty_like(sub)
    # the node's CPU budget split between the ranks on it (8 ranks with a team
    # of the whole budget each would oversubscribe the host 8x)
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    threads = max(1, n.default_cpu_threads() // local)
    n.cpu_convolve(sub, ref, a.width, hi - lo, a.channels, a.reps, get_filter(a.filter).to_native(), True, threads)
    return ref.reshape(hi - lo, -1)[band.y0 - lo:band.y0 - lo + band.rows]


def mismatching_bytes(got, ref) -> int:
    """Bytes of this rank's newest image that differ from the oracle, summed
    over ranks (every rank must call it)."""
    import numpy as np

    from pconv.parallel.bootstrap import sum_over_ranks

    return int(sum_over_ranks(int(np.count_nonzero(got.reshape(ref.shape) != ref))))


def gather_floats(v: float):
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [float(v)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, float(v))
    return [float(x) for x in out]


def gather_ints(v: int):
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [int(v)]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, int(v))
    return [int(x) for x in out]


# Halo modes timed after the pre-loaded headline at N>1 (each with the same K
# steps, barriers and device syncs as the headline):
#   slot_exchange: each image on its slot's own stream with its own
#       communicator; one exchange of the whole ghost zone in stream order,
#       then the repetitions; with RCCL the whole image (upload, send/recv,
#       launches, download) is ONE captured hipGraph (slots overlap each other);
#   slot_exchange_direct: the same, issued directly (upload, the group's
#       RCCL calls, the repetitions as a cached graph, download);
#   event: one communicator, shared H2D / compute / D2H / comm streams; the
#       whole ghost zone of image k+1 is exchanged on the comm stream while
#       image k computes (event-ordered);
#   overlap: the reference's algorithm (mpi/mpi_convolution.c:156-240,
#       Isend/Irecv, inner compute, Wait, edges) with a T-deep halo: an
#       exchange every fused launch on the comm stream, the interior launch
#       concurrently on the compute stream, the edge strips after the halo
#       event;
#   ipc: slot_exchange's pipeline with the HIP-IPC transport instead of RCCL
#       (ipc_halo.hpp): each rank pulls its neighbours' boundary rows straight
#       out of their frames (opened once with hipIpcOpenMemHandle), ordered by
#       device-side flag kernels — no communication-library kernel; every
#       image ONE captured graph.
HALO_MODES = ("slot_exchange", "slot_exchange_direct", "event", "overlap", "ipc")


def mode_transport(mode: str, transport: str) -> str:
    return "ipc" if mode == "ipc" else transport


def policy_kwargs(a) -> dict:
    """Pipeline policy flags -> DistributedBlur / native EngineOptions (echoed in the JSON config)."""
    return dict(cu_mask_queues=getattr(a, "cu_mask_queues", True),
                head_on_slot_streams=getattr(a, "head_on_slot_streams", True),
                head_alt_uploads=getattr(a, "head_alt_uploads", True),
                lazy_head=None if getattr(a, "lazy_head", None) is None else a.lazy_head == "on",
                ipc_pull=getattr(a, "ipc_pull", "grid"))


def stream_weights(a) -> list:
    """--stream-weights "3,4,4,5,5" -> [3, 4, 4, 5, 5] ([]: the native default 5, ..., 5, 6)."""
    w = getattr(a, "stream_weights", None)
    return [int(x) for x in w.split(",")] if w else []


def mode_kwargs(a, mode: str, fuse: int) -> dict:
    kw = dict(preload_halo=False, slots=a.slots, variant=a.variant, fuse=a.fuse, overlap=not a.no_overlap,
              halo=a.halo, concurrent={"auto": -1, "on": 1, "off": 0}[a.concurrent], **policy_kwargs(a))
    if mode in ("slot_exchange", "slot_exchange_direct", "ipc"):
        kw["slot_exchange"] = True
        kw["graph_capture"] = mode != "slot_exchange_direct"
    elif mode == "overlap":
        # T-deep ghost zone: one exchange per fused launch on the comm stream
        # beside the interior launch, edges after the halo event (event-ordered
        # streams; the same loop captured as one graph per image on slot
        # streams, DistributedBlur(slot_comm=True), measured slower: 0.303 vs
        # 0.246 ms per 8-way rank step, profiles/r03/emulate8/captured_split/)
        kw.update(halo=int(fuse), overlap=True)
    elif mode != "event":
        raise ValueError(f"unknown halo mode {mode!r}")
    return kw


def resident_loop(blur, a, ipc: bool = False) -> dict:
    """The resident loop with `--resident-images` concurrent images (the
    reported ms_per_image), and — when that is more than one — also one
    image alone, the reference's single-image loop ('one_image')."""
    # concurrent images need a capturable transport (RCCL, IPC): a host-staged
    # one (gloo-host, rehearsals) runs the single-image loop
    nimg = max(1, int(a.resident_images)) if (ipc or blur.comm is not None) else 1
    out = resident_loop_n(blur, a, ipc, nimg)
    if nimg > 1:
        one = resident_loop_n(blur, a, ipc, 1)
        out["one_image"] = {k: one[k] for k in ("ms_per_image", "mpix_per_s", "exchanges_per_image",
                                                "launches_per_image")}
    return out


def resident_loop_n(blur, a, ipc: bool, nimg: int) -> dict:
    """The reference's MPI loop (mpi/mpi_convolution.c:156-240, loop-only
    timing) on the bands already resident on the GPUs: `reps` repetitions
    with the ghost rows exchanged every `halo` repetitions through the
    pipeline's transport (RCCL over xGMI between real GPUs), no PCIe.  Its own
    engine runs the exchanges on the compute stream, so with a capturable
    transport (RCCL) the whole loop — exchanges and launches — replays as ONE
    cached graph per image (EngineOptions::capture_exchanges).  K loops
    between barriers, max over ranks; ghost contents are whatever the frames
    hold (timing only: the pipelined mode's images were oracle-checked).
    `ipc`: the ghost rows pulled by the CUs from the neighbours' frames
    through HIP-IPC instead (its own transports, `--ipc-pull` form), also
    captured."""
    import numpy as np
    import torch

    import pconv
    from pconv.parallel.bootstrap import barrier, make_rccl_comm, max_over_ranks

    n = pconv.native
    b = blur.band
    overlap = a.resident_overlap == "on"
    # `nimg` independent images, each its own engine (frames, compute and
    # communication streams) and its own transport, their loops concurrent
    engs = [n.BandEngine.for_band(a.width, a.height, a.channels, a.filter, b, blur.device,
                                  halo=int(blur.engine.halo), fuse=int(blur.engine.fuse), overlap=overlap,
                                  variant=a.variant, graph=True, capture_exchanges=True) for _ in range(nimg)]
    ts, comms = [], []
    if ipc:
        from pconv.parallel.bootstrap import make_ipc_transports

        ts = make_ipc_transports(engs, a.exchange_timeout, pull=a.ipc_pull)
        for e, x in zip(engs, ts):
            e.attach_transport(x)
        transport = f"ipc-{a.ipc_pull}"
    elif blur.comm is not None:
        comms = [blur.comm] + [make_rccl_comm(blur.device) for _ in range(nimg - 1)]
        for e, c in zip(engs, comms):
            e.attach_rccl(c)
        transport = "rccl"
    elif blur.transport is not None:
        if nimg > 1:
            raise RuntimeError("resident loop: concurrent images need a capturable transport (rccl, ipc)")
        engs[0].attach_transport(blur.transport)
        transport = type(blur.transport).__name__
    else:
        raise RuntimeError("resident loop: the pipeline has no halo transport")
    for e in engs:
        e.upload(np.ascontiguousarray(blur.inputs[0][:b.rows]).reshape(-1), 0, b.rows)
    steps = a.loop_steps if a.loop_steps is not None else a.steps

    def once():
        for e in engs:
            e.set_halo_valid(False)  # exchange every `halo` reps, as the reference does every rep
            e.run(a.reps)

    def sync():
        for e in engs:
            e.synchronize()

    for _ in range(2):  # the first run captures the graph (tuning first)
        once()
    sync()
    torch.cuda.synchronize()
    barrier()
    t = time.perf_counter()
    for _ in range(steps):
        once()
    sync()
    torch.cuda.synchronize()
    for x in ts:
        x.check()  # a timed-out device-side wait raises
    elapsed = max_over_ranks(time.perf_counter() - t)
    eng = engs[0]
    st = eng.stats
    px = a.width * a.height * a.reps
    images = steps * nimg
    out = {"ms_per_image": round(elapsed / images * 1e3, 4), "mpix_per_s": round(px * images / elapsed / 1e6, 2),
           "steps": steps, "concurrent_images": nimg, "overlap_split": overlap,
           "exchanges_per_image": int(st.exchanges), "launches_per_image": int(st.launches),
           "halo_rows": int(eng.halo), "one_graph_per_image": int(eng.cached_graphs) > 0, "transport": transport,
           # per rank: the ghost rows it receives per exchange (both sides for an interior band)
           "ghost_bytes_per_exchange": gather_ints(int(eng.halo) * int(blur.row_bytes) *
                                                   (int(b.up >= 0) + int(b.down >= 0)))}
    del ts, eng, engs
    comms = comms[1:]
    del comms
    barrier()  # every rank's transports are closed before any frame goes away
    return out


def measure_mode(a, mode, ref_rows, world, rank, device, transport, fuse, oracle=None):
    """Time K steps of one halo mode exactly like the headline (barrier +
    device sync on both sides, max over ranks) and compare its newest image
    with the headline's bytes and (when checking) with the CPU oracle.  Never
    raises: a failure is reported in the returned dict (status), and every
    rank tears the pipeline down."""
    import gc

    import numpy as np

    from pconv.parallel.bootstrap import barrier, sum_over_ranks
    from pconv.parallel.dist_engine import DistributedBlur

    transport = mode_transport(mode, transport)
    res = {"status": "ok", "transport": transport}
    xb = None
    try:
        if a.stall_exchange and rank == world - 1:  # tests: the last rank never joins
            time.sleep(3600)
        xb = DistributedBlur(a.width, a.height, a.channels, a.filter, a.reps, rank=rank, world=world, device=device,
                             transport=transport, **mode_kwargs(a, mode, fuse))
        xb.load_synthetic(a.seed)
        for _ in range(min(a.warmup, 5) + a.slots):
            xb.submit(a.reps)
        xb.drain(timeout_s=a.exchange_timeout)
        elapsed, mine = timed_steps(xb, a.steps, a.reps, a.exchange_timeout)
        got = xb.step(a.reps)
        bad = sum_over_ranks(int(np.count_nonzero(got != ref_rows)))
        if oracle is not None:
            res["mismatches"] = mismatching_bytes(got, oracle)
        per_rank = gather_floats(mine)
        h2d_b, d2h_b = gather_ints(xb.h2d_bytes_per_image), gather_ints(xb.d2h_bytes_per_image)
        st = xb.stats
        px = a.width * a.height * a.reps
        res.update(steps=a.steps, ms_per_step=round(elapsed / a.steps * 1e3, 4),
                   value=round(px * a.steps / elapsed / 1e6, 2), mismatches_vs_headline=int(bad),
                   per_rank_ms_per_step=[round(t / a.steps * 1e3, 4) for t in per_rank],
                   h2d_bytes_per_step=h2d_b, d2h_bytes_per_step=d2h_b,
                   halo_depth=int(xb.engine.halo), fuse=int(xb.engine.fuse),
                   launches_per_step=int(st.launches), exchanges_per_step=int(st.exchanges),
                   slot_streams=bool(xb.pipe.graphs), step_graphs=bool(xb.pipe.step_graphs),
                   concurrent_images=bool(xb.pipe.concurrent),
                   overlap_split=mode == "overlap" or (mode == "event" and not a.no_overlap))
        if mode in ("event", "ipc") and a.resident_loop == "on":
            try:
                res["resident_loop"] = resident_loop(xb, a, ipc=mode == "ipc")
            except Exception as e:  # noqa: BLE001  (the mode's own timing stands)
                res["resident_loop"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    except Exception as e:  # reported, never fatal for the headline line
        res["status"] = f"error: {type(e).__name__}: {e}"[:400]
    finally:
        # communicators are torn down on every rank at the same point
        del xb
        gc.collect()
        try:
            barrier()
        except Exception:
            pass
    return res


def timed_steps(blur, steps: int, reps: int, timeout_s: float):
    """K end-to-end steps of one pipeline between barriers + device syncs;
    returns (max over ranks of the elapsed seconds, this rank's seconds)."""
    import torch

    from pconv.parallel.bootstrap import barrier, max_over_ranks

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        blur.submit(reps)
    blur.drain(timeout_s=timeout_s)
    torch.cuda.synchronize()
    barrier()
    mine = time.perf_counter() - t0
    return max_over_ranks(mine), mine


def spawn_ranks(a) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start the N
    ranks through torch.distributed.run as CHILD processes (this process has
    not touched the GPU) and return their exit code."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def copy_floor_ms(in_bytes: int, out_bytes: int, device: int, iters: int = 8):
    """This box's copy floor for one step: the step's H2D alone and its D2H
    alone (pinned host memory, one stream, median of `iters`).  A pipelined
    step cannot be shorter than the slower of the two; it makes every BENCH
    line self-explaining across boxes with different PCIe rates (the round-1
    driver box measured 0.46 ms/step where others give 0.31)."""
    import torch

    hin = torch.empty(in_bytes, dtype=torch.uint8, pin_memory=True)
    hout = torch.empty(out_bytes, dtype=torch.uint8, pin_memory=True)
    din = torch.empty(in_bytes, dtype=torch.uint8, device=device)
    dout = torch.empty(out_bytes, dtype=torch.uint8, device=device)

    def timed(fn):
        ts = []
        for i in range(iters + 2):
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(device)
            if i >= 2:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2] * 1e3

    h2d = timed(lambda: din.copy_(hin, non_blocking=True))
    d2h = timed(lambda: hout.copy_(dout, non_blocking=True))
    return h2d, d2h


CONCURRENT_FLOOR_MS = 20.0  # each rank's concurrent copies span at least this long at its solo rate


def copy_floors(run, world: int, rank: int):
    """A copy floor per rank twice: SOLO (rank r runs while every other rank
    waits between barriers, one rank at a time; the better of two runs of 8
    pairs) and CONCURRENT (every rank at once between two barriers, one run
    long enough — CONCURRENT_FLOOR_MS at the slowest solo rate — that the
    barrier's release skew is small against the span the ranks overlap, and
    its mean, not a minimum).  `run(n)` times n copy pairs, ms per pair.
    With one GPU per rank on its own PCIe link, concurrent = solo; a larger
    concurrent floor means the ranks share something on the host side (host
    DRAM bandwidth, a PCIe switch) — what the first 8-GPU line must separate
    from link rates.  Every rank must call it; returns (solo per rank,
    concurrent per rank); one rank: concurrent = solo."""
    import math

    from pconv.parallel.bootstrap import barrier

    solo = -1.0
    for r in range(world):
        barrier()
        if r == rank:
            solo = min(run(8), run(8))
    solos = gather_floats(solo)
    if world == 1:
        return solos, solos
    valid = [s for s in solos if s > 0]
    n = min(4000, max(8, math.ceil(CONCURRENT_FLOOR_MS / max(valid)))) if valid else 8
    barrier()
    conc = run(n)
    barrier()
    return solos, gather_floats(conc)


def staging_numa(blur) -> dict:
    """NUMA placement of every slot's pinned staging pages (move_pages
    query): {"gpu_node": n, "in": [{node: pages}...], "out": [...]}."""
    try:
        import pconv

        n = pconv.native
        node = lambda b: {str(k): v for k, v in n.page_nodes(b.ptr, len(b)).items()}  # noqa: E731
        return {"gpu_node": n.device_numa_node(blur.device), "in": [node(b) for b in blur._in],
                "out": [node(b) for b in blur._out]}
    except Exception as e:  # noqa: BLE001  (diagnostics only)
        return {"error": str(e)[:200]}


def kfd_queue_count():
    """Hardware (HSA user-mode) queues this process holds, from the KFD's
    per-process sysfs (None when not readable): slot streams on CU-masked
    queues, the runtime's pool, and any queue torch or RCCL created."""
    pids = [os.getpid()]
    try:  # the KFD names processes by their PID in the host's namespace: NSpid lists every level
        for line in open("/proc/self/status"):
            if line.startswith("NSpid:"):
                pids = [int(x) for x in line.split()[1:]] + pids
    except OSError:
        pass
    for pid in pids:
        try:
            return len(os.listdir(f"/sys/class/kfd/kfd/proc/{pid}/queues"))
        except OSError:
            continue
    return None


def tuned_picks():
    """The SWAR tuner's choice per launch key: [channels, steps, rows, row
    bytes, step form, kernel (0 k_swar, 1 k_swar_pf), lanes, rows/wave, waves]."""
    import pconv

    return [list(k) + list(sh) for k, sh in pconv.native.swar_tuned()]


def window_diagnostics(blur, a, count: int) -> dict:
    """Replay the timed window (K images submitted to an idle pipeline,
    drained, barriers + device syncs around it, max over ranks) `count` times
    as it ran, then `count` times with per-image completion marks (one timing
    event after each image on the stream it completes on).  The slowest and
    fastest marked windows keep their per-image completion times, so a slow
    window shows whether every image is slower (a rate) or a few stall (a gap).
    Outside the timed region; diagnostics only."""
    import torch

    from pconv.parallel.bootstrap import barrier, max_over_ranks

    def window(marked: bool):
        if marked:
            blur.pipe.enable_marks(a.steps)
        barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            blur.submit(a.reps)
        blur.drain()
        torch.cuda.synchronize()
        barrier()
        ms = max_over_ranks(time.perf_counter() - t) / a.steps * 1e3
        return ms, (blur.pipe.marks() if marked else None)

    plain = [round(window(False)[0], 4) for _ in range(count)]
    marked = [window(True) for _ in range(count)]

    def detail(ms, rows):
        done = [round(r[1], 4) for r in rows]
        return {"ms_per_step": round(ms, 4), "slots": [int(r[0]) for r in rows],
                "head_streamed": [int(r[2]) for r in rows], "completion_ms": done,
                "deltas_ms": [round(y - x, 4) for x, y in zip([0.0] + done[:-1], done)]}

    slow = max(marked, key=lambda m: m[0])
    fast = min(marked, key=lambda m: m[0])
    out = {"ms_per_step": plain, "marked_ms_per_step": [round(m[0], 4) for m in marked],
           "slowest_marked": detail(*slow), "fastest_marked": detail(*fast)}
    # each slot's own pinned staging buffers through the copy floor: H2D alone, D2H alone, the pair (a slot whose
    # buffers copy slower than the others' shows here)
    try:
        import pconv

        rows_in = blur.inputs[0].shape[0]
        out["slot_buffer_copy_ms"] = [
            [round(x, 4) for x in pconv.native.copy_floor_on(blur.device, blur._in[k].ptr, blur._out[k].ptr,
                                                             blur.row_bytes, rows_in, blur.band.rows, 6)]
            for k in range(blur.slots)]
    except Exception as e:  # noqa: BLE001  (diagnostics only)
        out["slot_buffer_copy_ms"] = f"not measured: {e}"[:200]
    return out


def hw_queue_budget(a) -> int:
    """GPU_MAX_HW_QUEUES for this process.  With CU-masked slot streams (the
    default) every image slot has its own dedicated hardware queue outside
    the runtime's pool, and the pool keeps the runtime's default of 4:
    measured on one box, 6 interleaved pairs of the driver's 20-image
    command, 4 pool queues 0.335-0.349 ms per step (mean 0.342) against
    0.346-0.355 (0.350) with 8 (profiles/r05/c/).  Pool slot streams
    (--pool-queues) get one queue per stream of the pipeline (H2D, D2H, comm
    and one per slot) so independent streams never alias a queue.
    N > 1 (and the per-rank proxy) keeps the larger pool: its halo modes
    run event-ordered pipelines on pool streams (H2D, D2H, comm, compute)."""
    if a.hw_queues:
        return a.hw_queues
    return 4 if a.cu_mask_queues and a.gpus == 1 and not a.emulate else max(8, a.slots + 3)


def run_native(a) -> int:
    """`bench.py --native`: the serving step of the `conv` binary (C++ fork
    launcher + BandPipeline on the HIP runtime it links) instead of this
    torch process; its single JSON line is passed through.  Nothing here
    touches the GPU (the child is started before any HIP call)."""
    import subprocess

    if int(os.environ.get("RANK", "0")) != 0:
        return 0  # under torchrun: rank 0 runs the native launcher for all ranks
    conv = os.path.join(ROOT, "parallel-image-convolution-using-mpi-openmp-and-cuda_amd", "bin", "conv")
    cmd = [conv, "synthetic.raw", str(a.width), str(a.height), str(a.reps), a.channels, "--synthetic", str(a.seed),
           "--gpus", str(a.gpus), "--bench", str(a.steps), "--warmup", str(min(a.warmup, 100)), "--slots",
           str(a.slots), "--stream-chunks", str(a.stream_chunks), "--filter", a.filter]
    if a.fuse:
        cmd += ["--fuse", str(a.fuse)]
    if a.check:
        cmd.append("--check")
    if a.transport == "gloo-host":
        cmd += ["--transport", "shm"]  # rehearsal: ranks may share one GPU
    cmd += [] if a.cu_mask_queues else ["--pool-queues"]
    cmd += [] if a.head_on_slot_streams else ["--head-pool-streams"]
    cmd += [] if a.numa_bind == "on" else ["--no-numa-bind"]
    cmd += [] if a.qualify_staging == "on" else ["--no-qualify-staging"]
    cmd += [] if a.flush_staging == "on" else ["--no-flush-staging"]
    if a.emulate:
        cmd[cmd.index("--gpus") + 1] = "1"
        cmd += ["--emulate", a.emulate]  # one rank of a WORLD-way split, alone (per-rank proxy)
    env = dict(os.environ)
    want = hw_queue_budget(a)  # as for the torch pipeline below
    if a.hw_queues or int(env.get("GPU_MAX_HW_QUEUES", "4")) < want:
        env["GPU_MAX_HW_QUEUES"] = str(min(want, 32))
    r = subprocess.run(cmd, capture_output=True, text=True, env=env)
    sys.stderr.write(r.stderr)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or len(lines) != 1:
        sys.stderr.write(r.stdout)
        return r.returncode or 1
    print(lines[0], flush=True)
    return 0


def main():
    a = parse()
    if a.slots is None:
        a.slots = 4
    if a.native:
        sys.exit(run_native(a))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not a.emulate:
        sys.exit(spawn_ranks(a))
    # The runtime's hardware-queue pool (must be set before the HIP runtime
    # initialises): see hw_queue_budget.
    want = hw_queue_budget(a)
    if a.hw_queues or int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(want, 32))
    import torch

    import pconv
    from pconv.parallel.bootstrap import barrier, bind_to_device_numa, init_distributed, max_over_ranks, shutdown
    from pconv.parallel.dist_engine import DistributedBlur, preload_is_exchange_free

    pconv.native.install_crash_handler()  # a native crash prints its C++ frames
    ctx = init_distributed("gloo")
    world = ctx.world
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    rank = ctx.rank
    transport = a.transport
    a.preload_halo = a.preload_halo or a.halo_mode == "preload"
    # Pre-loaded ghost rows make every image exchange-free: the headline
    # pipeline then needs no communicator (the max over ranks goes through
    # gloo), so an RCCL problem can only affect the secondary halo-mode
    # measurement, never the headline line.
    # Bands shorter than `reps` cannot pre-load a ghost zone for every
    # repetition: the headline then exchanges halos through the transport.
    exchange_free = a.preload_halo and preload_is_exchange_free(a.height, world, a.reps)
    head_transport = "none" if (exchange_free and world > 1) else transport
    if a.emulate:
        if world != 1:
            raise SystemExit("--emulate runs in a single process")
        world, rank = (int(v) for v in a.emulate.split(":"))
        a.preload_halo, transport, head_transport = True, "none", "none"
        if a.emulate_halo != "preload":
            t = mode_transport(a.emulate_halo, "rccl")
            a.preload_halo, transport, head_transport = False, t, t
    device = ctx.local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    # host thread + first-touch pinned buffers on the GPU's own socket
    cpu_bind = bind_to_device_numa(device, enabled=a.numa_bind == "on")

    if a.emulate and a.emulate_halo != "preload":
        fuse0 = a.fuse if a.fuse is not None else DistributedBlur(
            a.width, a.height, a.channels, a.filter, a.reps, rank=rank, world=world, device=device,
            preload_halo=True, slots=1, transport="none").engine.fuse
        blur = DistributedBlur(a.width, a.height, a.channels, a.filter, a.reps, rank=rank, world=world,
                               device=device, transport=mode_transport(a.emulate_halo, "rccl"),
                               self_neighbours=True, **mode_kwargs(a, a.emulate_halo, fuse0))
    else:
        blur = DistributedBlur(a.width, a.height, a.channels, a.filter, a.reps, rank=rank, world=world,
                               device=device, halo=a.halo, fuse=a.fuse, overlap=not a.no_overlap,
                               preload_halo=a.preload_halo, slots=a.slots, variant=a.variant,
                               transport=head_transport, concurrent={"auto": -1, "on": 1, "off": 0}[a.concurrent],
                               step_graphs={"auto": None, "on": True, "off": False}[a.step_graphs],
                               graph_capture=a.graph_capture == "on", stream_chunks=a.stream_chunks,
                               stream_weights=stream_weights(a), stream_min_bytes=int(a.stream_min_mb * 2 ** 20),
                               qualify_staging=a.qualify_staging == "on", flush_staging=a.flush_staging == "on",
                               **policy_kwargs(a))
    blur.load_synthetic(a.seed)
    # --emulate-rccl: hold a (1-rank) RCCL communicator through the timed
    # region, as every real N>1 rank of the exchange path does.
    held_comm = None
    if a.emulate and a.emulate_rccl:
        from pconv.parallel.bootstrap import make_rccl_comm

        held_comm = make_rccl_comm(device)

    for _ in range(a.warmup):
        blur.submit(a.reps)
    blur.drain()

    # ---- timed: K end-to-end steps (H2D + reps + D2H per image, `slots`
    # images in flight), all K complete inside the region; max over ranks
    if a.mark_timed:
        blur.pipe.enable_marks(a.steps)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        blur.submit(a.reps)
    blur.drain()
    torch.cuda.synchronize()
    barrier()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine)
    per_rank = gather_floats(mine)  # diagnostics: load balance across ranks
    timed_marks = blur.pipe.marks() if a.mark_timed else None
    queues_at_timed = kfd_queue_count()
    # ---- diagnostics (not timed): the same window replayed, plain and marked
    windows = window_diagnostics(blur, a, a.diag_windows) if a.diag_windows > 0 else None
    # PCIe bytes per image of every rank (band + pre-loaded ghost rows in, owned rows out): whether an N>1
    # line is link-bound or host-memory-bound
    h2d_bytes, d2h_bytes = gather_ints(blur.h2d_bytes_per_image), gather_ints(blur.d2h_bytes_per_image)
    stats = blur.stats
    # ---- oracle check of the newest image (not timed): every rank compares
    # its owned rows with the CPU oracle of its dependency cone.  Not with
    # --emulate-halo: a self-neighbour rank's ghost rows are its own rows.
    oracle = None
    if a.check and not (a.emulate and a.emulate_halo != "preload"):
        oracle = oracle_rows(a, blur.band)
    mismatches = mismatching_bytes(blur.step(a.reps), oracle) if oracle is not None else None
    if a.trace:
        blur.pipe.enable_trace(a.trace)
        for _ in range(a.trace):
            blur.submit(a.reps)
        rows = blur.pipe.trace()
        if ctx.rank == 0:
            os.makedirs(os.path.dirname(a.trace_out) or ".", exist_ok=True)
            with open(a.trace_out, "w") as f:
                json.dump({"stages": ["slot", "h2d_start", "h2d_end", "reps_end", "d2h_end"], "ms": rows,
                           "args": vars(a)}, f)
    # ---- extra: single-image latency (one image in flight, nothing else
    # queued): H2D + reps + D2H, the reference's GPU_convolution() scope.
    lat = []
    for _ in range(max(3, min(20, a.steps))):
        t = time.perf_counter()
        blur.step(a.reps)
        lat.append(time.perf_counter() - t)
    lat.sort()
    latency_ms = max_over_ranks(lat[len(lat) // 2]) * 1e3
    b = blur.band
    h2d_ms, d2h_ms = copy_floor_ms(blur.inputs[0].size, b.rows * blur.row_bytes, device)
    h2d_ms = max_over_ranks(h2d_ms / 1e3) * 1e3
    d2h_ms = max_over_ranks(d2h_ms / 1e3) * 1e3
    # ... and both directions at once, pitched like the pipeline's copies: the
    # floor a PCIe-bound step converges to (diagnostic only: never fatal)
    try:
        probe = pconv.native.CopyProbe(device, blur.row_bytes, blur.inputs[0].size // blur.row_bytes, b.rows)
    except Exception as e:  # noqa: BLE001
        print(f"bench: copy pair floor not measured: {e}", file=sys.stderr)
        probe = None

    def pair_run(n):
        try:
            return probe.run(n) if probe is not None else -1.0
        except Exception as e:  # noqa: BLE001
            print(f"bench: copy pair floor not measured: {e}", file=sys.stderr)
            return -1.0

    # per rank: alone on the node (one rank at a time) and with every rank copying at once (N > 1: whether
    # the ranks' host paths are independent, or share host DRAM / a switch)
    pair_solo, pair_conc = copy_floors(pair_run, ctx.world, ctx.rank)
    del probe  # its pinned rows and device frames
    pair_ms = max(pair_conc)
    if a.emulate:
        world = 1

    # ---- extra: device-resident loop only (reps on the resident band)
    eng = blur.engine
    ls = a.loop_steps if a.loop_steps is not None else a.steps
    def loop_once():
        if blur.preload_halo:
            eng.set_halo_valid(True)  # ghost rows stay resident (timing only)
        eng.run(a.reps)

    for _ in range(3):
        loop_once()
        eng.synchronize()
    barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(ls):
        loop_once()
    eng.synchronize()
    torch.cuda.synchronize()
    barrier()
    loop_elapsed = max_over_ranks(time.perf_counter() - t1)

    px = a.width * a.height * a.reps
    value = px * a.steps / elapsed / 1e6
    loop_value = px * ls / loop_elapsed / 1e6 if ls else None
    runtime = pconv.native.runtime_info()  # the HIP runtime / RCCL this process actually runs on
    head_mode = "preload" if blur.preload_halo else ("none" if world == 1 else "event")
    out = None
    if ctx.rank == 0:
        out = {
            "metric": metric_for(a),
            "value": round(value, 2),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / BASELINE_MPIX, 2) if (a.width, a.height, a.channels, a.reps) == HEADLINE
            and a.filter == "gaussian" else None,
            # value / BASELINE.md's 190.3 Mpix/s: pipelined steady-state throughput here against the
            # reference's single cold end-to-end CLI run (HIP/CUDA init and file I/O included there).
            # The like-for-like end-to-end comparison is the `conv` CLI table in docs/PERFORMANCE.md.
            "vs_baseline_basis": "pipelined throughput vs reference single-run end-to-end (CUDA, GTX 970)",
            "dtype": "fp32-exact (packed 16-bit integer, bit-identical to the reference float32)",
            "data": "synthetic random bytes",
            "config": {
                "model": f"3x3 {a.filter} convolution, {a.width}x{a.height} {a.channels}, {a.reps} reps",
                "global_batch": 1,
                "seq_len": a.height,
                "parallelism": f"rowband{world}",
                "step": "H2D + reps + D2H per image (reference GPU_convolution scope)",
                "halo_mode": head_mode,
                "images_in_flight": a.slots,
                "concurrent_images": bool(blur.pipe.concurrent),
                "slot_streams": bool(blur.pipe.graphs),
                "step_graphs": bool(blur.pipe.step_graphs),
                "halo_depth": int(blur.engine.halo),
                "fuse": int(blur.engine.fuse),
                "stream_chunks": int(len(stream_weights(a)) if a.stream_weights else a.stream_chunks),
                "stream_weights": list(blur.pipe.options["stream_weights"]),
                "lazy_head": bool(blur.pipe.options["lazy_head"]),
                "stream_min_mb": a.stream_min_mb,
                "preload_halo": bool(blur.preload_halo),
                "launches_per_step": int(stats.launches),
                "exchanges_per_step": int(stats.exchanges),
                "cu_mask_queues": bool(a.cu_mask_queues),
                "head_on_slot_streams": bool(a.head_on_slot_streams),
                "head_alt_uploads": bool(a.head_alt_uploads),
                "ipc_pull": a.ipc_pull,
                "numa_bind": a.numa_bind == "on",
                "qualify_staging": a.qualify_staging == "on",
                "flush_staging": a.flush_staging == "on",
            },
            "latency_ms": round(latency_ms, 4),
            "copy_floor": {"h2d_ms": round(h2d_ms, 4), "d2h_ms": round(d2h_ms, 4),
                           "floor_ms": round(max(h2d_ms, d2h_ms), 4),
                           # one pitched H2D + one pitched D2H of a step issued together (the PCIe-bound
                           # pipeline's floor; null if the measurement failed)
                           "pair_ms": round(pair_ms, 4) if pair_ms > 0 else None,
                           # per rank: alone (one rank at a time), and all ranks at once between two barriers
                           "pair_ms_solo": [round(x, 4) for x in pair_solo],
                           "pair_ms_concurrent": [round(x, 4) for x in pair_conc]},
            "loop_only": {
                "ms_per_step": round(loop_elapsed / ls * 1e3, 4) if ls else None,
                "mpix_per_s": round(loop_value, 2) if loop_value else None,  # (reps 0: copy-only diagnostics)
                "us_per_rep": round(loop_elapsed / ls / a.reps * 1e6, 3) if ls and a.reps else None,
            },
            "device": torch.cuda.get_device_name(device),
            "runtime": runtime,
            "rccl": runtime["rccl_version"],
            "headline_transport": head_transport if world > 1 else None,
            "pconv": pconv.__version__,
            "per_rank_ms_per_step": [round(t / a.steps * 1e3, 4) for t in per_rank],
            "h2d_bytes_per_step": h2d_bytes,
            "d2h_bytes_per_step": d2h_bytes,
            "rank0_cpus_bound": cpu_bind,
            # the timed window replayed (plain, then with per-image completion marks), the tuner's picks and
            # the hardware queues this process held during the timed window: a slow window explains itself
            "windows": windows,
            "tuned": tuned_picks(),
            "hw_queues": {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "kfd_queues": queues_at_timed},
            # staging qualification (set-up): every slot's pinned buffers timed, slow ones replaced
            "staging": blur.staging,
            # where each slot's pinned pages live (NUMA node -> pages) and the GPU's own node
            "staging_numa": staging_numa(blur),
        }
        if timed_marks is not None:
            out["timed_window_marked"] = {"completion_ms": [round(r[1], 4) for r in timed_marks],
                                          "slots": [int(r[0]) for r in timed_marks],
                                          "head_streamed": [int(r[2]) for r in timed_marks]}
        if mismatches is not None:
            out["mismatches"] = mismatches
            out["check"] = "newest image of every rank vs the CPU oracle (OpenMP, bit-exact float32 semantics), " \
                           "after the timed region"
        if a.emulate:
            out["emulated"] = f"rank {rank} of a {a.emulate.split(':')[0]}-way split on one GPU; value = this " \
                              "rank's step rate x full-image pixels (proxy, not a multi-GPU measurement)"
            out["config"]["halo_mode"] = a.emulate_halo
            if a.emulate_halo != "preload":
                how = "IPC pulls of its own rows" if a.emulate_halo == "ipc" else "RCCL send/recv to self"
                out["emulated"] += f"; halos exchanged with the rank itself ({how}): real exchange costs, ghost " \
                                   "contents not those of its neighbours"
    if a.emulate and a.emulate_halo in ("event", "ipc") and a.resident_loop == "on":
        # the resident MPI loop of this rank's band, ghost rows through RCCL send/recv / IPC pulls to itself
        rl = resident_loop(blur, a, ipc=a.emulate_halo == "ipc")
        if out is not None:
            out["resident_loop" if a.emulate_halo == "event" else "resident_loop_ipc"] = rl

    import threading

    emit_lock = threading.Lock()
    emitted = []
    state = {"out": out}

    def emit(line):  # the one JSON line, printed once whichever path gets here first
        with emit_lock:
            if line is not None and not emitted:
                print(json.dumps(line), flush=True)
                emitted.append(True)

    dog = None
    modes = [m for m in a.halo_modes.split(",") if m] if world > 1 and not a.emulate and \
        a.exchange_check in ("on", "auto") else []
    modes = [m for m in modes if m != head_mode]
    if modes:
        # The other halo modes, each timed exactly like the headline AFTER the
        # headline is final.  A watchdog on every rank bounds the whole
        # measurement (communicator set-up included): on expiry rank 0 prints
        # the line as it stands (the mode in progress marked timed out) and
        # every rank exits, so a stuck peer can never cost the headline.
        results = {}
        pending = {"mode": None}
        if out is not None:
            out["halo_modes"] = results
            results[out["config"]["halo_mode"]] = {
                "status": "ok", "transport": head_transport, "ms_per_step": out["ms_per_step"],
                "value": out["value"], "halo_depth": out["config"]["halo_depth"],
                "exchanges_per_step": out["config"]["exchanges_per_step"]}
            if "mismatches" in out:
                results[out["config"]["halo_mode"]]["mismatches"] = out["mismatches"]

        def expire():
            if state["out"] is not None:
                line = dict(state["out"])
                hm = dict(line.get("halo_modes", {}))
                if pending["mode"]:
                    hm[pending["mode"]] = {"transport": transport, "status": "watchdog timeout"}
                line["halo_modes"] = hm
                line["watchdog"] = "fired: a halo-mode measurement stalled (exit status 3)"
                emit(line)
            sys.stdout.flush()
            sys.stderr.flush()
            # the headline line is out, but a stalled exchange is a failure the
            # caller must see: exit non-zero (no restart, no exec)
            os._exit(3)

        dog = threading.Timer(a.watchdog if a.watchdog is not None else
                              len(modes) * (a.exchange_timeout + 10.0) + 30.0, expire)
        dog.daemon = True
        dog.start()
        ref_rows = blur.step(a.reps).copy()
        for m in modes:
            pending["mode"] = m
            r = measure_mode(a, m, ref_rows, world, rank, device, transport, int(blur.engine.fuse), oracle)
            pending["mode"] = None
            if out is not None:
                results[m] = r
        # the reference's loop-only MPI semantics, ghost rows crossing between the GPUs (RCCL / IPC)
        if out is not None and "resident_loop" in results.get("event", {}):
            out["resident_loop"] = results["event"]["resident_loop"]
        if out is not None and "resident_loop" in results.get("ipc", {}):
            out["resident_loop_ipc"] = results["ipc"]["resident_loop"]
        # Halo mode chosen by measurement: every rank sees the same reduced
        # numbers, so they agree; rank 0 reports.
        if out is not None:
            head_ms = out["ms_per_step"]
            # a mode qualifies only when bit-exact: against the oracle when the
            # check ran, and byte-equal with the headline pipeline in any case
            ok = {m: r for m, r in results.items()
                  if m != head_mode and r.get("status") == "ok" and r.get("mismatches_vs_headline") == 0
                  and r.get("mismatches", 0) == 0}
            forced = a.halo_select if a.halo_select not in ("auto", "off") else None
            if forced == "exchange":
                forced = "slot_exchange"
            pick = None
            if forced:
                pick = forced if forced in ok else None
                why = "forced" if pick else f"forced mode {forced} not available or not bit-exact"
            elif a.halo_select == "auto" and ok:
                best = min(ok, key=lambda m: ok[m]["ms_per_step"])
                if ok[best]["ms_per_step"] < 0.97 * head_ms:
                    pick, why = best, f"{best} >=3% faster than {head_mode}"
                else:
                    why = f"{head_mode} fastest (within 3%)"
            else:
                why = "selection off" if a.halo_select == "off" else "no other mode bit-exact"
            if pick:
                r = ok[pick]
                adopted = dict(out)
                adopted.update(value=r["value"], ms_per_step=r["ms_per_step"], headline_transport=transport,
                               per_rank_ms_per_step=r["per_rank_ms_per_step"],
                               h2d_bytes_per_step=r["h2d_bytes_per_step"], d2h_bytes_per_step=r["d2h_bytes_per_step"])
                if adopted["vs_baseline"] is not None:
                    adopted["vs_baseline"] = round(r["value"] / BASELINE_MPIX, 2)
                adopted["config"] = dict(out["config"], halo_mode=pick, preload_halo=False,
                                         halo_depth=r["halo_depth"], fuse=r["fuse"],
                                         launches_per_step=r["launches_per_step"],
                                         exchanges_per_step=r["exchanges_per_step"], images_in_flight=a.slots,
                                         slot_streams=r["slot_streams"], step_graphs=r["step_graphs"],
                                         concurrent_images=r["concurrent_images"], stream_chunks=0)
                # fields measured on the pre-loaded pipeline move under its entry: every top-level
                # field describes the reported pipeline
                pre = results[head_mode]
                for k in ("latency_ms", "loop_only"):
                    pre[k] = adopted.pop(k)
                if "mismatches" in r:
                    adopted["mismatches"] = r["mismatches"]  # the adopted mode's own oracle check
                out = adopted
            out["halo_select"] = {"mode": pick or head_mode, "reason": why,
                                  "candidates": {m: results[m].get("ms_per_step") for m in results}}
            state["out"] = out
    emit(out)
    # The watchdog (N>1) stays armed through the process-group shutdown: a
    # peer stuck in the exchange can then never keep this rank alive.
    shutdown(ctx)
    if dog is not None:
        dog.cancel()

if __name__ == "__main__":
    main()
