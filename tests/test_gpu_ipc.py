"""On-device, cross-process halo exchange on ONE GPU: HIP IPC (ipc_halo.hpp).

N processes share the gpurun box's single GPU (RCCL refuses two ranks on one
device; IPC does not).  Each rank exports its slot frames with
hipIpcGetMemHandle, opens its neighbours' frames, and every exchange pulls the
neighbours' boundary rows device-to-device, ordered by flag kernels on the
rank's own stream — the path the 8-GPU node takes over xGMI, with no host
staging.  Every image of every rank is compared with the NumPy oracle, for
N = 2..8, ghost zones shallower than the repetitions (several exchanges per
image), with and without the interior || exchange split, captured graphs and
direct issue, grey / RGB and a float filter.  The reference's algorithm being
replaced: Isend/Irecv of boundary rows, inner compute, Wait, edges
(mpi/mpi_convolution.c:157-234).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from pconv.parallel.bootstrap import barrier, init_distributed, shutdown
    from pconv.parallel.dist_engine import DistributedBlur

    ctx = init_distributed("gloo")
    try:
        if cfg.get("devices"):  # one GPU per rank (the 8-GPU node's layout)
            import torch

            torch.cuda.set_device(rank % cfg["devices"])
        blur = DistributedBlur(cfg["w"], cfg["h"], cfg["ch"], cfg["filter"], cfg["reps"], rank=rank, world=world,
                               device=rank % cfg["devices"] if cfg.get("devices") else 0, halo=cfg["halo"], fuse=cfg["fuse"], slots=cfg["slots"], transport="ipc",
                               slot_exchange=True, graph_capture=cfg["graph"], slot_comm=cfg["overlap"],
                               overlap=cfg["overlap"], ipc_timeout_s=cfg.get("timeout", 30.0),
                               ipc_pull=cfg.get("pull", "grid"))
        assert all(t.pull == cfg.get("pull", "grid") for t in blur.ipc)
        info = {"self_tested": [t.self_tested for t in blur.ipc], "mailbox": [t.mailbox_kind for t in blur.ipc],
                "peer_devices": [(t.peer_device(0), t.peer_device(1)) for t in blur.ipc]}
        if cfg.get("stall") and rank == world - 1:
            barrier()  # set-up done; this rank then never exchanges
            q.put((rank, None, None, 0, info))
            barrier()
            return
        barrier()
        blur.load_synthetic(cfg["seed"])
        ks = [blur.submit(cfg["reps"]) for _ in range(cfg["images"])]
        err = None
        try:
            blur.drain()
        except Exception as e:  # noqa: BLE001 - reported to the test
            err = str(e)
        outs = [blur.outputs[k].copy() for k in ks[-cfg["slots"]:]]
        # exchanges the device performed (graph replays included), summed over slots
        q.put((rank, blur.band.y0, outs if err is None else err, sum(t.device_count for t in blur.ipc), info))
        barrier()  # every rank done with its neighbours' frames before any exits
        del blur
    finally:
        shutdown(ctx)


def _run(pconv_mod, world, cfg, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=timeout) for _ in range(world)], key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


CASES = [
    (2, "rgb", "gaussian", 8, 8, 40, True, False),     # one zone exchange per image, captured
    (2, "grey", "gaussian", 4, 4, 19, True, True),     # 5 exchanges per image, split phases, captured
    (3, "rgb", "gaussian", 6, 3, 19, False, True),     # direct issue, interior || exchange
    (4, "rgb", "box", 4, 4, 13, True, False),          # float filter
    (4, "grey", "edge", 3, 3, 11, False, False),
    (8, "rgb", "gaussian", 8, 8, 40, True, False),     # the 8-way split of the headline's shape
    (8, "grey", "gaussian", 5, 5, 23, True, True),
]


@pytest.mark.parametrize("world,ch,filt,halo,fuse,reps,graph,overlap,pull",
                         [c + ("grid",) for c in CASES] +
                         [CASES[i] + (p,) for p in ("single", "sdma") for i in (1, 2, 3, 5, 6)])
def test_ipc_halo_bit_exact(pconv_mod, world, ch, filt, halo, fuse, reps, graph, overlap, pull):
    """Every pull form: grid (the default, one dispatch of >= 8 workgroups,
    each with its own acquire), single (one workgroup) and sdma (flag kernels
    around SDMA copies)."""
    w, h, slots = 57, 160, 2
    cfg = dict(w=w, h=h, ch=ch, filter=filt, reps=reps, halo=halo, fuse=fuse, slots=slots, graph=graph,
               overlap=overlap, seed=11, images=slots + 2, pull=pull)
    if pull == "grid":
        assert pconv_mod.native.ipc_grid_workgroups(halo * 256) >= 8
    res = _run(pconv_mod, world, cfg)
    img = pconv_mod.synthetic_image(w, h, ch, seed=11)
    ref = pconv_mod.numpy_convolve(img, reps, filt).reshape(h, -1)
    per_image = -(-reps // halo)  # exchanges per image (ghost zone of `halo` rows)
    for rank, y0, outs, n_exch, info in res:
        assert not isinstance(outs, str), f"rank {rank}: {outs}"
        for o in outs:
            assert np.array_equal(o, ref[y0:y0 + o.shape[0]]), (rank, world)
        # + the connect self-test's one exchange per slot
        assert n_exch == per_image * cfg["images"] + slots, (rank, n_exch)
        assert all(info["self_tested"]) and all(k in ("uncached", "fine-grained") for k in info["mailbox"]), info


def test_ipc_connect_self_test_and_mailbox(pconv_mod):
    """Every transport runs the connect self-test (sentinel rows through the
    real protocol) and its mailbox is explicitly coherent device memory
    (uncached, or fine-grained): the words a neighbour on another GPU stores
    over xGMI.  Neighbours' devices are reported per side."""
    cfg = dict(w=40, h=96, ch="rgb", filter="gaussian", reps=4, halo=4, fuse=4, slots=2, graph=True,
               overlap=False, seed=5, images=2)
    res = _run(pconv_mod, 3, cfg)
    for rank, _, outs, _, info in res:
        assert not isinstance(outs, str), outs
        assert info["self_tested"] == [True, True], info
        assert set(info["mailbox"]) <= {"uncached", "fine-grained"}, info
        up, down = info["peer_devices"][0]
        assert (up == 0) == (rank > 0) and (down == 0) == (rank < 2), info  # -1 where no neighbour


def test_ipc_cross_device_exchange(pconv_mod):
    """One rank per GPU (frames and mailboxes reached over xGMI): the
    self-test and a bit-exact 2-way image.  Needs >= 2 visible GPUs."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (the gpurun box has one)")
    cfg = dict(w=57, h=160, ch="rgb", filter="gaussian", reps=19, halo=4, fuse=4, slots=2, graph=True,
               overlap=True, seed=7, images=3, devices=2)
    res = _run(pconv_mod, 2, cfg)
    img = pconv_mod.synthetic_image(57, 160, "rgb", seed=7)
    ref = pconv_mod.numpy_convolve(img, 19, "gaussian").reshape(160, -1)
    for rank, y0, outs, _, info in res:
        assert not isinstance(outs, str), outs
        assert info["peer_devices"][0] == ((-1, 1) if rank == 0 else (0, -1)), info
        for o in outs:
            assert np.array_equal(o, ref[y0:y0 + o.shape[0]])


@pytest.mark.parametrize("pull", ["grid", "single", "sdma"])
def test_ipc_stalled_neighbour_times_out(pconv_mod, pull):
    """A neighbour that never exchanges: the waiting rank's flag kernel gives
    up after its timeout (no wave spins forever) and drain() raises."""
    cfg = dict(w=40, h=64, ch="grey", filter="gaussian", reps=8, halo=8, fuse=8, slots=1, graph=True,
               overlap=False, seed=3, images=1, stall=True, timeout=2.0, pull=pull)
    res = _run(pconv_mod, 2, cfg, timeout=200)
    r0 = res[0]
    assert isinstance(r0[2], str) and "timed out" in r0[2], r0


def test_ipc_segments_unlinked():
    """Every IPC job unlinks its flag segment once all ranks have mapped it:
    nothing of this suite is left in /dev/shm."""
    import glob

    assert not glob.glob("/dev/shm/pconv_ipc_*") and not glob.glob("/dev/shm/pconv_conv_*")


@pytest.mark.parametrize("form,workgroups", [("grid", 0), ("grid", 8), ("grid", 13), ("grid", 64), ("single", 0),
                                             ("sdma", 0)])
@pytest.mark.parametrize("host_source", [False, True])
def test_ipc_pull_probe(pconv_mod, form, workgroups, host_source):
    """One process, self-neighbour flag protocol: each pull form moves the
    8-way headline rank's ghost zone (2 x 40 rows x 5,760 B, ~460 KB) from
    this GPU's HBM or from pinned host memory (the stand-in for a peer GPU
    behind xGMI); the probe checks the exchange count, the error word and
    every byte pulled, and returns ms per exchange."""
    n = pconv_mod.native
    ms = n.ipc_pull_probe(form, 40 * 5760, host_source, 20, 0, workgroups)
    assert 0 < ms < 50, ms


@pytest.mark.parametrize("pull", ["grid", "single", "sdma"])
@pytest.mark.parametrize("world,rank", [(8, 3), (4, 0), (2, 1), (2, 0)])
def test_ipc_self_neighbour_emulated_band_byte_placement(pconv_mod, rng, pull, world, rank):
    """The one-GPU emulation of rank `rank` of a `world`-way split (bench.py
    --emulate W:R --emulate-halo ipc): its band carries world 1 with itself
    as up and down neighbour, so the transport must take the neighbour's
    frame layout from the engine itself, not from row_band(height, 1, 0)
    (the whole image: the first version read that far past the band's
    frame).  Ghost rows above = the band's own last `halo` rows, below = its
    first `halo` rows, every byte; an edge rank keeps its single neighbour
    (the first version's one-sided self-signalling timed out); also captured
    in the rep-loop graph."""
    import torch

    from pconv.parallel.bootstrap import make_ipc_transports

    n = pconv_mod.native
    w, h, halo = 57, 400, 12
    b = n.row_band(h, world, rank)
    has_up, has_down = b.up >= 0, b.down >= 0  # an edge rank keeps its one neighbour (itself)
    b.up, b.down, b.rank, b.world = (0 if has_up else -1), (0 if has_down else -1), 0, 1
    eng = n.BandEngine.for_band(w, h, "rgb", "gaussian", b, 0, halo, 4, False, "auto", graph=True,
                                capture_exchanges=True)
    (t,) = make_ipc_transports([eng], 10.0, pull=pull)
    eng.attach_transport(t)
    rb = w * 3
    owned = rng.integers(0, 256, size=(b.rows, rb), dtype=np.uint8)
    eng.upload(owned.reshape(-1), 0, b.rows)
    eng.exchange_now(eng.compute_stream)
    eng.synchronize()
    t.check()
    got = np.empty((b.rows + 2 * halo, rb), np.uint8)
    eng.read_frame(got.reshape(-1), -halo, b.rows + halo)
    assert np.array_equal(got[:halo], owned[-halo:] if has_up else 0 * owned[:halo]), "ghost rows above"
    assert np.array_equal(got[halo:halo + b.rows], owned)
    assert np.array_equal(got[-halo:], owned[:halo] if has_down else 0 * owned[:halo]), "ghost rows below"
    for _ in range(3):  # exchanges captured with the launches: capture, replay, other parity
        eng.set_halo_valid(False)
        eng.run(8)
        eng.synchronize()
        t.check()
        assert eng.stats.exchanges >= 1 and eng.cached_graphs >= 1
    del t, eng
    torch.cuda.synchronize()
