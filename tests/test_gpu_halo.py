"""Halo-exchange paths on the GPU: the RCCL transport's byte placement (a
1-rank communicator whose band is its own up/down neighbour: ncclSend/ncclRecv
to self), the production phase path (comm stream || interior launch, edge
launches after the halo event) driven by a device-asynchronous transport, the
tuning-vs-graph input hazard and the pre-load range check.

Reference behaviour being replaced: MPI_Isend/Irecv of the boundary rows,
inner compute, MPI_Wait, edge compute (mpi/mpi_convolution.c:156-240)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from halo_oracle import reflected_ghost_oracle

pytestmark = pytest.mark.gpu


def _self_band(n, h):
    b = n.Band()
    b.rank, b.world, b.y0, b.rows, b.up, b.down = 0, 1, 0, h, 0, 0
    return b


@pytest.mark.parametrize("ch,w,h,halo", [("rgb", 61, 40, 3), ("grey", 1920, 64, 8), ("rgba", 33, 17, 5)])
def test_rccl_self_exchange_byte_placement(pconv_mod, rng, ch, w, h, halo):
    """RcclTransport::exchange with peer == self: ghost rows above must hold
    the band's top `halo` rows (sent 'up', received 'from up') and ghost rows
    below its bottom rows — every byte, pads excluded."""
    n = pconv_mod.native
    c = {"grey": 1, "rgb": 3, "rgba": 4}[ch]
    comm = n.RcclComm(n.rccl_unique_id(), 0, 1, 0)
    eng = n.BandEngine.for_band(w, h, ch, "gaussian", _self_band(n, h), 0, halo, 1, True, "auto")
    eng.attach_rccl(comm)
    img = rng.integers(0, 256, size=(h, w * c), dtype=np.uint8)
    eng.upload(img.reshape(-1), 0, h)
    eng.synchronize()
    # one exchange through the production path: a 1-step run starts with it
    plan = eng.plan(1)
    assert plan[0].exchange_depth == halo
    frame = np.zeros((h + 2 * halo, w * c), np.uint8)
    eng.exchange_now()  # the full ghost zone, on the comm stream
    comm.wait(eng.comm_stream, 60.0)
    eng.read_frame(frame.reshape(-1), -halo, h + halo)
    assert np.array_equal(frame[:halo], img[:halo])
    assert np.array_equal(frame[halo:halo + h], img)
    assert np.array_equal(frame[halo + h:], img[h - halo:])


@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("reps,halo,fuse", [(13, 4, 4), (20, 8, 8), (5, 1, 1)])
def test_rccl_self_band_runs_exact(pconv_mod, rng, overlap, reps, halo, fuse):
    """A whole run whose every exchange phase goes through RCCL send/recv on
    the comm stream, overlapped (split launches) with the interior kernel.
    Ghost rows of a self-neighbour band lie outside the image, where the
    kernel forces zeros, so the result must equal the zero-padded oracle."""
    n = pconv_mod.native
    w, h = 57, 48
    comm = n.RcclComm(n.rccl_unique_id(), 0, 1, 0)
    eng = n.BandEngine.for_band(w, h, "rgb", "gaussian", _self_band(n, h), 0, halo, fuse, overlap, "auto")
    eng.attach_rccl(comm)
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    eng.upload(img.reshape(-1), 0, h)
    eng.run(reps)
    comm.wait(eng.comm_stream, 60.0)
    comm.wait(eng.compute_stream, 60.0)
    eng.synchronize()
    assert eng.stats.exchanges == len([p for p in eng.plan(reps) if p.exchange_depth])
    assert eng.stats.exchanges >= 1
    out = np.empty_like(img)
    eng.download(out.reshape(-1), 0, h)
    eng.synchronize()
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps))


def _mid_band(n, y0, rows):
    """A band in the MIDDLE of a taller image whose up and down neighbour is
    itself (1-rank communicator): RCCL send/recv-to-self then delivers the
    band's own top rows as its ghost rows above and its bottom rows as its
    ghost rows below.  Those ghost rows lie INSIDE the image, so the kernel
    reads them (no zero boundary there) and the result depends on every byte
    RCCL delivered, at every exchange phase."""
    b = n.Band()
    b.rank, b.world, b.y0, b.rows, b.up, b.down = 0, 1, y0, rows, 0, 0
    return b


@pytest.fixture(scope="module")
def self_comm(pconv_mod):
    import gc

    n = pconv_mod.native
    c = n.RcclComm(n.rccl_unique_id(), 0, 1, 0)
    yield c
    # communicators hold device queues and proxy threads: release them before
    # later tests (the multi-process ones) open their own
    del c
    gc.collect()


@pytest.fixture(autouse=True)
def _release_native_objects():
    """Collect every engine / pipeline / communicator a test created when it
    ends (their streams and RCCL resources are process-wide)."""
    import gc

    yield
    gc.collect()


@pytest.mark.parametrize("ch,w", [("rgb", 57), ("grey", 1920)])
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("reps,halo,fuse", [(13, 4, 4), (20, 8, 8), (5, 1, 1), (17, 6, 3), (40, 40, 8), (24, 12, 8)])
def test_rccl_mid_image_band_consumes_exchanged_rows(pconv_mod, rng, self_comm, ch, w, overlap, reps, halo, fuse):
    """The RCCL-received ghost rows are CONSUMED: a mid-image self-neighbour
    band (y0 > 0, y0 + rows < height) runs every exchange phase through
    ncclSend/ncclRecv on the comm stream — with overlap, the interior launch
    concurrently and the edge launches after ev_halo — and must equal the
    reflected-ghost oracle byte for byte.  The reference's loop being replaced:
    Isend/Irecv, inner compute, Wait, edges (mpi/mpi_convolution.c:156-240)."""
    n = pconv_mod.native
    c = {"grey": 1, "rgb": 3}[ch]
    y0, rows, height = 37, 48, 130
    eng = n.BandEngine.for_band(w, height, ch, "gaussian", _mid_band(n, y0, rows), 0, halo, fuse, overlap, "auto")
    eng.attach_rccl(self_comm)
    owned = rng.integers(0, 256, size=(rows, w * c), dtype=np.uint8)
    plan = eng.plan(reps)
    n_ex = len([p for p in plan if p.exchange_depth])
    assert n_ex >= 1
    if overlap and eng.halo < reps:
        assert any(len(p.launches) > 1 and any(l.after_halo for l in p.launches) for p in plan if p.exchange_depth)
    ref = reflected_ghost_oracle(n, plan, eng.halo, owned, y0, height, ch)
    # the oracle really depends on the exchanged rows: zero ghost rows differ
    assert not np.array_equal(ref, pconv_mod.numpy_convolve(owned.reshape(rows, w, c) if c > 1 else owned, reps)
                              .reshape(rows, -1))
    for _ in range(2):  # twice: the second run starts from the other frame parity
        eng.upload(owned.reshape(-1), 0, rows)
        eng.run(reps)
        self_comm.wait(eng.comm_stream, 60.0)
        self_comm.wait(eng.compute_stream, 60.0)
        eng.synchronize()
        assert eng.stats.exchanges == n_ex
        out = np.empty_like(owned)
        eng.download(out.reshape(-1), 0, rows)
        eng.synchronize()
        bad = int(np.count_nonzero(out != ref))
        assert bad == 0, f"{bad} bytes differ from the reflected-ghost oracle"


@pytest.mark.parametrize("ch,w", [("rgb", 57), ("grey", 1920)])
@pytest.mark.parametrize("reps,halo,fuse", [(13, 4, 4), (20, 8, 8), (40, 40, 8), (24, 12, 8)])
@pytest.mark.parametrize("overlap", [False, True])
def test_rccl_band_exchanges_captured_in_the_loop_graph(pconv_mod, rng, self_comm, ch, w, reps, halo, fuse, overlap):
    """EngineOptions::capture_exchanges (bench.py's resident loop): the
    exchange phases' ncclSend/ncclRecv are captured with the launches into
    the cached rep-loop graph — in stream order on the compute stream, or
    (overlap) forked: the interior launch on the communication stream beside
    the exchange, the edge strips after it — the first run captures, later
    runs (both frame parities) replay; every run equals the reflected-ghost
    oracle byte for byte and counts its exchanges."""
    n = pconv_mod.native
    c = {"grey": 1, "rgb": 3}[ch]
    y0, rows, height = 37, 48, 130
    eng = n.BandEngine.for_band(w, height, ch, "gaussian", _mid_band(n, y0, rows), 0, halo, fuse, overlap, "auto",
                                graph=True, capture_exchanges=True)
    eng.attach_rccl(self_comm)
    # exchanges in stream order with the launches, or beside the interior launch
    assert (eng.comm_stream == eng.compute_stream) == (not overlap)
    owned = rng.integers(0, 256, size=(rows, w * c), dtype=np.uint8)
    plan = eng.plan(reps)
    n_ex = len([p for p in plan if p.exchange_depth])
    ref = reflected_ghost_oracle(n, plan, eng.halo, owned, y0, height, ch)
    for i in range(4):  # capture, replay, and the other frame parity
        eng.upload(owned.reshape(-1), 0, rows)
        eng.run(reps)
        self_comm.wait(eng.compute_stream, 60.0)
        eng.synchronize()
        assert eng.stats.exchanges == n_ex and eng.cached_graphs >= 1, (i, eng.stats.exchanges, eng.cached_graphs)
        out = np.empty_like(owned)
        eng.download(out.reshape(-1), 0, rows)
        eng.synchronize()
        assert np.array_equal(out, ref), i


@pytest.mark.parametrize("bands", [2, 3, 5, 8])
@pytest.mark.parametrize("halo,fuse,overlap,preload", [(1, 1, True, False), (4, 4, True, False), (8, 4, True, True),
                                                       (6, 3, False, False), (16, 8, True, False)])
def test_local_cluster_device_async(pconv_mod, rng, bands, halo, fuse, overlap, preload):
    """Bands on one device through the PRODUCTION phase path with a transport
    that is asynchronous on the device (D2D copies on each band's comm
    stream): nothing synchronises on the host between phases, so the
    ev_ready / ev_halo / per-phase neighbour events are all that keeps the
    result exact."""
    n = pconv_mod.native
    h, w = 23 * bands + 11, 45
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    cl = n.LocalCluster(w, h, "rgb", "gaussian", bands, 0, halo, fuse, "auto", overlap)
    for reps in (1, 6, 13, 30):
        cl.upload(img.reshape(-1), preload)
        cl.run(reps, True)
        out = np.empty_like(img)
        cl.download(out.reshape(-1))
        assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps)), (bands, halo, fuse, reps)


def test_local_cluster_device_async_large(pconv_mod, rng):
    """Long bands (interior launches much longer than the halo copies): the
    interior kernel really runs while the copy is in flight."""
    n = pconv_mod.native
    w, h, reps = 1920, 2520, 40
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    cl = n.LocalCluster(w, h, "rgb", "gaussian", 4, 0, 16, 8, "auto", True)
    cl.upload(img.reshape(-1), False)
    cl.run(reps, True)
    out = np.empty_like(img)
    cl.download(out.reshape(-1))
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps))


def test_graph_tuning_never_touches_the_input(pconv_mod, rng):
    """A captured run whose launches are tuned on first use: tuning must not
    write into the uploaded frame.  reps=10 with fuse=8 gives an odd second
    phase (2 steps) on a fresh geometry after the tuning cache is cleared."""
    n = pconv_mod.native
    n.clear_swar_tuning()
    w, h = 211, 97
    eng = pconv_mod.Engine(w, h, "rgb", device=0, fuse=8, graph=True)
    for reps in (10, 13, 10):
        img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        assert np.array_equal(eng(img, reps), pconv_mod.numpy_convolve(img, reps)), reps
        n.clear_swar_tuning()


def test_process_graph_rejects_partial_preload(pconv_mod):
    """Input rows must be exactly the owned rows or the owned rows plus the
    full ghost zone on both sides; anything else would silently compute from
    stale ghost rows."""
    n = pconv_mod.native
    eng = n.BandEngine(40, 90, "grey", "gaussian", 1, 3, 0, halo=8, fuse=4)
    b = eng.band
    assert not eng.input_preloaded(0, b.rows)
    assert eng.input_preloaded(-8, b.rows + 8)
    buf = n.PinnedBuffer((b.rows + 16) * 40)
    out = n.PinnedBuffer(b.rows * 40)
    for r0, r1 in ((-1, b.rows), (-8, b.rows), (0, b.rows + 8), (-4, b.rows + 4)):
        with pytest.raises(RuntimeError, match="ghost zone"):
            eng.process_graph(buf.ptr, r0, r1, out.ptr, 4)
    top = n.BandEngine(40, 90, "grey", "gaussian", 0, 3, 0, halo=8, fuse=4)
    assert top.input_preloaded(0, top.band.rows + 8)


def test_rccl_loaded_lazily(tmp_path):
    """The 1-GPU `conv` binary never maps librccl (it is dlopen'ed on the
    first RCCL call; the binary does not link it).  Python processes map
    torch's own copy at `import torch`, so the CLI is where this shows."""
    from conftest import CONV_BIN

    r = subprocess.run([CONV_BIN, "x.raw", "64", "48", "3", "grey", "--synthetic", "1", "--json", "--quiet",
                        "--out", str(tmp_path / "o.raw")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["rccl_loaded"] is False


def test_cli_gpu1_phase_breakdown(pconv_mod, tmp_path):
    """`conv --json` reports where the end-to-end time goes; the phases sum to
    (at most) the e2e time."""
    from conftest import CONV_BIN

    r = subprocess.run([CONV_BIN, "x.raw", "640", "480", "10", "grey", "--synthetic", "3", "--json", "--quiet",
                        "--out", str(tmp_path / "o.raw")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    ph = meta["phases_s"]
    for k in ("hip_init", "pinned_alloc", "synthesize", "queue", "device_alloc", "h2d", "loop", "d2h", "write"):
        assert k in ph and ph[k] >= 0
    assert sum(ph.values()) <= meta["e2e_s"] + 1e-3
    assert meta["since_exec_s"] >= meta["e2e_s"] - 0.02


@pytest.mark.parametrize("extra", [["--gpus", "2", "--transport", "shm"], ["--gpus", "3", "--transport", "shm",
                                                                           "--exchange-halo"]])
def test_cli_multi_rank_checkpoints(pconv_mod, tmp_path, rng, extra):
    """--checkpoint-every under --gpus N: every <out>.repK holds the whole
    image after K repetitions (each rank pwrites its band)."""
    from conftest import CONV_BIN

    img = rng.integers(0, 256, size=(53, 41, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "im.raw"), img)
    r = subprocess.run([CONV_BIN, "im.raw", "41", "53", "11", "rgb", "--checkpoint-every", "4", "--check",
                        "--json"] + extra, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for k in (4, 8):
        got = pconv_mod.read_raw(str(tmp_path / f"blur_im.raw.rep{k}"), 41, 53, "rgb")
        assert np.array_equal(got, pconv_mod.numpy_convolve(img, k)), k
    assert not (tmp_path / "blur_im.raw.rep12").exists()
    out = pconv_mod.read_raw(str(tmp_path / "blur_im.raw"), 41, 53, "rgb")
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 11))


def _port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("height,mode", [(1200, "preload"), (1200, "exchange"), (200, "preload")])
def test_bench_four_ranks_100_reps(height, mode):
    """The verdict's bar for the multi-GPU path: 4 ranks, 100 repetitions, a
    tall image, both halo modes, 0 mismatches.  height 200 gives 50-row bands,
    shorter than the 100 repetitions: pre-loading cannot cover them, so the
    headline exchanges halos through the transport instead of crashing."""
    port = _port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "4", "--steps", "3", "--warmup", "1", "--transport", "gloo-host", "--check", "--reps", "100",
           "--width", "96", "--height", str(height), "--halo-mode", mode, "--exchange-check", "off"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    meta = json.loads(lines[0])
    assert meta["n_gpus"] == 4 and meta["mismatches"] == 0
    assert "96x%d RGB, 100 reps" % height in meta["metric"] and meta["vs_baseline"] is None
    if mode == "preload" and height == 1200:
        assert meta["headline_transport"] == "none" and meta["config"]["halo_depth"] >= 100
    else:
        assert meta["headline_transport"] == "gloo-host" and meta["config"]["exchanges_per_step"] >= 1


def test_bench_spawns_its_ranks():
    """`bench.py --gpus 2` with no launcher starts its own two ranks."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--transport", "gloo-host", "--width", "64", "--height", "120", "--reps", "8", "--exchange-check", "off",
           "--check"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    meta = json.loads(lines[0])
    assert meta["n_gpus"] == 2 and meta["mismatches"] == 0
    assert meta["latency_ms"] > 0 and meta["copy_floor"]["floor_ms"] > 0


@pytest.mark.parametrize("w,h,ch", [(61, 45, "rgb"), (1920, 64, "grey"), (33, 17, "rgba"), (1, 1, "grey"),
                                    (257, 300, "rgb")])
def test_kernel_copies_bit_exact(pconv_mod, rng, w, h, ch):
    """Host<->frame copies by CU kernels (the one-shot CLI path): unaligned
    row sizes and pinned or pageable host buffers, every byte exact, nothing
    written past the host rows (guard bytes)."""
    n = pconv_mod.native
    c = {"grey": 1, "rgb": 3, "rgba": 4}[ch]
    eng = n.BandEngine(w, h, ch, "gaussian", 0, 1, 0, halo=8, fuse=8, kernel_copies=True)
    img = rng.integers(0, 256, size=h * w * c, dtype=np.uint8)
    pin_in, pin_out = n.PinnedBuffer(img.size + 64), n.PinnedBuffer(img.size + 64)
    np.asarray(pin_in)[:img.size] = img
    np.asarray(pin_out)[:] = 0xAB
    eng.upload_ptr(pin_in.ptr, w * c, 0, h)
    eng.run(11)
    eng.download_ptr(pin_out.ptr, w * c, 0, h)
    eng.synchronize()
    got = np.asarray(pin_out)
    ref = pconv_mod.numpy_convolve(img.reshape(h, w, c) if c > 1 else img.reshape(h, w), 11).reshape(-1)
    assert np.array_equal(got[:img.size], ref)
    assert (got[img.size:] == 0xAB).all()


@pytest.mark.parametrize("copies", ["kernel", "sdma"])
def test_cli_copies_modes(pconv_mod, tmp_path, rng, copies):
    from conftest import CONV_BIN

    img = rng.integers(0, 256, size=(77, 61, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "img.raw"), img)
    r = subprocess.run([CONV_BIN, "img.raw", "61", "77", "9", "rgb", "--copies", copies, "--json", "--check"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    assert meta["copies"] == copies and meta["mismatches"] == 0


# --------------------------------------------------------------------------
# The RCCL self-tests on BOTH stacks: this (torch) process runs torch's bundled
# HIP runtime and librccl; the `conv` CLI runs ROCm's own.  Each compares the
# bytes RCCL delivered and the kernels consumed with the reflected-ghost model.

def test_rccl_selftests_torch_stack(pconv_mod):
    n = pconv_mod.native
    ex = json.loads(n.rccl_selftest_exchange(0))
    assert ex["status"] == "ok" and ex["cases"] >= 7 and ex["exchanges"] >= 14
    # three communicators (one per slot stream) in flight together, 60 exchange images per case
    mc = json.loads(n.rccl_selftest_multicomm(0, 3, 60, 60.0))
    assert mc["status"] == "ok" and mc["communicators"] == 3 and mc["images_per_case"] == 60
    info = n.runtime_info()
    assert info["rccl_path"] and info["rccl_version"] == ex["rccl_version"]


@pytest.mark.parametrize("name", ["rccl-exchange", "rccl-multicomm"])
def test_rccl_selftests_cli_stack(name):
    from conftest import CONV_BIN

    r = subprocess.run([CONV_BIN, "--selftest", name, "--slots", "3", "--images", "60"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines[0]["status"] == "ok" and lines[-1]["status"] == "ok"
    # the CLI binds ROCm's librccl / HIP runtime, not torch's copies
    assert "torch" not in lines[0]["rccl_path"] and "torch" not in lines[-1]["hip_runtime_path"]


@pytest.mark.parametrize("captured,slot_comm", [(True, False), (False, False), (True, True), (False, True)])
@pytest.mark.parametrize("reps,halo,fuse", [(40, 40, 8), (20, 8, 4), (13, 13, 4), (24, 8, 8)])
def test_slot_pipeline_rccl_exchange_images(pconv_mod, captured, slot_comm, reps, halo, fuse):
    """Slot-exchange pipeline on a mid-image self-neighbour band, one 1-rank
    communicator per slot stream (three in flight together): images issued
    directly, or each captured as ONE hipGraph (upload, ncclSend/ncclRecv of
    the ghost zone, launches, download — BandEngine::process_graph).  Every
    image equals the reflected-ghost oracle.  slot_comm: each slot also has a
    communication stream, an exchange phase's interior launch runs beside the
    exchange and the edges after the halo event (captured: the reference's
    per-phase loop as ONE graph with a fork/join per exchange)."""
    n = pconv_mod.native
    w, height, y0, rows, slots = 301, 520, 211, 96, 3
    pipe = n.BandPipeline(w, height, "rgb", "gaussian", 0, 1, 0, halo=halo, fuse=fuse, slots=slots, graphs=True,
                          step_graphs=captured, band=_mid_band(n, y0, rows), slot_comm=slot_comm)
    assert pipe.step_graphs == captured
    comms = [n.RcclComm(n.rccl_unique_id(), 0, 1, 0) for _ in range(slots)]
    for k, c in enumerate(comms):
        pipe.attach_slot_rccl(k, c)
    e0 = pipe.slot(0)
    zone = e0.exchange_free(reps, True)
    e0.set_halo_valid(zone)
    plan = e0.plan(reps)
    e0.set_halo_valid(False)
    rb = e0.row_bytes
    rng = np.random.default_rng(reps * 100 + halo)
    ins = [n.PinnedBuffer(rows * rb) for _ in range(slots)]
    outs = [n.PinnedBuffer(rows * rb) for _ in range(slots)]
    refs = []
    for k in range(slots):
        owned = rng.integers(0, 256, size=(rows, rb), dtype=np.uint8)
        np.asarray(ins[k])[:] = owned.reshape(-1)
        refs.append(reflected_ghost_oracle(n, plan, e0.halo, owned, y0, height, "rgb",
                                           pre_exchange=e0.halo if zone else 0))
    for rnd in range(4):
        for k in range(slots):
            np.asarray(outs[k])[:] = 0
            pipe.submit(ins[k].ptr, 0, rows, outs[k].ptr, reps)
        for k, c in enumerate(comms):
            c.wait(pipe.slot(k).compute_stream, 60.0)
        pipe.drain()
        for k in range(slots):
            got = np.asarray(outs[k]).reshape(rows, rb)
            bad = int(np.count_nonzero(got != refs[k]))
            assert bad == 0, (rnd, k, bad)
    st = pipe.slot(0).stats
    assert st.exchanges == (1 if zone else len([p for p in plan if p.exchange_depth]))
    if slot_comm and not zone:  # split exchange phases: interior || exchange, edges after the halo event
        assert any(len(p.launches) > 1 for p in plan if p.exchange_depth)
    if captured:
        assert pipe.slot(0).cached_step_graphs >= 1
