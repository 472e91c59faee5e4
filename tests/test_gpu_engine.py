"""Engine-level GPU tests: convolve() on numpy and CUDA tensors, graphs,
one-device multi-band emulation (LocalCluster), RCCL single-rank, CLI."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import CONV_BIN

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(1, 1), (7, 3), (2520 // 8, 1920 // 8, 3), (61, 77, 3), (33, 50, 4), (100, 129)])
@pytest.mark.parametrize("reps", [0, 1, 2, 7, 40])
def test_convolve_hip_numpy(pconv_mod, rng, shape, reps):
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    got = pconv_mod.convolve(img, reps, backend="hip")
    assert np.array_equal(got, pconv_mod.numpy_convolve(img, reps))


@pytest.mark.parametrize("filt", ["gaussian", "box", "edge"])
def test_convolve_hip_tensor(pconv_mod, rng, filt):
    import torch

    img = rng.integers(0, 256, size=(45, 67, 3), dtype=np.uint8)
    x = torch.from_numpy(img).cuda()
    y = pconv_mod.convolve(x, 9, filter=filt)
    assert y.is_cuda and y.dtype == torch.uint8
    assert np.array_equal(y.cpu().numpy(), pconv_mod.numpy_convolve(img, 9, filt))
    assert np.array_equal(x.cpu().numpy(), img)  # input untouched


def test_engine_graph_cache_bounded(pconv_mod, rng):
    """Graphs are cached per (reps, start buffer): many distinct repetition
    counts must not grow the cache past its bound, and results stay exact
    across the eviction."""
    eng = pconv_mod.Engine(37, 29, "grey", device=0, fuse=4, graph=True)
    cap = eng._eng.max_cached_graphs
    img = rng.integers(0, 256, size=(29, 37), dtype=np.uint8)
    for reps in range(1, cap + 12):
        got = eng.run_numpy(img, reps)
        assert eng._eng.cached_graphs <= cap
        if reps in (1, cap - 1, cap, cap + 1, cap + 11):
            assert np.array_equal(got, pconv_mod.numpy_convolve(img, reps)), reps
    assert eng._eng.cached_graphs < cap


@pytest.mark.parametrize("fuse", [1, 2, 5, 8])
@pytest.mark.parametrize("graph", [False, True])
def test_engine_reuse_fuse_graph(pconv_mod, rng, fuse, graph):
    eng = pconv_mod.Engine(53, 41, "rgb", device=0, fuse=fuse, graph=graph)
    for reps in (1, 3, 8, 17, 8):
        img = rng.integers(0, 256, size=(41, 53, 3), dtype=np.uint8)
        assert np.array_equal(eng(img, reps), pconv_mod.numpy_convolve(img, reps)), (fuse, graph, reps)


@pytest.mark.parametrize("bands", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("halo,fuse,preload", [(1, 1, False), (4, 1, True), (4, 4, False), (8, 4, True)])
def test_local_cluster_bit_exact(pconv_mod, rng, bands, halo, fuse, preload):
    n = pconv_mod.native
    img = rng.integers(0, 256, size=(70, 45, 3), dtype=np.uint8)
    cl = n.LocalCluster(45, 70, "rgb", "gaussian", bands, 0, halo, fuse)
    for reps in (1, 6, 13):
        cl.upload(img.reshape(-1), preload)
        cl.run(reps)
        out = np.empty_like(img)
        cl.download(out.reshape(-1))
        assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps)), (bands, halo, fuse, reps)


def test_local_cluster_float_filter(pconv_mod, rng):
    n = pconv_mod.native
    img = rng.integers(0, 256, size=(40, 31), dtype=np.uint8)
    cl = n.LocalCluster(31, 40, "grey", "box", 4, 0, 3, 1)
    cl.upload(img.reshape(-1), False)
    cl.run(7)
    out = np.empty_like(img)
    cl.download(out.reshape(-1))
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 7, "box"))


def test_rccl_single_rank_and_dist_engine(pconv_mod):
    from pconv.parallel.dist_engine import DistributedBlur

    n = pconv_mod.native
    comm = n.RcclComm(n.rccl_unique_id(), 0, 1, 0)
    assert comm.allreduce_max(3.5) == 3.5 and comm.allreduce_sum(2.0) == 2.0
    comm.barrier()
    blur = DistributedBlur(96, 50, "rgb", "gaussian", 12, rank=0, world=1, device=0)
    blur.load_synthetic(3)
    blur.step(12)
    ref = pconv_mod.numpy_convolve(pconv_mod.synthetic_image(96, 50, "rgb", seed=3), 12)
    assert np.array_equal(blur.output.reshape(ref.shape), ref)


def test_cli_hip(pconv_mod, tmp_path, rng):
    img = rng.integers(0, 256, size=(77, 61, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "img.raw"), img)
    for extra in ([], ["--graph"], ["--fuse", "3"], ["--gpus", "1", "--format", "both"]):
        r = subprocess.run([CONV_BIN, "img.raw", "61", "77", "11", "rgb", "--check", "--json"] + extra,
                           cwd=tmp_path, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert "Execution time:" in r.stdout
        meta = json.loads(r.stdout.strip().splitlines()[-1])
        assert meta["mismatches"] == 0
        out = pconv_mod.read_raw(str(tmp_path / "blur_img.raw"), 61, 77, "rgb")
        assert np.array_equal(out, pconv_mod.numpy_convolve(img, 11))


@pytest.mark.parametrize("typ,filt,chunk", [("rgb", "gaussian", 30000), ("grey", "gaussian", 5000),
                                            ("rgb", "edge", 65536), ("grey", "box", 1)])
def test_cli_hip_ring_staging(pconv_mod, tmp_path, rng, typ, filt, chunk):
    """One-shot run through a ring of small pinned chunks (read chunk k+1 ||
    upload chunk k; download chunk k+1 || write chunk k): chunk sizes that
    leave a remainder, one row per chunk, a file input (not synthetic)."""
    c = 3 if typ == "rgb" else 1
    w, h = 203, 311
    img = rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "img.raw"), img)
    r = subprocess.run([CONV_BIN, "img.raw", str(w), str(h), "13", typ, "--filter", filt, "--json",
                        "--ring-chunk-bytes", str(chunk)], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    assert "read_and_h2d" in meta["phases_s"] and "d2h_and_write" in meta["phases_s"], meta["phases_s"]
    out = pconv_mod.read_raw(str(tmp_path / "blur_img.raw"), w, h, typ)
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 13, filt))


@pytest.mark.parametrize("transport,extra", [
    ("shm", ["--gpus", "2"]),
    ("shm", ["--gpus", "3", "--exchange-halo"]),
    ("shm", ["--gpus", "4", "--halo", "2", "--fuse", "2"]),
    ("shm", ["--gpus", "2", "--filter", "box"]),
    ("shm", ["--gpus", "3", "--no-overlap", "--exchange-halo", "--filter", "edge"]),
    ("ipc", ["--gpus", "2", "--exchange-halo"]),
    ("ipc", ["--gpus", "3", "--exchange-halo", "--halo", "2", "--fuse", "2"]),
    ("ipc", ["--gpus", "4", "--exchange-halo", "--no-overlap", "--filter", "box"]),
    ("ipc", ["--gpus", "5", "--halo", "3", "--fuse", "3", "--checkpoint-every", "5"]),
])
def test_cli_multi_rank_shm(pconv_mod, tmp_path, rng, transport, extra):
    """Native fork launcher, several ranks on one GPU: host-staged shm halos,
    or device-side IPC pulls of the neighbours' rows (ipc_halo.hpp) —
    exchanges at every phase with --exchange-halo / shallow halos."""
    img = rng.integers(0, 256, size=(77, 61, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "img.raw"), img)
    r = subprocess.run([CONV_BIN, "img.raw", "61", "77", "13", "rgb", "--transport", transport, "--check", "--json",
                        "--timeout", "30"] + extra, cwd=tmp_path, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    assert meta["mismatches"] == 0
    assert meta["gpus"] == int(extra[1])
    if "--exchange-halo" in extra or "--halo" in extra:
        assert meta["exchanges"] >= 1
    filt = extra[extra.index("--filter") + 1] if "--filter" in extra else "gaussian"
    out = pconv_mod.read_raw(str(tmp_path / "blur_img.raw"), 61, 77, "rgb")
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 13, filt))


@pytest.mark.parametrize("slots,reps,fuse", [(1, 5, 8), (2, 13, 8), (3, 7, 4), (3, 0, 8)])
def test_pipeline_step_graphs(pconv_mod, rng, slots, reps, fuse):
    """Whole-step hipGraphs on per-slot streams: every image bit-exact, across
    graph-cache hits and both start frames (odd phase counts flip them)."""
    from pconv.parallel.dist_engine import DistributedBlur

    w, h = 67, 45
    blur = DistributedBlur(w, h, "rgb", "gaussian", reps, rank=0, world=1, device=0, fuse=fuse, slots=slots,
                           step_graphs=True)
    assert blur.pipe.graphs
    for rnd in range(3):
        imgs = [rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for _ in range(slots)]
        ks = []
        for i, img in enumerate(imgs):
            k = blur._next
            blur.load_image(img, slot=k)
            ks.append(blur.submit(reps))
        blur.drain()
        for img, k in zip(imgs, ks):
            assert np.array_equal(blur.outputs[k].reshape(h, w, 3), pconv_mod.numpy_convolve(img, reps)), (rnd, k)


def test_pipeline_step_graphs_preloaded_band(pconv_mod, rng):
    """A middle band of a 3-way split with pre-loaded ghost rows >= reps runs
    as step graphs and matches the oracle rows (no transport involved)."""
    from pconv.parallel.dist_engine import DistributedBlur

    w, h, reps = 53, 90, 11
    img = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    blur = DistributedBlur(w, h, "grey", "gaussian", reps, rank=1, world=3, device=0, halo=reps, fuse=4,
                           preload_halo=True, slots=2, transport="none")
    assert blur.pipe.graphs
    blur.load_image(img)
    out = blur.step(reps)
    b = blur.band
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps)[b.y0:b.y0 + b.rows])


@pytest.mark.parametrize("capture", [True, False])
def test_pipeline_slot_streams_direct_and_graph(pconv_mod, rng, capture):
    """Slot-stream pipeline with and without whole-step graph capture."""
    from pconv.parallel.dist_engine import DistributedBlur

    w, h, reps = 71, 52, 10
    blur = DistributedBlur(w, h, "rgb", "gaussian", reps, rank=0, world=1, device=0, slots=3, step_graphs=True,
                           graph_capture=capture)
    assert blur.pipe.graphs and blur.pipe.step_graphs == capture
    imgs = [rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for _ in range(3)]
    ks = []
    for img in imgs:
        blur.load_image(img, slot=blur._next)
        ks.append(blur.submit(reps))
    blur.drain()
    for img, k in zip(imgs, ks):
        assert np.array_equal(blur.outputs[k].reshape(h, w, 3), pconv_mod.numpy_convolve(img, reps))


def test_pipeline_staging_qualification(pconv_mod, rng):
    """DistributedBlur(qualify_staging=True): every slot's pinned buffers are
    timed through the copy engines at set-up (H2D alone, D2H alone, pair) and
    slow ones replaced; the numpy views follow the buffers that survived, so
    images loaded afterwards come back bit-exact from every slot."""
    from pconv.parallel.dist_engine import DistributedBlur

    w, h, reps = 301, 120, 9
    blur = DistributedBlur(w, h, "rgb", "gaussian", reps, rank=0, world=1, device=0, slots=4, step_graphs=True,
                           qualify_staging=True)
    st = blur.staging
    assert st is not None and st["replaced"] >= 0
    for key in ("h2d_d2h_pair_ms_first", "h2d_d2h_pair_ms"):
        assert len(st[key]) == 4 and all(len(r) == 3 and min(r) > 0 for r in st[key]), st
    assert len(st["fresh_ms"]) == 3 and min(st["fresh_ms"]) > 0  # the fresh-buffer reference
    for k in range(4):
        assert blur.inputs[k].ctypes.data == blur._in[k].ptr and blur.outputs[k].ctypes.data == blur._out[k].ptr
    imgs = [rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for _ in range(4)]
    ks = []
    for img in imgs:
        blur.load_image(img, slot=blur._next)
        ks.append(blur.submit(reps))
    blur.drain()
    for img, k in zip(imgs, ks):
        assert np.array_equal(blur.outputs[k].reshape(h, w, 3), pconv_mod.numpy_convolve(img, reps))


@pytest.mark.parametrize("lazy", [False, True])
def test_pipeline_per_image_completion(pconv_mod, rng, lazy):
    """Slot-stream pipeline: every image ends in its slot's completion event
    — wait_image(k) makes that image's output final without draining the
    others, ready(k) reports it; completion marks (the bench's diagnostic
    pass) give one time per image, increasing.  The burst's first image is
    row-streamed when issued eagerly, a step graph when held (lazy_head)."""
    from pconv.parallel.dist_engine import DistributedBlur

    w, h, reps = 97, 88, 16
    blur = DistributedBlur(w, h, "rgb", "gaussian", reps, rank=0, world=1, device=0, slots=4, step_graphs=True,
                           stream_chunks=4, stream_min_bytes=0, lazy_head=lazy)
    imgs = [rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for _ in range(4)]
    for k, img in enumerate(imgs):
        blur.load_image(img, slot=k)
    blur.pipe.enable_marks(4)
    ks = [blur.submit(reps) for _ in range(4)]
    for k in ks:
        blur.pipe.wait_image(k)
        assert blur.pipe.ready(k)
        assert np.array_equal(blur.outputs[k].reshape(h, w, 3), pconv_mod.numpy_convolve(imgs[k], reps)), k
    marks = blur.pipe.marks()
    assert [int(m[0]) for m in marks] == ks and [int(m[2]) for m in marks] == [0 if lazy else 1, 0, 0, 0]
    assert all(b[1] >= a[1] > 0 for a, b in zip(marks, marks[1:])), marks


def test_xcd_swizzle_off_and_model_table(pconv_mod, native, rng):
    """Tile order without the XCD remap gives the same bytes; the shape model
    sees the runtime's real VGPR / LDS numbers for every instantiation."""
    img = rng.integers(0, 256, size=(300, 257, 3), dtype=np.uint8)
    ref = pconv_mod.numpy_convolve(img, 9)
    try:
        native.set_xcd_swizzle(False)
        out_off = pconv_mod.convolve(img, 9, backend="hip", fuse=8)
    finally:
        native.set_xcd_swizzle(True)
    out_on = pconv_mod.convolve(img, 9, backend="hip", fuse=8)
    assert np.array_equal(out_off, ref) and np.array_equal(out_on, ref)
    table = native.swar_model_table(8, "rgb", 2520, 5760)
    assert len(table) == len(native.swar_shapes())
    for lw, m, nw, vgpr, lds, measured, cycles in table:
        assert measured and 0 < vgpr <= 512 and lds >= 16384 and cycles > 0


def test_filter_pipeline_hip(pconv_mod, rng):
    """A gaussian/box/edge/custom pipeline on the GPU equals the NumPy chain."""
    img = rng.integers(0, 256, size=(64, 77, 3), dtype=np.uint8)
    p = pconv_mod.FilterPipeline.from_spec("gaussian:9,box:2,edge:1,gaussian:3")
    assert np.array_equal(p.apply(img, backend="hip"), p.reference(img))
    import torch

    t = torch.from_numpy(img).cuda()
    assert np.array_equal(p.apply(t).cpu().numpy(), p.reference(img))


@pytest.mark.gpu
def test_device_pci_id_and_numa_bind(pconv_mod):
    """PCI address of the device and the per-rank NUMA binding used by the
    multi-GPU launchers (kept CPUs are local to the GPU and a subset of the
    previously allowed ones)."""
    import os
    import re

    from pconv.parallel.bootstrap import bind_to_device_numa, device_local_cpus

    bdf = pconv_mod.native.device_pci_bus_id(0)
    assert re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]", bdf), bdf
    before = os.sched_getaffinity(0)
    try:
        kept = bind_to_device_numa(0)
        after = os.sched_getaffinity(0)
        assert after <= before
        if kept is not None:
            assert kept == len(after) and after <= (device_local_cpus(0) or set())
    finally:
        os.sched_setaffinity(0, before)


def test_step_graph_cache_bounded_across_host_buffers(pconv_mod, rng):
    """Whole-step graphs are keyed on the host buffers: cycling more distinct
    pinned (in, out) pairs than the cache holds evicts and re-captures, every
    result stays exact, and the repetition-loop graph cache is untouched."""
    n = pconv_mod.native
    w, h, reps = 45, 23, 9
    eng = n.BandEngine(w, h, "rgb", "gaussian", 0, 1, 0, halo=8, fuse=8, graph=True)
    cap = eng.max_cached_graphs
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    ref = pconv_mod.numpy_convolve(img, reps)
    # one loop graph first (run() with graph=True), it must survive the step-graph evictions
    eng.upload(img.reshape(-1), 0, h)
    eng.run(reps)
    eng.synchronize()
    loop_graphs = eng.cached_graphs - eng.cached_step_graphs
    assert loop_graphs == 1
    bufs = [(n.PinnedBuffer(img.size), n.PinnedBuffer(img.size)) for _ in range(cap + 6)]
    for k, (bi, bo) in enumerate(bufs):
        np.asarray(bi)[:] = img.reshape(-1)
        eng.process_graph(bi.ptr, 0, h, bo.ptr, reps)
        eng.synchronize()
        assert eng.cached_step_graphs <= cap
        assert np.array_equal(np.asarray(bo).reshape(h, w, 3), ref), k
    assert eng.cached_graphs - eng.cached_step_graphs == loop_graphs


@pytest.mark.parametrize("direct", [True, False])
@pytest.mark.parametrize("slots,reps,world,rank", [(1, 9, 1, 0), (2, 9, 1, 0), (3, 13, 1, 0), (2, 12, 8, 3),
                                                   (3, 7, 3, 1)])
def test_pipeline_streamed_rings(pconv_mod, rng, direct, slots, reps, world, rank):
    """Row-streamed images (stream_chunks=4): three rings of images over the
    same slot inputs with no host synchronisation in between.  A slot reused
    before its previous image's last download finished would have its result
    frame overwritten by the next image's first chunk (the raw input or a
    partial level would come back), so every output must equal the oracle of
    its slot's input."""
    from pconv.parallel.dist_engine import DistributedBlur

    w, h = 83, 120
    blur = DistributedBlur(w, h, "rgb", "gaussian", reps, rank=rank, world=world, device=0, slots=slots,
                           preload_halo=True, transport="none", stream_chunks=4, stream_min_bytes=0,
                           step_graphs=False if direct else None)  # every image / the head image streamed
    b = blur.band
    imgs = [rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for _ in range(slots)]
    for k, img in enumerate(imgs):
        blur.load_image(img, slot=k)
    for _ in range(3 * slots):
        blur.submit(reps)
    blur.drain()
    for k, img in enumerate(imgs):
        ref = pconv_mod.numpy_convolve(img, reps).reshape(h, -1)[b.y0:b.y0 + b.rows]
        assert np.array_equal(blur.outputs[k], ref), k


def test_copy_pair_floor(native):
    """The pipeline's PCIe floor (bench.py copy_floor.pair_ms): pitched H2D +
    D2H issued together; positive, and a pair is no faster than either copy
    alone could be at the link's one-way peak (64 GB/s for PCIe Gen5 x16)."""
    rb, rows = 5760, 2520
    ms = native.copy_pair_floor_ms(0, rb, rows, rows, 4)
    assert 0 < ms < 100
    assert ms >= rb * rows / 64e9 * 1e3
    with pytest.raises(Exception):
        native.copy_pair_floor_ms(0, rb, 0, rows, 4)


def test_copy_probe(native):
    """CopyProbe (bench.py's solo and concurrent floors): set up once, then
    timed runs of H2D alone, D2H alone and both together, ms per copy —
    each at most the link's one-way peak, a pair no faster than its slower
    copy could be; an empty run refused."""
    rb, rows = 5760, 630
    p = native.CopyProbe(0, rb, rows, rows)
    floor = rb * rows / 64e9 * 1e3
    h2d, d2h, pair = p.run(8, True, False), p.run(8, False, True), p.run(8)
    assert all(floor <= ms < 50 for ms in (h2d, d2h, pair))
    assert pair >= 0.9 * max(h2d, d2h)
    with pytest.raises(Exception):
        p.run(0)
    with pytest.raises(Exception):
        p.run(4, False, False)


@pytest.mark.parametrize("typ,filt,reps", [("rgb", "gaussian", 40), ("grey", "edge", 9)])
def test_cli_auto_backend_gpu_path(pconv_mod, tmp_path, typ, filt, reps):
    """`--backend auto` on a job priced above the GPU's start-up (forced with
    --auto-gpu-min 0): the GPU path runs on its own, all repetitions on the
    GPU, bit-exact with the oracle."""
    w, h = 320, 200
    r = subprocess.run([CONV_BIN, "s.raw", str(w), str(h), str(reps), typ, "--synthetic", "3", "--backend", "auto",
                        "--filter", filt, "--json", "--check", "--quiet", "--auto-gpu-min", "0"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    assert meta["gpus"] == 1 and meta["cpu_reps"] == 0 and meta["gpu_reps"] == reps and meta["mismatches"] == 0
    assert meta["auto_choice"].startswith("gpu (") and not meta["kernel"].startswith("cpu")
    out = pconv_mod.read_raw(str(tmp_path / "blur_s.raw"), w, h, typ)
    assert np.array_equal(out, pconv_mod.numpy_convolve(pconv_mod.synthetic_image(w, h, typ, seed=3), reps, filt))
