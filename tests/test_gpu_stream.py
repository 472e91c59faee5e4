"""Row streaming within one image on the GPU (EngineOptions::stream_chunks).

Each image's rows are uploaded in chunks and every level advances behind
them (schedule.hpp plan_streamed); H2D, launches and D2H of one image run on
three streams (shared H2D / compute / D2H streams, one event pair per chunk;
the pipeline's event-ordered mode), checked bit-exact against the NumPy
oracle (tests/test_stream_plan.py checks the plans themselves on the CPU).
Output buffers are pre-filled with junk so a row never downloaded shows up.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CH = {"grey": 1, "rgb": 3, "rgba": 4}


def _blur(w, h, ch, filt, reps, chunks, slots=2, mode="direct", **kw):
    """mode "direct": every image streamed on shared event-ordered streams;
    "head": step-graph pipeline that streams only images submitted while it
    is idle (the first of every burst here) and runs the others as graphs."""
    from pconv.parallel.dist_engine import DistributedBlur

    kw.setdefault("stream_min_bytes", 0)  # head-stream these small images too
    b = DistributedBlur(w, h, ch, filt, reps, device=0, slots=slots, stream_chunks=chunks,
                        step_graphs=None if mode == "head" else False, **kw)
    assert b.pipe.graphs == (mode == "head")
    return b


def _run_images(pconv_mod, rng, blur, w, h, ch, filt, reps, rounds=2):
    c = CH[ch]
    b = blur.band
    for rnd in range(rounds):
        imgs = [rng.integers(0, 256, size=(h, w, c), dtype=np.uint8) for _ in range(blur.slots)]
        ks = []
        for img in imgs:
            k = blur._next
            blur.load_image(img, slot=k)
            blur.outputs[k][:] = 0xAB
            ks.append(blur.submit(reps))
        blur.drain()
        for img, k in zip(imgs, ks):
            ref = pconv_mod.numpy_convolve(img if c > 1 else img[..., 0], reps, filt).reshape(h, -1)
            got = blur.outputs[k].reshape(b.rows, -1)
            assert np.array_equal(got, ref[b.y0:b.y0 + b.rows]), (rnd, k)


@pytest.mark.parametrize("mode", ["direct", "head"])
@pytest.mark.parametrize("slots", [1, 3])
@pytest.mark.parametrize("chunks", [2, 3, 5, 8])
@pytest.mark.parametrize("w,h,ch,reps", [(67, 45, "rgb", 9), (64, 133, "grey", 40), (50, 71, "rgba", 13),
                                         (1920, 252, "rgb", 40)])
def test_streamed_pipeline_bit_exact(pconv_mod, rng, mode, slots, chunks, w, h, ch, reps):
    blur = _blur(w, h, ch, "gaussian", reps, chunks, slots=slots, mode=mode)
    sp = blur.engine.stream_plan(reps, 0, h)
    assert len(sp.chunks) == min(chunks, h) and sp.levels == len(blur.plan(reps))
    _run_images(pconv_mod, rng, blur, w, h, ch, "gaussian", reps)
    assert blur.stats.launches >= sp.levels


@pytest.mark.parametrize("mode", ["direct", "head"])
@pytest.mark.parametrize("filt", ["box", "edge"])
def test_streamed_float_filters(pconv_mod, rng, mode, filt):
    _run_images(pconv_mod, rng, _blur(59, 83, "rgb", filt, 11, 4, mode=mode), 59, 83, "rgb", filt, 11)


@pytest.mark.parametrize("fuse", [8, 16])
def test_streamed_reps_exceed_chunks(pconv_mod, rng, fuse):
    """More repetitions than rows per chunk (the last level lags several
    chunks behind the uploads), an odd height and a last launch of 1 step."""
    blur = _blur(33, 37, "grey", "gaussian", 41, 9, fuse=fuse, halo=fuse)
    _run_images(pconv_mod, rng, blur, 33, 37, "grey", "gaussian", 41)


@pytest.mark.parametrize("mode", ["direct", "head"])
@pytest.mark.parametrize("world,rank", [(2, 0), (3, 1), (4, 3), (8, 5)])
def test_streamed_preloaded_bands(pconv_mod, rng, mode, world, rank):
    """A rank's band with pre-loaded ghost rows (the N>1 headline) streamed:
    the ghost rows travel with the first / last chunks."""
    w, h, reps = 61, 400, 40
    blur = _blur(w, h, "rgb", "gaussian", reps, 3, rank=rank, world=world, preload_halo=True, transport="none",
                 mode=mode)
    _run_images(pconv_mod, rng, blur, w, h, "rgb", "gaussian", reps)


@pytest.mark.parametrize("on_slots,alt", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("slots", [2, 3, 4])
def test_head_stream_modes(pconv_mod, rng, on_slots, alt, slots):
    """head_on_slot_streams: the streamed head image's copies on two pool
    streams, or on the next two slots' streams (falls back below 3 slots);
    head_alt_uploads (>= 4 slots): its chunk uploads alternating over two
    slots' streams; bursts and single images (blur.step) bit-exact."""
    w, h, reps = 96, 120, 40
    blur = _blur(w, h, "rgb", "gaussian", reps, 4, slots=slots, mode="head", head_on_slot_streams=on_slots,
                 head_alt_uploads=alt)
    assert blur.pipe.options["head_alt_uploads"] is alt
    _run_images(pconv_mod, rng, blur, w, h, "rgb", "gaussian", reps, rounds=3)
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    blur.load_image(img)
    for _ in range(3):
        assert np.array_equal(blur.step(reps).reshape(h, w, 3), pconv_mod.numpy_convolve(img, reps))


@pytest.mark.parametrize("weights", [[3, 4, 4, 5, 5], [1, 1, 1, 1, 1, 1, 1, 1, 1], [5, 1, 1, 5]])
@pytest.mark.parametrize("w,h,ch,filt,reps,fuse", [(96, 120, "rgb", "gaussian", 40, 8),
                                                   (33, 37, "grey", "gaussian", 41, 8),
                                                   (59, 83, "rgb", "box", 11, None)])
def test_head_stream_weights(pconv_mod, rng, weights, w, h, ch, filt, reps, fuse):
    """stream_weights: uneven streamed chunks, including chunks thinner than
    the plan's lag (chunks without launches); bursts and single images
    bit-exact."""
    kw = {} if fuse is None else dict(fuse=fuse, halo=fuse)
    blur = _blur(w, h, ch, filt, reps, 4, slots=4, mode="head", stream_weights=weights, **kw)
    assert blur.pipe.options["stream_weights"] == weights
    _run_images(pconv_mod, rng, blur, w, h, ch, filt, reps, rounds=2)
    c = CH[ch]
    img = rng.integers(0, 256, size=(h, w, c), dtype=np.uint8)
    ref = pconv_mod.numpy_convolve(img if c > 1 else img[..., 0], reps, filt).reshape(h, -1)
    blur.load_image(img)
    for _ in range(3):
        assert np.array_equal(blur.step(reps).reshape(h, -1), ref)
    assert blur.pipe.streamed_heads >= 5


@pytest.mark.parametrize("weights", [None, [2, 3, 3, 4], [1, 2, 2, 2, 2, 1]])
def test_head_stream_weights_headline_frame(pconv_mod, rng, weights):
    """The headline frame (1920x2520 RGB, 40 reps) through the chunk weights
    the latency runs use: single images and a burst of four, against the CPU
    oracle (OpenMP, bit-exact to the NumPy one)."""
    from pconv.ops.stencil import convolve

    w, h, reps = 1920, 2520, 40
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    ref = convolve(img, reps, backend="omp")
    blur = _blur(w, h, "rgb", "gaussian", reps, 4, slots=4, mode="head", stream_weights=weights,
                 stream_min_bytes=None, lazy_head=False)  # the burst's head streamed too
    blur.load_image(img)
    for _ in range(3):
        assert np.array_equal(blur.step(reps).reshape(h, w, 3), ref)
    ks = [blur.submit(reps) for _ in range(4)]
    blur.drain()
    for k in ks:
        assert np.array_equal(blur.outputs[k].reshape(h, w, 3), ref), k
    assert blur.pipe.streamed_heads == 4


@pytest.mark.parametrize("slots", [3, 4])
def test_lazy_head(pconv_mod, rng, slots):
    """lazy_head: a burst's first image is held until the next submit (then a
    step graph: no streamed head) or until drain / wait_image / ready (then
    row-streamed); bursts, single images and per-image waits bit-exact."""
    w, h, reps = 96, 120, 40
    blur = _blur(w, h, "rgb", "gaussian", reps, 4, slots=slots, mode="head", lazy_head=True)
    assert blur.pipe.options["lazy_head"] is True
    for rnd in range(3):  # bursts: every slot loaded first, then submitted back to back
        imgs = [rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8) for _ in range(slots)]
        for k, img in enumerate(imgs):
            blur.load_image(img, slot=k)
            blur.outputs[k][:] = 0xAB
        ks = [blur.submit(reps) for _ in imgs]
        blur.drain()
        for k in ks:
            assert np.array_equal(blur.outputs[k].reshape(h, w, 3), pconv_mod.numpy_convolve(imgs[k], reps)), (rnd, k)
    assert blur.pipe.streamed_heads == 0  # every burst's first image ran as a step graph
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    ref = pconv_mod.numpy_convolve(img, reps)
    blur.load_image(img)
    for i in range(3):
        assert np.array_equal(blur.step(reps).reshape(h, w, 3), ref)
        assert blur.pipe.streamed_heads == i + 1  # single images: streamed at drain
    k = blur.submit(reps)  # held
    blur.pipe.wait_image(k)  # issues it (streamed) and waits for it
    assert blur.pipe.ready(k) and blur.pipe.streamed_heads == 4
    assert np.array_equal(blur.outputs[k].reshape(h, w, 3), ref)
    blur.drain()
    ks = [blur.submit(reps) for _ in range(2 * slots)]
    blur.drain()
    for k in ks:
        assert np.array_equal(blur.outputs[k].reshape(h, w, 3), ref), k
    assert blur.pipe.streamed_heads == 4


def test_head_stream_threshold(pconv_mod, rng):
    """EngineOptions::stream_min_bytes (default 8 MiB): the headline frame
    (14.5 MB) is head-streamed, its 8-way band (2.3 MB) runs as one step
    graph unless the threshold is lowered; both bit-exact."""
    from pconv.parallel.dist_engine import DistributedBlur

    w, h, reps = 1920, 2520, 8
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    ref = pconv_mod.numpy_convolve(img, reps).reshape(h, -1)
    for world, rank, kw, streamed in ((1, 0, {}, True), (8, 3, {}, False), (8, 3, {"stream_min_bytes": 0}, True)):
        b = DistributedBlur(w, h, "rgb", "gaussian", reps, rank=rank, world=world, device=0, slots=3,
                            preload_halo=world > 1, transport="none", stream_chunks=4, **kw)
        assert b.pipe.options["stream_min_bytes"] == kw.get("stream_min_bytes", 8 << 20)
        b.load_image(img)
        out = b.step(reps)
        assert b.pipe.streamed_heads == (1 if streamed else 0), (world, kw)
        assert np.array_equal(out, ref[b.band.y0:b.band.y0 + b.band.rows]), (world, kw)


@pytest.mark.parametrize("mode", ["direct", "head"])
def test_streamed_step_and_reps_zero(pconv_mod, rng, mode):
    """blur.step (one image alone: streamed in both modes) and reps = 0
    (nothing to stream: the whole-image path) through a streaming pipeline."""
    w, h = 40, 30
    blur = _blur(w, h, "rgb", "gaussian", 7, 4, mode=mode)
    img = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    blur.load_image(img)
    assert np.array_equal(blur.step(7).reshape(h, w, 3), pconv_mod.numpy_convolve(img, 7))
    assert len(blur.engine.stream_plan(0, 0, h).chunks) == 0
    assert np.array_equal(blur.step(0).reshape(h, w, 3), img)
    assert np.array_equal(blur.step(7).reshape(h, w, 3), pconv_mod.numpy_convolve(img, 7))


@pytest.mark.parametrize("gpus,extra", [(1, []), (1, ["--stream-chunks", "4"]), (2, ["--transport", "gloo-host"])])
def test_native_bench_line(gpus, extra):
    """`bench.py --native`: the same serving step in the `conv` binary (ROCm's
    HIP runtime, no torch; fork launcher for N > 1, here two ranks sharing the
    GPU), one JSON line with the bench contract's fields, oracle-checked."""
    import json
    import os
    import subprocess
    import sys

    from conftest import ROOT

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--native", "--gpus", str(gpus), "--steps", "12",
           "--warmup", "3"] + extra
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["metric"] == "Mpixels/sec (and wall-time) for 1920x2520 RGB, 40 reps at 1/2/4/8 MI355X"
    assert d["n_gpus"] == gpus and d["steps"] == 12 and d["value"] > 0 and d["mismatches"] == 0
    assert d["runtime"]["stack"].startswith("native") and "torch" not in d["runtime"]["hip_runtime_path"]
    assert d["config"]["parallelism"] == f"rowband{gpus}" and len(d["per_rank_ms_per_step"]) == gpus
    assert d["latency_ms"] > 0 and d["copy_floor"]["pair_ms"] > 0


def test_native_bench_emulated_rank():
    """`bench.py --native --emulate 8:3`: the per-rank proxy on the native
    stack (its band + pre-loaded ghost rows), oracle-checked on its rows."""
    import json
    import os
    import subprocess
    import sys

    from conftest import ROOT

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--native", "--emulate", "8:3", "--steps", "20",
           "--warmup", "3"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["mismatches"] == 0 and "rank 3 of a 8-way split" in d["emulated"]
    assert d["config"]["halo_mode"] == "preload" and d["config"]["halo_depth"] == 40
