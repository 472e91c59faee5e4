"""Wave images on the GPU: a whole serving step (H2D, every repetition, D2H)
as ONE persistent launch (EngineOptions::stream_chunks = -1,
kernels/stencil_wave.hip; the task lists themselves are checked on the CPU
in tests/test_wave_plan.py).

An image submitted to an idle step-graph pipeline runs as a wave launch, the
images behind it as step graphs; every result is compared with the oracle
(NumPy for small frames, the native OpenMP oracle for large ones) and output
buffers are pre-filled with junk so a row never stored shows up.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CH = {"grey": 1, "rgb": 3, "rgba": 4}


def _blur(w, h, ch, reps, slots=1, **kw):
    from pconv.parallel.dist_engine import DistributedBlur

    b = DistributedBlur(w, h, ch, "gaussian", reps, device=0, slots=slots, stream_chunks=-1, **kw)
    assert b.pipe.graphs and b.pipe.step_graphs
    return b


def _oracle(pconv_mod, img, reps):
    h, w = img.shape[:2]
    ch = "grey" if img.ndim == 2 else {3: "rgb", 4: "rgba"}[img.shape[2]]
    if img.size <= 200_000:
        return pconv_mod.numpy_convolve(img, reps).reshape(h, -1)
    ref = np.empty_like(img)
    pconv_mod.native.cpu_convolve(img.reshape(-1), ref.reshape(-1), w, h, ch, reps, "gaussian", True, 0)
    return ref.reshape(h, -1)


def _image(rng, w, h, ch):
    c = CH[ch]
    return rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)


@pytest.mark.parametrize("w,h,ch,reps", [
    (68, 45, "rgb", 9), (64, 133, "grey", 40), (52, 71, "rgba", 13), (36, 37, "grey", 41), (256, 300, "grey", 1),
    (100, 9, "rgb", 17), (1920, 252, "rgb", 40), (1920, 2520, "rgb", 40), (4096, 1024, "grey", 200),
])
def test_wave_image_bit_exact(pconv_mod, rng, w, h, ch, reps):
    blur = _blur(w, h, ch, reps)
    assert blur.engine.wave_able(reps, 0, h)
    for _ in range(3):
        img = _image(rng, w, h, ch)
        blur.load_image(img)
        blur.outputs[0][:] = 0xAB
        got = blur.step(reps).reshape(h, -1)
        assert np.array_equal(got, _oracle(pconv_mod, img, reps))
    assert blur.engine.wave_tasks(reps, 0, h) > 0
    assert blur.stats.launches == 1  # the whole step was one launch


@pytest.mark.parametrize("slots", [2, 3])
def test_wave_head_then_graphs(pconv_mod, rng, slots):
    """A burst: the first image (idle pipeline) is a wave launch on its slot's
    stream, the others step graphs on theirs; then another burst."""
    w, h, ch, reps = 120, 200, "rgb", 24
    blur = _blur(w, h, ch, reps, slots=slots)
    for _ in range(2):
        imgs = [_image(rng, w, h, ch) for _ in range(slots)]
        ks = []
        for img in imgs:
            k = blur._next
            blur.load_image(img, slot=k)
            blur.outputs[k][:] = 0xAB
            ks.append(blur.submit(reps))
        blur.drain()
        for img, k in zip(imgs, ks):
            assert np.array_equal(blur.outputs[k].reshape(h, -1), _oracle(pconv_mod, img, reps)), k


@pytest.mark.parametrize("world,rank", [(2, 0), (3, 1), (4, 3), (8, 5)])
def test_wave_preloaded_bands(pconv_mod, rng, world, rank):
    """A rank's band with pre-loaded ghost rows (the N>1 headline) as a wave:
    the ghost rows are loaded with the band, every level shrinks into them."""
    w, h, reps = 64, 400, 40
    blur = _blur(w, h, "rgb", reps, rank=rank, world=world, preload_halo=True, transport="none")
    a, b = blur.input_rows
    assert blur.engine.wave_able(reps, -blur.above, blur.band.rows + blur.below)
    img = _image(rng, w, h, "rgb")
    blur.load_image(img)
    blur.outputs[0][:] = 0xAB
    got = blur.step(reps)
    ref = _oracle(pconv_mod, img, reps)
    assert np.array_equal(got.reshape(blur.band.rows, -1), ref[blur.band.y0:blur.band.y0 + blur.band.rows])


def test_wave_small_grid(pconv_mod, rng, monkeypatch):
    """Few workgroups for many tasks (PCONV_WAVE_GRID): every workgroup walks
    long runs of tickets; still bit-exact and no wait times out."""
    monkeypatch.setenv("PCONV_WAVE_GRID", "3")
    w, h, ch, reps = 200, 300, "rgb", 40
    blur = _blur(w, h, ch, reps)
    img = _image(rng, w, h, ch)
    blur.load_image(img)
    assert np.array_equal(blur.step(reps).reshape(h, -1), _oracle(pconv_mod, img, reps))


def test_wave_timeout_raises_and_recovers(pconv_mod, rng, monkeypatch):
    """A dependency wait that gives up (a 1-microsecond limit: the first level
    tile cannot find its rows loaded in time) aborts the launch — every
    workgroup drains — and the host raises; a fresh engine then runs fine."""
    monkeypatch.setenv("PCONV_WAVE_TIMEOUT_S", "0.000001")
    w, h, ch, reps = 1920, 600, "rgb", 40
    blur = _blur(w, h, ch, reps)
    blur.load_image(_image(rng, w, h, ch))
    with pytest.raises(Exception, match="timed out"):
        blur.step(reps)
    monkeypatch.delenv("PCONV_WAVE_TIMEOUT_S")
    blur2 = _blur(w, h, ch, reps)
    img = _image(rng, w, h, ch)
    blur2.load_image(img)
    assert np.array_equal(blur2.step(reps).reshape(h, -1), _oracle(pconv_mod, img, reps))
