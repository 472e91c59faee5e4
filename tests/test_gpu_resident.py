"""Register-resident fused gaussian (kernels/stencil_resident.hip): all
repetitions of a single-band frame in ONE launch, tiles exchanging halo rings
through memory between K-step phases.  Bit-exact against the CPU oracle, over
geometries that exercise edge strips, the strip-pair wrap partner, partial
last phases, several launches in a row (flag epochs) and the fallback for
frames too large for one workgroup per CU."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CH = {"grey": 1, "rgb": 3, "rgba": 4}


def _oracle(n, img, w, h, ch, reps):
    from pconv.models.filters import get_filter

    ref = np.empty_like(img.reshape(-1))
    n.cpu_convolve(np.ascontiguousarray(img.reshape(-1)), ref, w, h, ch, reps, get_filter("gaussian").to_native(),
                   True, 0)
    return ref.reshape(h, -1)


def _run(n, e, img, w, h, reps):
    e.upload(img.reshape(-1), 0, h)
    e.synchronize()
    e.run(reps)
    e.synchronize()
    out = np.empty((h, w * img.shape[-1] if img.ndim == 3 else w), np.uint8)
    e.download(out.reshape(-1), 0, h)
    e.synchronize()
    return out


@pytest.mark.parametrize("w,h,ch,reps", [
    (1920, 2520, "rgb", 40),   # the headline frame: one workgroup per CU
    (1920, 630, "grey", 10),
    (1920, 1260, "grey", 100),
    (640, 480, "rgba", 23),    # partial last phase (23 = 2 x 8 + 7)
    (333, 212, "rgb", 7),      # a single phase, no exchange
    (100, 50, "grey", 3),
    (1000, 37, "rgb", 17),     # one tile row
])
def test_resident_matches_oracle(pconv_mod, w, h, ch, reps):
    n = pconv_mod.native
    e = n.BandEngine(w, h, ch, "gaussian", 0, 1, 0, halo=8, fuse=8, variant="temporal", resident=True)
    img = pconv_mod.synthetic_image(w, h, ch, seed=11 + reps)
    ref = _oracle(n, img, w, h, ch, reps)
    for k in range(3):  # consecutive launches reuse the flags with higher epochs
        out = _run(n, e, img, w, h, reps)
        assert e.stats.launches == 1, "resident path not taken"
        bad = np.count_nonzero(out != ref)
        assert bad == 0, (k, bad)


def test_resident_falls_back_for_large_frames(pconv_mod):
    """More tiles than CUs: the tile kernel runs instead (still exact)."""
    n = pconv_mod.native
    w, h, ch, reps = 4096, 2048, "rgb", 9
    e = n.BandEngine(w, h, ch, "gaussian", 0, 1, 0, halo=8, fuse=8, variant="temporal", resident=True)
    img = pconv_mod.synthetic_image(w, h, ch, seed=5)
    out = _run(n, e, img, w, h, reps)
    assert e.stats.launches == 2
    assert np.array_equal(out, _oracle(n, img, w, h, ch, reps))


def test_resident_matches_tile_kernel_bytes(pconv_mod):
    """Same frame through both paths of one geometry, byte for byte."""
    n = pconv_mod.native
    w, h, ch, reps = 1920, 2520, "rgb", 40
    img = pconv_mod.synthetic_image(w, h, ch, seed=3)
    a = _run(n, n.BandEngine(w, h, ch, "gaussian", 0, 1, 0, halo=8, fuse=8, variant="temporal", resident=True),
             img, w, h, reps)
    b = _run(n, n.BandEngine(w, h, ch, "gaussian", 0, 1, 0, halo=8, fuse=8, variant="temporal"), img, w, h, reps)
    assert np.array_equal(a, b)


def test_resident_wait_timeout_aborts_cleanly(pconv_mod, monkeypatch):
    """A wait that times out sets the error word, every workgroup exits (no
    hang) and synchronize() raises; the next launch on the same engine (new
    flag epoch) is exact again."""
    n = pconv_mod.native
    w, h, ch, reps = 1920, 2520, "rgb", 40
    img = pconv_mod.synthetic_image(w, h, ch, seed=4)
    ref = _oracle(n, img, w, h, ch, reps)
    e = n.BandEngine(w, h, ch, "gaussian", 0, 1, 0, halo=8, fuse=8, variant="temporal", resident=True)
    e.upload(img.reshape(-1), 0, h)
    e.synchronize()
    monkeypatch.setenv("PCONV_RESIDENT_TIMEOUT_S", "1e-8")  # one clock tick: a wait that is not met at once
    e.run(reps)
    with pytest.raises(RuntimeError, match="timed out"):
        e.synchronize()
    monkeypatch.delenv("PCONV_RESIDENT_TIMEOUT_S")
    assert np.array_equal(_run(n, e, img, w, h, reps), ref)
