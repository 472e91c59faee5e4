"""Filter semantics and the two CPU oracles (native C++ vs independent NumPy)."""
import numpy as np
import pytest

SIZES = [(1, 1), (1, 7), (7, 1), (3, 3), (5, 17), (16, 16), (13, 33), (40, 29)]


def test_filter_zoo(pconv_mod):
    from pconv.models.filters import get_filter, list_filters

    assert list_filters() == ["box", "edge", "gaussian"]
    g = get_filter("gaussian")
    assert g.int_exact and g.shift == 4 and g.divisor == 16
    assert not get_filter("box").int_exact and not get_filter("edge").int_exact
    assert get_filter("edge_detection") is get_filter("edge")
    # reference construction: (float)(tap / (double)div)
    assert get_filter("box").weights[0] == float(np.float32(1 / 9.0))
    nf = pconv_mod.native.Filter.gaussian()
    assert nf.binomial121 and nf.int_exact and nf.shift == 4
    assert not pconv_mod.native.Filter.box().int_exact


def test_gaussian_float_equals_integer_formula(rng):
    """float32 MAC of p*(w/16) in reference order, then
    truncation, equals (sum w*p) >> 4 for every 3x3 patch."""
    taps = np.array([1, 2, 1, 2, 4, 2, 1, 2, 1])
    w32 = (taps / 16.0).astype(np.float32)
    patches = rng.integers(0, 256, size=(200_000, 9), dtype=np.int64)
    patches[:64] = 255
    patches[64:128] = 0
    acc = np.zeros(len(patches), dtype=np.float32)
    for i in range(9):
        acc = (acc + (patches[:, i].astype(np.float32) * w32[i]).astype(np.float32)).astype(np.float32)
    flt = np.trunc(acc).astype(np.int64)
    ints = (patches * taps).sum(axis=1) >> 4
    assert np.array_equal(flt, ints)


def test_box_float_differs_from_naive_integer():
    """box/9 is not integer-exact: e.g. nine 1s -> float32 sum of 9*(1/9f)."""
    w = np.float32(1 / 9.0)
    acc = np.float32(0)
    for _ in range(9):
        acc = np.float32(acc + np.float32(1) * w)
    # the reference truncates whatever float32 gives; pconv must follow it.
    assert int(np.trunc(acc)) in (0, 1)


@pytest.mark.parametrize("channels", ["grey", "rgb", "rgba"])
@pytest.mark.parametrize("filt", ["gaussian", "box", "edge"])
def test_native_oracle_matches_numpy(native, rng, channels, filt):
    from pconv.ops.reference import numpy_convolve

    c = {"grey": 1, "rgb": 3, "rgba": 4}[channels]
    for (h, w) in SIZES:
        shape = (h, w) if c == 1 else (h, w, c)
        img = rng.integers(0, 256, size=shape, dtype=np.uint8)
        for reps in (0, 1, 2, 5):
            ref = numpy_convolve(img, reps, filt)
            for omp in (False, True):
                out = np.empty_like(img)
                native.cpu_convolve(img.reshape(-1), out.reshape(-1), w, h, channels, reps, filt, omp, 0)
                assert np.array_equal(out, ref), (h, w, reps, omp)


def test_custom_filter_exactness(native):
    from pconv.models.filters import get_filter

    f = get_filter(((1, 1, 1, 1, 8, 1, 1, 1, 1), 16))
    assert f.int_exact
    nf = native.Filter.custom([1, 1, 1, 1, 8, 1, 1, 1, 1], 16)
    assert nf.int_exact and not nf.binomial121
    neg = native.Filter.custom([0, -1, 0, -1, 4, -1, 0, -1, 0], 1)
    assert not neg.int_exact


def test_zero_padding_semantics(pconv_mod):
    """A single bright pixel in a corner spreads with zero padding (the MPI /
    serial semantics chosen in SURVEY §0.1, not the CUDA border quirk)."""
    img = np.zeros((4, 5), np.uint8)
    img[0, 0] = 255
    out = pconv_mod.convolve(img, 1, backend="omp")
    assert out[0, 0] == (255 * 4) >> 4
    assert out[0, 1] == (255 * 2) >> 4 and out[1, 0] == (255 * 2) >> 4
    assert out[1, 1] == 255 >> 4
    assert out[2:, :].sum() == 0 and out[:, 2:].sum() == 0


def test_convolve_backends_agree(pconv_mod, rng):
    import torch

    img = rng.integers(0, 256, size=(23, 31, 3), dtype=np.uint8)
    a = pconv_mod.convolve(img, 3, backend="numpy")
    b = pconv_mod.convolve(img, 3, backend="cpu")
    c = pconv_mod.convolve(img, 3, backend="omp")
    d = pconv_mod.convolve(torch.from_numpy(img), 3, backend="omp")
    assert np.array_equal(a, b) and np.array_equal(a, c) and np.array_equal(a, d.numpy())


def test_filter_pipeline_cpu(pconv_mod, rng):
    """Multi-stage pipelines = composition of single-filter runs (omp backend
    vs the NumPy oracle of the whole chain)."""
    img = rng.integers(0, 256, size=(29, 31, 3), dtype=np.uint8)
    p = pconv_mod.FilterPipeline.from_spec("gaussian:3, box:2, edge")
    assert p.total_reps == 6 and [s.filter.name for s in p.stages] == ["gaussian", "box", "edge"]
    assert np.array_equal(p.apply(img, backend="omp"), p.reference(img))
    q = pconv_mod.FilterPipeline([("gaussian", 2), (([1, 1, 1, 1, 8, 1, 1, 1, 1], 16), 1)])
    assert np.array_equal(q.apply(img, backend="cpu"), q.reference(img))
    with pytest.raises(ValueError):
        pconv_mod.FilterPipeline.from_spec("gaussian:-1")


def test_convolve_file_cpu(pconv_mod, tmp_path, rng):
    img = rng.integers(0, 256, size=(17, 23), dtype=np.uint8)
    src = str(tmp_path / "g.raw")
    pconv_mod.write_raw(src, img)
    dst = pconv_mod.convolve_file(src, 23, 17, 4, "grey", backend="omp")
    assert dst.endswith("blur_g.raw")
    assert np.array_equal(pconv_mod.read_raw(dst, 23, 17, "grey"), pconv_mod.numpy_convolve(img, 4))


def test_custom_int_filter_cpu_matches_oracle(pconv_mod, rng):
    """The integer row path (int-exact custom filters, not the binomial) in
    both CPU backends — each row kernel runs as its AVX2 clone where the CPU
    has AVX2 — against the NumPy float32 oracle (exact for power-of-two
    divisors)."""
    filt = ((1, 1, 1, 1, 8, 1, 1, 1, 1), 16)
    for shape in ((37, 53, 3), (29, 41), (16, 300, 4)):
        img = rng.integers(0, 256, size=shape, dtype=np.uint8)
        ref = pconv_mod.numpy_convolve(img, 3, filt)
        for be in ("cpu", "omp"):
            assert np.array_equal(pconv_mod.convolve(img, 3, filter=filt, backend=be), ref), (shape, be)
