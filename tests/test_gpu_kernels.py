"""HIP kernel numerics on a real MI355X: every variant vs the fp32-semantics
oracles, odd sizes, partial row ranges, guard-band canaries (catches the
out-of-bounds class of bug the reference's RGB kernel had)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GUARD = 4096
CANARY = 0xA5
CH = {"grey": 1, "rgb": 3, "rgba": 4}


def _frame(native, torch, row_bytes, rows, halo):
    lay = native.frame_layout(row_bytes, rows, halo)
    buf = torch.full((lay["bytes"] + 2 * GUARD,), CANARY, dtype=torch.uint8, device="cuda")
    buf[GUARD : GUARD + lay["bytes"]] = 0
    return lay, buf


def _rows(buf, lay, halo, rows):
    v = buf[GUARD : GUARD + lay["bytes"]].view(rows + 2 * halo, lay["pitch"])
    return v


def _run_kernel(native, img, filt, variant, steps=1, r0=None, r1=None, halo=None):
    import torch

    h = img.shape[0]
    row_bytes = img.size // h
    halo = halo if halo is not None else max(1, steps)
    lay, src = _frame(native, torch, row_bytes, h, halo)
    _, dst = _frame(native, torch, row_bytes, h, halo)
    sv = _rows(src, lay, halo, h)
    sv[halo : halo + h, 16 : 16 + row_bytes] = torch.from_numpy(img.reshape(h, row_bytes)).cuda()
    base = lay["pitch"] * halo + 16
    r0 = 0 if r0 is None else r0
    r1 = h if r1 is None else r1
    native.launch_stencil(filt, {1: "grey", 3: "rgb", 4: "rgba"}[img.size // (h * img.shape[1])],
                          src.data_ptr() + GUARD + base, dst.data_ptr() + GUARD + base, lay["pitch"], row_bytes,
                          r0, r1, -halo, h + halo, steps, 0, h, torch.cuda.current_stream().cuda_stream, variant)
    torch.cuda.synchronize()
    d = dst.cpu().numpy()
    assert (d[:GUARD] == CANARY).all() and (d[-GUARD:] == CANARY).all(), "write outside the frame"
    dv = d[GUARD:-GUARD].reshape(h + 2 * halo, lay["pitch"])
    assert (dv[:, :16] == 0).all() and (dv[:, 16 + row_bytes :] == 0).all(), "write into the pad columns"
    outside = np.ones(h + 2 * halo, bool)
    outside[halo + r0 : halo + r1] = False
    assert (dv[outside] == 0).all(), "write outside the requested rows"
    return dv[halo : halo + h, 16 : 16 + row_bytes].reshape(img.shape)


SIZES = [(1, 1), (1, 5), (5, 1), (3, 3), (2, 16), (17, 16), (9, 33), (31, 100), (64, 65), (130, 257)]


@pytest.mark.parametrize("channels", ["grey", "rgb", "rgba"])
@pytest.mark.parametrize("filt,variant", [("gaussian", "auto"), ("gaussian", "binomial"), ("gaussian", "int9"),
                                          ("gaussian", "float9"), ("box", "auto"), ("edge", "auto")])
def test_single_step_matches_oracle(native, rng, channels, filt, variant):
    from pconv.ops.reference import numpy_convolve

    c = CH[channels]
    for (h, w) in SIZES:
        img = rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)
        got = _run_kernel(native, img, filt, variant)
        assert np.array_equal(got, numpy_convolve(img, 1, filt)), (h, w)


def test_extreme_values(native):
    from pconv.ops.reference import numpy_convolve

    for val in (0, 1, 15, 16, 128, 254, 255):
        img = np.full((19, 23, 3), val, np.uint8)
        for f in ("gaussian", "box", "edge"):
            assert np.array_equal(_run_kernel(native, img, f, "auto"), numpy_convolve(img, 1, f))


def test_partial_rows(native, rng):
    from pconv.ops.reference import numpy_convolve

    img = rng.integers(0, 256, size=(40, 37, 3), dtype=np.uint8)
    ref = numpy_convolve(img, 1)
    for r0, r1 in [(0, 1), (5, 6), (3, 29), (39, 40), (0, 40), (13, 14)]:
        got = _run_kernel(native, img, "gaussian", "auto", r0=r0, r1=r1)
        assert np.array_equal(got[r0:r1], ref[r0:r1])
        assert (got[:r0] == 0).all() and (got[r1:] == 0).all()


def test_shape_guard_rejects_out_of_frame(native):
    import torch

    lay, src = _frame(native, torch, 64, 8, 1)
    _, dst = _frame(native, torch, 64, 8, 1)
    base = lay["pitch"] + 16
    with pytest.raises(RuntimeError, match="exceed frame"):
        native.launch_stencil("gaussian", "grey", src.data_ptr() + GUARD + base, dst.data_ptr() + GUARD + base,
                              lay["pitch"], 64, -1, 8, -1, 9, 1, 100, 1 << 40, 0, "auto")


def _run_fused(native, img, steps, r0, r1, halo, g_row0, height, variant="auto", filt="gaussian"):
    """Run one fused launch on a band frame whose row 0 is global row g_row0;
    returns (gpu_rows, cpu_rows) of the whole frame's data columns."""
    import torch

    h = img.shape[0]  # frame owned rows
    row_bytes = img.size // h
    ch = {1: "grey", 3: "rgb", 4: "rgba"}[img.size // (h * img.shape[1])]
    lay, src = _frame(native, torch, row_bytes, h, halo)
    _, dst = _frame(native, torch, row_bytes, h, halo)
    full = np.zeros((h + 2 * halo, lay["pitch"]), np.uint8)
    # fill ghost + owned rows that lie inside the image with random data
    rng = np.random.default_rng(steps * 1000 + r0)
    for fr in range(-halo, h + halo):
        if 0 <= g_row0 + fr < height:
            full[halo + fr, 16 : 16 + row_bytes] = rng.integers(0, 256, row_bytes, dtype=np.uint8)
    src[GUARD : GUARD + lay["bytes"]] = torch.from_numpy(full.reshape(-1)).cuda()
    base = lay["pitch"] * halo + 16
    native.launch_stencil(filt, ch, src.data_ptr() + GUARD + base, dst.data_ptr() + GUARD + base,
                          lay["pitch"], row_bytes, r0, r1, -halo, h + halo, steps, g_row0, height,
                          torch.cuda.current_stream().cuda_stream, variant)
    torch.cuda.synchronize()
    d = dst.cpu().numpy()
    assert (d[:GUARD] == CANARY).all() and (d[-GUARD:] == CANARY).all(), "write outside the frame"
    gpu = d[GUARD:-GUARD].reshape(h + 2 * halo, lay["pitch"])
    cpu = np.zeros(lay["bytes"], np.uint8)
    native.cpu_fused_launch(filt, ch, row_bytes, h, halo, full.reshape(-1), cpu, r0, r1, steps, g_row0, height)
    return gpu, cpu.reshape(h + 2 * halo, lay["pitch"])


@pytest.mark.parametrize("channels", ["grey", "rgb", "rgba"])
@pytest.mark.parametrize("steps", [1, 2, 3, 4, 5, 8, 11, 16])
def test_temporal_matches_fused_reference(native, rng, channels, steps, variant="temporal"):
    c = CH[channels]
    for (h, w) in [(1, 3), (7, 5), (40, 33), (97, 130), (150, 700), (33, 1500)]:
        img = rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)
        gpu, cpu = _run_fused(native, img, steps, 0, h, steps, 0, h, variant=variant)
        assert np.array_equal(gpu, cpu), (h, w, steps)


def _custom_filter(native):
    # asymmetric, non-uniform, one negative tap: exercises the tap order and the clamp at 0
    return native.Filter.custom([3, 1, 0, 2, 5, 1, -1, 2, 4], 17, "custom")


FLOAT_FILTERS = ["box", "edge", "custom"]


@pytest.mark.parametrize("filt", FLOAT_FILTERS)
@pytest.mark.parametrize("channels", ["grey", "rgb", "rgba"])
@pytest.mark.parametrize("steps", [1, 2, 3, 4, 5, 8, 11, 16])
def test_float_temporal_matches_fused_reference(native, rng, filt, channels, steps):
    """Any 3x3 filter in the reference's float32 semantics (mul then add, row-
    major tap order, truncation every step), `steps` per launch: byte for byte
    the CPU twin of a fused launch (mpi/mpi_convolution.c:90-100,303-307),
    guard-band canaries and pad columns untouched (checked by _run_fused)."""
    f = _custom_filter(native) if filt == "custom" else filt
    c = CH[channels]
    for (h, w) in [(1, 3), (7, 5), (40, 33), (97, 130), (150, 700), (33, 1500)]:
        img = rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)
        gpu, cpu = _run_fused(native, img, steps, 0, h, steps, 0, h, variant="float_temporal", filt=f)
        assert np.array_equal(gpu, cpu), (filt, h, w, steps)


@pytest.mark.parametrize("filt", FLOAT_FILTERS)
@pytest.mark.parametrize("steps", [2, 4, 8, 16])
def test_float_temporal_band_regions(native, filt, steps):
    f = _custom_filter(native) if filt == "custom" else filt
    _band_regions(native, steps, "float_temporal", f)


def test_float_temporal_equals_repeated_single_steps(pconv_mod, rng):
    """A fused float launch of T steps == T reference single steps (NumPy float32 oracle)."""
    img = rng.integers(0, 256, size=(123, 211, 3), dtype=np.uint8)
    for f in ("box", "edge"):
        for t in (2, 5, 13):
            got = _run_kernel(pconv_mod.native, img, f, "float_temporal", steps=t)
            assert np.array_equal(got, pconv_mod.numpy_convolve(img, t, f)), (f, t)


@pytest.mark.parametrize("steps", [2, 4, 8, 16])
def test_temporal_band_regions(native, rng, steps):
    _band_regions(native, steps, "temporal")


def _band_regions(native, steps, variant, filt="gaussian"):
    """Bands in the middle / at the edges of a taller image, regions reaching
    into ghost rows (what the distributed schedule asks for)."""
    H = 300
    h = 60
    img = np.zeros((h, 45, 3), np.uint8)
    halo = 16
    for g_row0 in (0, 100, H - h):
        for (r0, r1) in [(0, h), (-(halo - steps), h + (halo - steps)), (steps, h - steps), (-3, 5), (h - 2, h + 1)]:
            if r0 - steps < -halo or r1 + steps > h + halo or r0 >= r1:
                continue
            gpu, cpu = _run_fused(native, img, steps, r0, r1, halo, g_row0, H, variant=variant, filt=filt)
            fr0, fr1 = halo + r0, halo + r1
            assert np.array_equal(gpu[fr0:fr1], cpu[fr0:fr1]), (variant, g_row0, r0, r1, steps)
            # nothing written outside [r0, r1)
            assert (gpu[:fr0] == 0).all() and (gpu[fr1:] == 0).all()


def test_temporal_equals_repeated_single_steps(pconv_mod, rng):
    """A fused launch of T steps == T single-step launches (whole image)."""
    img = rng.integers(0, 256, size=(123, 211, 3), dtype=np.uint8)
    for t in (2, 6, 13):
        got = _run_kernel(pconv_mod.native, img, "gaussian", "temporal", steps=t)
        assert np.array_equal(got, pconv_mod.numpy_convolve(img, t)), t


@pytest.mark.parametrize("form", [0, 1])
def test_every_swar_shape_bit_exact(native, rng, form):
    """Force each instantiated SWAR tile shape (lane width, rows/wave, waves)
    in each step form (0: truncate every step, 1: pairs of steps with a x16
    intermediate) and compare a fused launch with the CPU fused reference: odd and even step
    counts, a band whose ghost rows reach the image top."""
    try:
        native.set_swar_alt(form)
        for (lw, m, nw) in native.swar_shapes():
            native.set_swar_shape(lw, m, nw)
            for channels, steps in (("grey", 3), ("rgb", 4), ("rgba", 2), ("rgb", 8), ("grey", 7), ("rgb", 1)):
                if m * nw <= 2 * steps or lw < CH[channels]:
                    continue
                c = CH[channels]
                img = rng.integers(0, 256, size=(71, 301, c) if c > 1 else (71, 301), dtype=np.uint8)
                gpu, cpu = _run_fused(native, img, steps, 0, 71, steps, 0, 71, variant="temporal")
                assert np.array_equal(gpu, cpu), (lw, m, nw, channels, steps)
                gpu, cpu = _run_fused(native, img[:40], steps, -5, 45, 16, 30, 200, variant="temporal")
                assert np.array_equal(gpu[11:61], cpu[11:61]), (lw, m, nw, channels, steps, "band")
    finally:
        native.set_swar_shape(0, 0, 0)
        native.set_swar_alt(-1)


@pytest.mark.parametrize("swizzle", [True, False])
@pytest.mark.parametrize("form", [0, 1])
def test_prefetch_kernel_every_shape_bit_exact(native, rng, form, swizzle):
    """The buffer-op tile kernel (k_swar_pf), forced in each shape and step
    form, with and without the XCD-aware tile order: whole images and band
    regions with ghost rows and image edges, guard-band canaries, untouched
    rows outside [r0, r1)."""
    try:
        native.set_swar_alt(form)
        native.set_xcd_swizzle(swizzle)
        native.set_prefetch_mode(1)
        for (lw, m, nw) in native.swar_prefetch_shapes():
            native.set_swar_shape(lw, m, nw)
            for channels, steps in (("grey", 3), ("rgb", 4), ("rgba", 2), ("rgb", 8), ("grey", 8), ("rgb", 1)):
                if m * nw <= 2 * steps:
                    continue
                c = CH[channels]
                w = 300 if c == 1 else 100  # row bytes multiple of 4 (the kernel's contract)
                img = rng.integers(0, 256, size=(131, w, c) if c > 1 else (131, w), dtype=np.uint8)
                gpu, cpu = _run_fused(native, img, steps, 0, 131, steps, 0, 131, variant="temporal")
                assert np.array_equal(gpu, cpu), (lw, m, nw, channels, steps)
                gpu, cpu = _run_fused(native, img[:40], steps, -5, 45, 16, 30, 200, variant="temporal")
                assert np.array_equal(gpu[11:61], cpu[11:61]), (lw, m, nw, channels, steps, "band")
    finally:
        native.set_prefetch_mode(-1)
        native.set_xcd_swizzle(True)
        native.set_swar_shape(0, 0, 0)
        native.set_swar_alt(-1)
        native.clear_swar_tuning()


def test_prefetch_kernel_tuned_large_frame(native, rng):
    """Tuned (default) choice on a frame with many tiles (thousands of
    workgroups), with the buffer-op kernel among the candidates, against the
    CPU fused reference; and the buffer-op kernel forced in a tall shape."""
    import torch

    h, w = 1536, 4096
    img = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    try:
        native.clear_swar_tuning()
        gpu, cpu = _run_fused(native, img, 8, 0, h, 8, 0, h, variant="temporal")
        assert np.array_equal(gpu, cpu)
        native.set_prefetch_mode(1)
        native.set_swar_shape(4, 16, 8)
        gpu, cpu = _run_fused(native, img, 8, 0, h, 8, 0, h, variant="temporal")
        assert np.array_equal(gpu, cpu)
    finally:
        native.set_prefetch_mode(-1)
        native.set_swar_shape(0, 0, 0)
        native.clear_swar_tuning()
        torch.cuda.synchronize()


def test_frame_beyond_2gib_offsets(pconv_mod, native):
    """64-bit offsets end to end: a 2.16 GB grey frame
    (65536 x 33000) through the fused kernel; rows near the top, the middle
    and the bottom are checked against the NumPy oracle on sub-windows (a row
    after `reps` repetitions depends only on the `reps` rows around it)."""
    import numpy as np

    w, h, reps = 65536, 33000, 3
    img = np.empty((h, w), np.uint8)
    native.synth_rows(img.reshape(-1), w, h, "grey", 11, 0, h)
    out = pconv_mod.convolve(img, reps, backend="hip", fuse=3)
    assert out.shape == img.shape
    for y0 in (0, h // 2 - 4, h - 8):
        lo, hi = max(0, y0 - reps), min(h, y0 + 8 + reps)
        # oracle on the window; rows [lo, hi) with zero padding is exact only
        # where the window edge is the image edge or >= reps rows away
        ref = pconv_mod.numpy_convolve(img[lo:hi, :2048], reps)
        got = out[y0:y0 + 8, :2048 - reps]
        exp = ref[y0 - lo:y0 - lo + 8, :2048 - reps]
        assert np.array_equal(got, exp), y0
