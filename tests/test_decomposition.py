"""Row-band partitioner, the reference grid chooser, the halo/launch planner,
and bit-exactness of the decomposed schedule on CPU (single process)."""
import numpy as np
import pytest


def test_row_bands_cover_image(native):
    for h in (1, 2, 7, 8, 9, 100, 2520, 4097):
        for n in range(1, 9):
            if h < n:
                with pytest.raises(Exception):
                    native.row_band(h, n, 0)
                continue
            bands = native.row_bands(h, n)
            assert bands[0].y0 == 0 and bands[0].up == -1 and bands[-1].down == -1
            assert sum(b.rows for b in bands) == h
            for i, b in enumerate(bands):
                assert b.rank == i and b.world == n and b.rows in (h // n, h // n + 1)
                if i:
                    assert b.y0 == bands[i - 1].y0 + bands[i - 1].rows and b.up == i - 1
                if i + 1 < n:
                    assert b.down == i + 1


def test_reference_rows_division(native):
    # Grids quoted in BASELINE.md for a 1920x2520 image: n=1,2,4,9,16,25 ->
    # 1x1, 2x1, 2x2, 3x3, 4x4, 5x5 (rows_to x cols_to).
    for n, rows_to in [(1, 1), (2, 2), (4, 2), (9, 3), (16, 4), (25, 5)]:
        assert native.reference_rows_division(n, 2520, 1920) == rows_to
    # 1920x5040, n=16 -> 8x2 (BASELINE.md "MPI 1920x5040 ... 8x2 grid")
    assert native.reference_rows_division(16, 5040, 1920) == 8
    # impossible split -> 0 ("Cannot divide to processes")
    assert native.reference_rows_division(7, 10, 10) == 0


def _simulate(plan, rows, up, down, reps, halo_preloaded, depth):
    """Track which frame rows hold values of which rep, verify every launch
    reads only up-to-date rows and that owned rows end at `reps`."""
    lo_f, hi_f = -depth, rows + depth
    INVALID = -10 ** 9
    cur = {r: (0 if (0 <= r < rows or halo_preloaded) else INVALID) for r in range(lo_f, hi_f)}
    # rows beyond a global edge are permanent zeros: valid at every rep
    EDGE = None
    for r in range(lo_f, hi_f):
        if (r < 0 and up < 0) or (r >= rows and down < 0):
            cur[r] = EDGE
    done = 0
    for ph in plan:
        if ph.exchange_depth:
            d = ph.exchange_depth
            for r in range(-d, 0):
                if up >= 0:
                    cur[r] = done
            for r in range(rows, rows + d):
                if down >= 0:
                    cur[r] = done
        nxt = dict(cur)
        for l in ph.launches:
            assert l.steps == ph.steps
            for r in range(l.lo - l.steps, l.hi + l.steps):
                v = cur[r]
                assert v is EDGE or v == done, (r, v, done, l.lo, l.hi)
            for r in range(l.lo, l.hi):
                nxt[r] = done + l.steps
        cur = nxt
        done += ph.steps
    assert done == reps
    for r in range(rows):
        assert cur[r] == reps


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("halo,fuse", [(1, 1), (4, 1), (4, 4), (8, 3), (16, 8)])
@pytest.mark.parametrize("preloaded", [False, True])
def test_plan_is_dependency_safe(native, world, halo, fuse, preloaded):
    h = 64
    for rank in range(world):
        b = native.row_band(h, world, rank)
        d, t = native.normalize_plan(halo, fuse, h // world if world > 1 else 0)
        for reps in (0, 1, 2, 7, 16, 33):
            for overlap in (False, True):
                plan = native.plan_band(b, reps, d, t, overlap, preloaded and world > 1)
                _simulate(plan, b.rows, b.up, b.down, reps, preloaded and world > 1, d)
                if overlap and world > 1:
                    for ph in plan:
                        if ph.exchange_depth and len(ph.launches) > 1:
                            assert not ph.launches[0].after_halo


def test_plan_exchange_count(native):
    b = native.row_band(2520, 8, 3)
    plan = native.plan_band(b, 40, 40, 8, True, False)
    assert sum(1 for p in plan if p.exchange_depth) == 1
    plan = native.plan_band(b, 40, 8, 8, True, False)
    assert sum(1 for p in plan if p.exchange_depth) == 5
    plan = native.plan_band(b, 40, 40, 8, True, True)
    assert sum(1 for p in plan if p.exchange_depth) == 0
    assert "exchange" in native.describe_plan(native.plan_band(b, 4, 4, 2, True, False))


@pytest.mark.parametrize("channels", ["grey", "rgb"])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("halo,fuse,preload", [(1, 1, False), (3, 1, True), (4, 2, False), (6, 3, True), (5, 5, False)])
def test_local_cpu_cluster_bit_exact(pconv_mod, rng, channels, world, halo, fuse, preload):
    from pconv.parallel.cpu_dist import local_cpu_cluster_convolve

    h, w = 37, 21
    shape = (h, w) if channels == "grey" else (h, w, 3)
    img = rng.integers(0, 256, size=shape, dtype=np.uint8)
    for reps in (1, 4, 9):
        ref = pconv_mod.numpy_convolve(img, reps)
        got = local_cpu_cluster_convolve(img, reps, world, halo=halo, fuse=fuse, preload_halo=preload)
        assert np.array_equal(got, ref), (world, halo, fuse, reps)


def test_local_cpu_cluster_float_filter(pconv_mod, rng):
    from pconv.parallel.cpu_dist import local_cpu_cluster_convolve

    img = rng.integers(0, 256, size=(30, 11, 3), dtype=np.uint8)
    for f in ("box", "edge"):
        ref = pconv_mod.numpy_convolve(img, 6, f)
        got = local_cpu_cluster_convolve(img, 6, 4, f, halo=4, fuse=2)
        assert np.array_equal(got, ref)


def test_cpu_fused_launch_matches_repeated_steps(native, rng):
    """cpu_fused_launch == `steps` full-image steps restricted to [lo, hi)."""
    from pconv.ops.reference import numpy_convolve

    h, w, halo = 20, 9, 4
    lay = native.frame_layout(w, h, halo)
    img = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    src = np.zeros(lay["bytes"], np.uint8)
    v = src.reshape(h + 2 * halo, lay["pitch"])
    v[halo : halo + h, 16 : 16 + w] = img
    for steps in (1, 2, 4):
        dst = np.zeros_like(src)
        native.cpu_fused_launch("gaussian", "grey", w, h, halo, src, dst, 3, 15, steps, 0, h)
        ref = numpy_convolve(img, steps)
        got = dst.reshape(h + 2 * halo, lay["pitch"])[halo + 3 : halo + 15, 16 : 16 + w]
        assert np.array_equal(got, ref[3:15])


def test_auto_fuse_policy(native, pconv_mod):
    """Repetitions per launch: 12 for grey frames far beyond the Infinity
    Cache (measured faster there), 8 for every other fusable frame, 1 for
    filters the fused kernel does not implement."""
    from pconv.models.filters import get_filter

    g = get_filter("gaussian").to_native()
    assert native.auto_fuse(g, "auto", 32768 * 32768, 1) == 12
    assert native.auto_fuse(g, "auto", 16384 * 16384, 1) == 12
    assert native.auto_fuse(g, "auto", 8192 * 8192 * 3, 3) == 8
    assert native.auto_fuse(g, "auto", 1920 * 2520 * 3, 3) == 8
    assert native.auto_fuse(g, "auto", 1920 * 2520, 1) == 8
    assert native.auto_fuse(g, "auto", 32768 * 4096, 1) == 8  # 8-way band of 32768^2
    assert native.auto_fuse(g, "auto", 32768 * 32768) == 8  # channels unknown
    # float filters: the temporal float32 kernel (8 grey, 4 RGB); one step with an explicit one-step kernel
    assert native.auto_fuse(get_filter("box").to_native(), "auto", 32768 * 32768, 1) == 8
    assert native.auto_fuse(get_filter("edge").to_native(), "auto", 1920 * 2520 * 3, 3) == 4
    assert native.auto_fuse(get_filter("box").to_native(), "float9", 1920 * 2520 * 3, 3) == 1


def _ext_model(owned, y0, height, plan, halo, reps):
    """Independent model of a self-neighbour band: the extended array of
    ghost + owned rows is stepped as a whole (zero outside it and outside the
    global image); each exchange re-reflects the band's own rows into the
    ghost zone.  Owned rows must match the frame-level oracle whenever the
    plan is dependency safe."""
    from pconv.ops.reference import numpy_convolve

    rows = owned.shape[0]
    ext = np.zeros((rows + 2 * halo,) + owned.shape[1:], np.uint8)
    ext[halo:halo + rows] = owned
    g = np.arange(-halo, rows + halo) + y0
    outside = (g < 0) | (g >= height)
    done = 0
    for ph in plan:
        d = ph.exchange_depth
        if d:
            ext[halo - d:halo] = ext[halo:halo + d]
            ext[halo + rows:halo + rows + d] = ext[halo + rows - d:halo + rows]
            ext[:halo - d] = 0  # stale beyond the exchanged depth: never read
            ext[halo + rows + d:] = 0
        for _ in range(ph.steps):
            ext[outside] = 0
            ext = numpy_convolve(ext, 1)
        done += ph.steps
    assert done == reps
    return ext[halo:halo + rows]


@pytest.mark.parametrize("reps,halo,fuse,overlap", [(13, 4, 4, True), (20, 8, 8, False), (5, 1, 1, True),
                                                    (17, 6, 3, True), (40, 40, 8, True), (24, 12, 8, False)])
@pytest.mark.parametrize("y0", [0, 9, 37])
def test_reflected_ghost_oracle_cpu(native, rng, reps, halo, fuse, overlap, y0):
    """The oracle of the GPU mid-image RCCL self-band tests
    (tests/test_gpu_halo.py) agrees with an independent model."""
    from halo_oracle import reflected_ghost_oracle

    rows, w, height = 48, 29, y0 + 48 + 45
    b = native.Band()
    b.rank, b.world, b.y0, b.rows, b.up, b.down = 0, 1, y0, rows, 0, 0
    d, t = native.normalize_plan(halo, fuse, 0)
    plan = native.plan_band(b, reps, d, t, overlap, False)
    owned = rng.integers(0, 256, size=(rows, w), dtype=np.uint8)
    got = reflected_ghost_oracle(native, plan, d, owned, y0, height, "grey")
    assert np.array_equal(got, _ext_model(owned, y0, height, plan, d, reps))


def test_cpu_rank_slices_are_disjoint():
    """MPI+OpenMP analog: the node's CPU budget split between its ranks
    (opt-in binding, parallel/bootstrap.py)."""
    from pconv.parallel.bootstrap import cpu_rank_slice

    allowed = set(range(0, 64, 2)) | {100, 101}
    for world in (1, 2, 3, 4, 9):
        slices = [cpu_rank_slice(r, world, allowed, 15) for r in range(world)]
        assert all(len(s) == max(1, 15 // world) for s in slices)
        flat = [c for s in slices for c in s]
        assert len(flat) == len(set(flat)) and set(flat) <= set(sorted(allowed)[:15])
    # more ranks than budget CPUs: round-robin sharing, never empty
    assert all(len(cpu_rank_slice(r, 20, allowed, 4)) == 1 for r in range(20))
