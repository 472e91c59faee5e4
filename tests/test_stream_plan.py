"""Row streaming within one image (schedule.hpp: plan_streamed) on the CPU.

The GPU engine uploads an image in row chunks and advances every level of
the plan as far as the rows on the device allow, with only two frames and
three streams (uploads run ahead, downloads trail behind).  These tests
replay the exact plans the engine issues:

* level tags: every launch reads only rows that hold the previous level, no
  launch writes a frame row that a later chunk's upload fills or that an
  earlier chunk's download still reads, and every owned row is downloaded
  exactly once at the final level;
* values: a NumPy replay of the plan (fused launches on two frames with junk
  in every row not yet written) equals the whole-image oracle, with uploads
  issued all up front or just in time and downloads right after their chunk
  or at the very end (the two extremes of the stream timing).
"""
import numpy as np
import pytest

from pconv.ops.reference import numpy_convolve

JUNK = -7


def _plan(native, height, world, rank, reps, fuse, preload):
    band = native.row_band(height, world, rank)
    depth, fuse = native.normalize_plan(reps if preload else fuse, fuse, height // world if world > 1 else 0)
    plan = native.plan_band(band, reps, depth, fuse, False, preload)
    if preload:
        in_lo = -min(depth, band.y0)
        in_hi = band.rows + min(depth, height - (band.y0 + band.rows))
    else:
        in_lo, in_hi = 0, band.rows
    return band, plan, in_lo, in_hi, depth


def _check_tags(sp, band, height, in_lo, in_hi):
    """Level bookkeeping of one streamed image (see module docstring)."""
    L = sp.levels
    g0 = band.y0

    def in_img(r):
        return 0 <= g0 + r < height

    lo_f, hi_f = in_lo - 64, in_hi + 64
    tag = [dict.fromkeys(range(lo_f, hi_f), JUNK), dict.fromkeys(range(lo_f, hi_f), JUNK)]
    chunks = sp.chunks
    # rows written (per frame) by each chunk's launches
    writes = []
    for ch in chunks:
        w = (set(), set())
        for l, lev in zip(ch.launches, ch.levels):
            for r in range(l.lo, l.hi):
                if in_img(r):
                    w[lev % 2].add(r)
        writes.append(w)
    downloaded = []
    for c, ch in enumerate(chunks):
        assert ch.up_hi > ch.up_lo
        for r in range(ch.up_lo, ch.up_hi):
            tag[0][r] = 0
        # uploads of LATER chunks may land at any time: no launch of this or an
        # earlier chunk writes their frame-0 rows
        for later in chunks[c + 1:]:
            assert not any(ch_w for ch_w in (set(range(later.up_lo, later.up_hi)) & writes[c][0])), \
                f"chunk {c} writes frame-0 rows that a later upload fills"
        for l, lev in zip(ch.launches, ch.levels):
            assert l.lo < l.hi
            src, dst = (lev - 1) % 2, lev % 2
            for r in range(l.lo - l.steps, l.hi + l.steps):
                if in_img(r):
                    assert tag[src][r] == lev - 1, f"level {lev} launch [{l.lo},{l.hi}) reads row {r} tagged " \
                                                   f"{tag[src][r]} (chunk {c})"
            for r in range(l.lo, l.hi):
                if in_img(r):
                    tag[dst][r] = lev
        if ch.down_hi > ch.down_lo:
            for r in range(ch.down_lo, ch.down_hi):
                assert tag[L % 2][r] == L, f"chunk {c} downloads row {r} at level {tag[L % 2][r]}"
                # a download may run late: no later chunk's launch rewrites its rows
                for later in writes[c + 1:]:
                    assert r not in later[L % 2], f"row {r} downloaded after chunk {c} is rewritten later"
            downloaded.extend(range(ch.down_lo, ch.down_hi))
    assert downloaded == list(range(band.rows)), "every owned row downloaded exactly once, in order"


def _step_rows(blk, ch, inimg):
    """One zero-padded gaussian step on a block of byte rows (int arithmetic,
    == the reference float32 result); rows outside the image forced to 0."""
    p = np.pad(blk.astype(np.int32), ((1, 1), (ch, ch)))
    h = p[:, :-2 * ch] + 2 * p[:, ch:-ch] + p[:, 2 * ch:]
    v = h[:-2] + 2 * h[1:-1] + h[2:]
    out = (v >> 4).astype(np.int32)
    out[~inimg] = 0
    return out


def _replay_values(sp, band, height, row_bytes, ch, img_rows, in_lo, in_hi, uploads_first, downloads_last, rng):
    off = 64 - in_lo  # frame row r lives at array row r + off
    n = in_hi - in_lo + 128
    frames = [rng.integers(0, 256, size=(n, row_bytes)).astype(np.int32) for _ in range(2)]
    g0 = band.y0
    out = np.full((band.rows, row_bytes), -1, np.int32)
    L = sp.levels

    def upload(c):
        u = sp.chunks[c]
        frames[0][u.up_lo + off:u.up_hi + off] = img_rows[g0 + u.up_lo:g0 + u.up_hi]

    def download(c):
        d = sp.chunks[c]
        out[d.down_lo:d.down_hi] = frames[L % 2][d.down_lo + off:d.down_hi + off]

    if uploads_first:
        for c in range(len(sp.chunks)):
            upload(c)
    for c, chunk in enumerate(sp.chunks):
        if not uploads_first:
            upload(c)
        for l, lev in zip(chunk.launches, chunk.levels):
            src, dst = frames[(lev - 1) % 2], frames[lev % 2]
            rows = np.arange(l.lo - l.steps, l.hi + l.steps)
            inimg = (g0 + rows >= 0) & (g0 + rows < height)
            blk = src[rows + off].copy()
            blk[~inimg] = 0
            for _ in range(l.steps):
                blk = _step_rows(blk, ch, inimg)
            keep = slice(l.steps, l.steps + (l.hi - l.lo))
            rr = np.arange(l.lo, l.hi)
            ok = (g0 + rr >= 0) & (g0 + rr < height)
            dst[rr[ok] + off] = blk[keep][ok]
        if not downloads_last:
            download(c)
    if downloads_last:
        for c in range(len(sp.chunks)):
            download(c)
    return out


@pytest.mark.parametrize("height,world,reps,fuse", [
    (200, 1, 40, 8), (97, 1, 9, 4), (61, 1, 5, 8), (300, 1, 41, 8), (120, 1, 1, 8), (64, 1, 16, 16),
    (2520, 1, 40, 8), (400, 4, 40, 8), (395, 8, 40, 8), (1000, 3, 30, 6),
])
def test_stream_plan_tags(native, height, world, reps, fuse):
    for rank in range(world):
        preload = world > 1
        band, plan, in_lo, in_hi, _ = _plan(native, height, world, rank, reps, fuse, preload)
        assert native.streamable(plan)
        for chunks in range(2, 13):
            cuts = native.stream_cuts(in_lo, in_hi, chunks)
            sp = native.plan_streamed(plan, in_lo, in_hi, band.rows, cuts)
            assert sp.levels == len(plan)
            _check_tags(sp, band, height, in_lo, in_hi)


def test_stream_plan_random_cuts(native, rng):
    """Arbitrary chunk boundaries (many tiny chunks, chunks thinner than the
    steps, a single-row chunk) keep every invariant."""
    for trial in range(120):
        height = int(rng.integers(8, 300))
        world = int(rng.integers(1, 5))
        if height < world * 2:
            continue
        rank = int(rng.integers(0, world))
        reps = int(rng.integers(1, 30))
        fuse = int(rng.integers(1, 17))
        preload = world > 1 and reps <= height // world
        if world > 1 and not preload:
            continue
        band, plan, in_lo, in_hi, _ = _plan(native, height, world, rank, reps, fuse, preload)
        n = in_hi - in_lo
        k = int(rng.integers(0, min(n - 1, 40) + 1))
        cuts = sorted(set(int(x) for x in rng.integers(in_lo + 1, in_hi, size=k))) if n > 1 else []
        sp = native.plan_streamed(plan, in_lo, in_hi, band.rows, cuts)
        _check_tags(sp, band, height, in_lo, in_hi)


@pytest.mark.parametrize("ch", [1, 3])
@pytest.mark.parametrize("height,world,reps,fuse,chunks", [
    (90, 1, 12, 4, 5), (57, 1, 7, 8, 3), (130, 1, 21, 8, 7), (160, 4, 12, 4, 4), (75, 2, 10, 8, 6),
])
def test_stream_plan_values(native, rng, ch, height, world, reps, fuse, chunks):
    width = 23
    img = rng.integers(0, 256, size=(height, width, ch), dtype=np.uint8) if ch > 1 else \
        rng.integers(0, 256, size=(height, width), dtype=np.uint8)
    ref = numpy_convolve(img, reps).reshape(height, -1)
    rows = img.reshape(height, -1).astype(np.int32)
    for rank in range(world):
        band, plan, in_lo, in_hi, _ = _plan(native, height, world, rank, reps, fuse, world > 1)
        sp = native.plan_streamed(plan, in_lo, in_hi, band.rows, native.stream_cuts(in_lo, in_hi, chunks))
        for uf in (True, False):
            for dl in (True, False):
                got = _replay_values(sp, band, height, width * ch, ch, rows, in_lo, in_hi, uf, dl, rng)
                assert np.array_equal(got, ref[band.y0:band.y0 + band.rows]), (rank, uf, dl)


def test_stream_cuts_shape(native):
    assert native.stream_cuts(0, 2520, 1) == []
    assert native.stream_cuts(0, 110, 2) == [50]  # 5, 6
    c = native.stream_cuts(0, 2520, 4)  # weights 5,5,5,6 / 21
    assert c == [600, 1200, 1800]
    c = native.stream_cuts(-40, 355, 4)
    assert all(-40 < x < 355 for x in c) and c == sorted(set(c))
    assert native.stream_cuts(0, 3, 10) == [1, 2] or len(native.stream_cuts(0, 3, 10)) <= 2


def test_stream_cuts_weighted(native):
    # the default weights through the weighted form
    assert native.stream_cuts_weighted(0, 2520, [5, 5, 5, 5, 5, 6]) == native.stream_cuts(0, 2520, 6)
    assert native.stream_cuts_weighted(0, 2520, [1, 2, 2, 2, 2, 1]) == [252, 756, 1260, 1764, 2268]
    assert native.stream_cuts_weighted(0, 2520, [3, 4, 4, 5, 5]) == [360, 840, 1320, 1920]
    assert native.stream_cuts_weighted(-40, 2560, [1]) == []
    # more chunks than rows: empty chunks merged, cuts strictly inside
    c = native.stream_cuts_weighted(0, 3, [1, 1, 1, 1, 1, 1])
    assert c == sorted(set(c)) and all(0 < x < 3 for x in c)
    with pytest.raises(Exception):
        native.stream_cuts_weighted(0, 100, [1, 0, 1])


def test_plan_streamed_rejects_exchanges(native):
    band = native.row_band(100, 2, 0)
    plan = native.plan_band(band, 20, 8, 8, True, False)  # needs exchanges
    assert not native.streamable(plan)
    with pytest.raises(Exception):
        native.plan_streamed(plan, 0, band.rows, band.rows, [10])
