"""Wave plan (schedule.hpp: plan_wave) on the CPU: ONE persistent launch per
image, whose workgroups take load / level-tile / store tasks in ticket order
and wait on per-tile counters.

These tests replay the exact task lists the GPU kernel runs with a model of
the kernel's concurrency: G workers claim tickets in order, and at every step
a RANDOM claimed task whose dependency counters are complete runs (the GPU
may finish them in any order).  Checked on every run:

* no deadlock: some claimed task is always runnable (the ticket order is
  topological), for any number of workers;
* every read sees the right level: a level-j tile reads only rows of frame
  (j-1) % 2 tagged j-1 (rows outside the image excepted), a store reads
  final rows;
* no write-after-read hazard: when a level-j tile overwrites level j-2 rows,
  every level-(j-1) tile that reads them has completed;
* values: the replay (junk in every frame row not yet written, column-group
  tasks of one tile each writing the whole tile) equals the oracle.
"""
import numpy as np
import pytest

from pconv.ops.reference import numpy_convolve

from test_stream_plan import _plan, _step_rows


def _wave(native, plan, in_lo, in_hi, rows, tile_rows, groups, lp, sp, gap=1):
    L = len(plan)
    return native.plan_wave(plan, in_lo, in_hi, rows, tile_rows, [0] + [groups] * L, lp, sp, 2, gap)


def _replay(native, wp, band, height, row_bytes, ch, img_rows, in_lo, in_hi, workers, rng, roles=False,
            dynamic=False):
    """roles=False: one queue in ticket order; roles=True: the GPU kernel's
    form — loads, level tiles and stores each in its own queue (in ticket
    order), with at least one worker per queue; dynamic=True (with roles): a
    level tile is claimed only once its dependencies are complete, from
    per-level queues in tile order, deepest level first (the kernel's
    default)."""
    L = wp.levels
    off = 64 - in_lo
    n = in_hi - in_lo + 128
    frames = [rng.integers(0, 256, size=(n, row_bytes)).astype(np.int32) for _ in range(2)]
    tags = [np.full(n, -99), np.full(n, -99)]
    g0 = band.y0
    out = np.full((band.rows, row_bytes), -1, np.int32)
    counters = [[0] * wp.tiles[j] for j in range(L + 1)]
    tasks = wp.tasks

    def ready(t):
        if t.kind == 0:
            return True
        d = t.dep_level
        return all(counters[d][x] == wp.arrivals[d] for x in range(t.dep_lo, t.dep_hi + 1))

    def in_img(r):
        return 0 <= g0 + r < height

    def tile_rows_of(j, x):
        a = wp.lo[j] + x * wp.tile_rows
        return a, min(a + wp.tile_rows, wp.hi[j])

    def run(t):
        if t.kind == 0:
            frames[0][t.a + off:t.b + off] = img_rows[g0 + t.a:g0 + t.b]
            tags[0][t.a + off:t.b + off] = 0
        elif t.kind == 1:
            j, s = t.level, wp.steps[t.level]
            src, dst = (j - 1) % 2, j % 2
            r = np.arange(t.a - s, t.b + s)
            inimg = (g0 + r >= 0) & (g0 + r < height)
            assert np.all(tags[src][r[inimg] + off] == j - 1), (j, t.a, t.b, tags[src][r[inimg] + off])
            if j >= 2:
                # WAR: level-(j-1) tiles reading rows [a, b) of frame dst (level j-2) are complete
                sp = wp.steps[j - 1]
                for x in range(wp.tiles[j - 1]):
                    a2, b2 = tile_rows_of(j - 1, x)
                    if a2 - sp < t.b and b2 + sp > t.a:
                        assert counters[j - 1][x] == wp.arrivals[j - 1], (j, t.a, t.b, x)
            blk = frames[src][r + off].copy()
            blk[~inimg] = 0
            for _ in range(s):
                blk = _step_rows(blk, ch, inimg)
            rr = np.arange(t.a, t.b)
            ok = (g0 + rr >= 0) & (g0 + rr < height)
            frames[dst][rr[ok] + off] = blk[s:s + (t.b - t.a)][ok]
            tags[dst][rr[ok] + off] = j
        else:
            assert np.all(tags[L % 2][np.arange(t.a, t.b) + off] == L)
            out[t.a:t.b] = frames[L % 2][t.a + off:t.b + off]
        if t.kind != 2:
            counters[t.level][t.tile] += 1

    if dynamic:
        loads = [t for t in tasks if t.kind == 0]
        stores = [t for t in tasks if t.kind == 2]
        levels = [[t for t in tasks if t.kind == 1 and t.level == j] for j in range(L + 1)]
        head = [0] * (L + 1)
        li = si = 0
        pending_l, pending_s = [], []
        while li < len(loads) or si < len(stores) or pending_l or pending_s or any(
                head[j] < len(levels[j]) for j in range(1, L + 1)):
            while len(pending_l) < 1 + workers // 8 and li < len(loads):
                pending_l.append(loads[li])
                li += 1
            while len(pending_s) < 1 + workers // 8 and si < len(stores):
                pending_s.append(stores[si])
                si += 1
            ready_levels = [j for j in range(L, 0, -1) if head[j] < len(levels[j]) and ready(levels[j][head[j]])]
            choices = [("l", i) for i, t in enumerate(pending_l)] + \
                      [("s", i) for i, t in enumerate(pending_s) if ready(t)] + \
                      [("c", j) for j in ready_levels]
            assert choices, "stalled: no load, ready store or ready level tile"
            kind, i = choices[int(rng.integers(0, len(choices)))]
            if kind == "l":
                run(pending_l.pop(i))
            elif kind == "s":
                run(pending_s.pop(i))
            else:
                run(levels[i][head[i]])
                head[i] += 1
        return out
    if roles:
        queues = [[t for t in tasks if t.kind == k] for k in (0, 1, 2)]
        caps = [1 + workers // 8, max(1, workers), 1 + workers // 8]
    else:
        queues, caps = [list(tasks)], [workers]
    nxt = [0] * len(queues)
    claimed = [[] for _ in queues]
    while any(nxt[q] < len(queues[q]) or claimed[q] for q in range(len(queues))):
        for q in range(len(queues)):
            while len(claimed[q]) < caps[q] and nxt[q] < len(queues[q]):
                claimed[q].append(queues[q][nxt[q]])
                nxt[q] += 1
        ok = [(q, i) for q in range(len(queues)) for i, t in enumerate(claimed[q]) if ready(t)]
        assert ok, "deadlock: every claimed task waits"
        q, i = ok[int(rng.integers(0, len(ok)))]
        run(claimed[q].pop(i))
    return out


@pytest.mark.parametrize("height,world,reps,fuse", [
    (200, 1, 40, 8), (97, 1, 9, 4), (61, 1, 5, 8), (300, 1, 41, 8), (2520, 1, 40, 8), (400, 4, 40, 8),
    (395, 8, 40, 8), (1000, 3, 30, 6), (64, 1, 16, 16),
])
@pytest.mark.parametrize("tile_rows", [1, 7, 48])
def test_wave_plan_order_and_counts(native, height, world, reps, fuse, tile_rows):
    for rank in range(world):
        band, plan, in_lo, in_hi, _ = _plan(native, height, world, rank, reps, fuse, world > 1)
        for groups, lp, sp in ((1, 1, 1), (3, 2, 2), (14, 2, 3)):
            wp = _wave(native, plan, in_lo, in_hi, band.rows, tile_rows, groups, lp, sp)
            assert wp.levels == len(plan)
            kinds = [t.kind for t in wp.tasks]
            L = wp.levels
            assert kinds.count(0) == wp.tiles[0] * lp
            assert kinds.count(1) == sum(wp.tiles[j] for j in range(1, L + 1)) * groups
            stored = sorted(r for t in wp.tasks if t.kind == 2 for r in range(t.a, t.b))
            assert stored == list(range(band.rows))  # every owned row stored exactly once


@pytest.mark.parametrize("ch", [1, 3])
@pytest.mark.parametrize("height,world,reps,fuse,tile_rows,workers", [
    (90, 1, 12, 4, 8, 3), (57, 1, 7, 8, 5, 64), (130, 1, 21, 8, 16, 7), (160, 4, 12, 4, 6, 5),
    (75, 2, 10, 8, 9, 2), (40, 1, 16, 8, 3, 1), (120, 1, 24, 8, 48, 20),
])
def test_wave_plan_values(native, rng, ch, height, world, reps, fuse, tile_rows, workers):
    width = 17
    img = rng.integers(0, 256, size=(height, width, ch), dtype=np.uint8) if ch > 1 else \
        rng.integers(0, 256, size=(height, width), dtype=np.uint8)
    ref = numpy_convolve(img, reps).reshape(height, -1)
    rows = img.reshape(height, -1).astype(np.int32)
    for rank in range(world):
        band, plan, in_lo, in_hi, _ = _plan(native, height, world, rank, reps, fuse, world > 1)
        for gap, roles, dyn in ((1, False, False), (1, True, False), (4, True, False), (1, True, True)):
            wp = _wave(native, plan, in_lo, in_hi, band.rows, tile_rows, 2, 2, 2, gap)
            for _ in range(2):
                got = _replay(native, wp, band, height, width * ch, ch, rows, in_lo, in_hi, workers, rng, roles, dyn)
                assert np.array_equal(got, ref[band.y0:band.y0 + band.rows]), (rank, gap, roles, dyn)


def test_wave_plan_rejects_exchanges(native):
    band = native.row_band(100, 2, 0)
    plan = native.plan_band(band, 20, 8, 8, True, False)
    with pytest.raises(Exception):
        native.plan_wave(plan, 0, band.rows, band.rows, 8, [1, 1, 1, 1], 1, 1)
