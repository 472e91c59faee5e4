"""Property-based tests (hypothesis) of the decomposition invariants: random
image heights, world sizes, halo depths, fusion depths and repetition counts.

  * the row-band partition tiles the image exactly, with balanced bands;
  * every band's schedule reads only up-to-date rows and ends at `reps`
    (the dependency simulator of test_decomposition);
  * the decomposed CPU schedule (N bands, halo messages between them) equals
    the serial oracle bit for bit, for the exact-integer and float filters.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from test_decomposition import _simulate

SETTINGS = dict(deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])


@settings(max_examples=200, **SETTINGS)
@given(h=st.integers(1, 5000), n=st.integers(1, 8))
def test_partition_tiles_image(native, h, n):
    if h < n:
        with pytest.raises(Exception):
            native.row_bands(h, n)
        return
    bands = native.row_bands(h, n)
    assert [b.y0 for b in bands] == sorted(b.y0 for b in bands)
    assert sum(b.rows for b in bands) == h and bands[0].y0 == 0
    assert max(b.rows for b in bands) - min(b.rows for b in bands) <= 1
    for i, b in enumerate(bands[1:], 1):
        assert b.y0 == bands[i - 1].y0 + bands[i - 1].rows


@settings(max_examples=150, **SETTINGS)
@given(h=st.integers(8, 300), world=st.integers(1, 8), halo=st.integers(1, 24), fuse=st.integers(1, 16),
       reps=st.integers(0, 60), overlap=st.booleans(), preloaded=st.booleans(), data=st.data())
def test_plan_dependency_safe(native, h, world, halo, fuse, reps, overlap, preloaded, data):
    if h < world:
        return
    rank = data.draw(st.integers(0, world - 1))
    b = native.row_band(h, world, rank)
    d, t = native.normalize_plan(halo, fuse, h // world if world > 1 else 0)
    pre = preloaded and world > 1
    plan = native.plan_band(b, reps, d, t, overlap, pre)
    _simulate(plan, b.rows, b.up, b.down, reps, pre, d)


@settings(max_examples=40, **SETTINGS)
@given(h=st.integers(1, 40), w=st.integers(1, 24), channels=st.sampled_from(["grey", "rgb"]),
       world=st.integers(1, 6), halo=st.integers(1, 6), fuse=st.integers(1, 6), reps=st.integers(0, 12),
       preload=st.booleans(), filt=st.sampled_from(["gaussian", "gaussian", "box", "edge"]), seed=st.integers(0, 99))
def test_decomposed_schedule_equals_serial(pconv_mod, h, w, channels, world, halo, fuse, reps, preload, filt, seed):
    from pconv.parallel.cpu_dist import local_cpu_cluster_convolve

    if h < world:
        return
    if filt != "gaussian":
        fuse = 1  # the float filters run one step per launch
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, size=(h, w) if channels == "grey" else (h, w, 3), dtype=np.uint8)
    ref = pconv_mod.numpy_convolve(img, reps, filt)
    got = local_cpu_cluster_convolve(img, reps, world, filt, halo=max(halo, fuse), fuse=fuse, preload_halo=preload)
    assert np.array_equal(got, ref)
