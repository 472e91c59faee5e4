"""bench.py's self-verification on the CPU (every BENCH line
must carry an oracle check).  The check is on by default; each rank's oracle
is the CPU stencil of its band's dependency cone, which must equal the rows
of the whole-image oracle for every split, and the mismatch count is what
lands in the JSON line's "mismatches" field."""
import importlib.util
import os
import sys
import types

import numpy as np
import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _args(bench, argv):
    old = sys.argv
    try:
        sys.argv = ["bench.py"] + argv
        return bench.parse()
    finally:
        sys.argv = old


def test_check_is_on_by_default(bench):
    assert _args(bench, []).check is True
    assert _args(bench, ["--check"]).check is True
    assert _args(bench, ["--no-check"]).check is False


@pytest.mark.parametrize("w,h,ch,reps,filt", [(37, 50, "rgb", 9, "gaussian"), (64, 41, "grey", 40, "gaussian"),
                                              (23, 60, "rgb", 7, "box")])
def test_cone_oracle_equals_whole_image_rows(bench, pconv_mod, w, h, ch, reps, filt):
    n = pconv_mod.native
    img = pconv_mod.synthetic_image(w, h, ch, seed=5)
    whole = pconv_mod.numpy_convolve(img, reps, filt).reshape(h, -1)
    for world in (1, 2, 3, 5, 8):
        for rank in range(world):
            band = n.row_band(h, world, rank)
            a = types.SimpleNamespace(width=w, height=h, channels=ch, reps=reps, filter=filt, seed=5)
            ref = bench.oracle_rows(a, band)
            assert np.array_equal(ref, whole[band.y0:band.y0 + band.rows]), (world, rank)
            # the JSON field: bytes that differ from the oracle (single process: no reduction)
            assert bench.mismatching_bytes(ref.copy(), ref) == 0
            bad = ref.copy()
            bad[0, :3] ^= 1
            assert bench.mismatching_bytes(bad, ref) == 3
