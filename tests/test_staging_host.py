"""Host-side staging helpers behind the round-6 slow-mode fix (CPU only):
flush_host_cache (clflush of CPU-written staging rows) leaves the bytes
unchanged, page_nodes reports where a range's pages live, and bench.py's
staging_numa / window diagnostics degrade to a reported error instead of
raising when they cannot measure."""
import numpy as np


def test_flush_host_cache_keeps_bytes(pconv_mod):
    n = pconv_mod.native
    rng = np.random.default_rng(3)
    for size in (1, 63, 64, 4097, 3 << 20):
        a = rng.integers(0, 256, size=size, dtype=np.uint8)
        ref = a.copy()
        n.flush_host_cache(a.ctypes.data + (1 if size > 1 else 0), max(0, size - 1))
        assert np.array_equal(a, ref)
    n.flush_host_cache(0, 0)  # nothing to do


def test_page_nodes_counts_every_page(pconv_mod):
    import os

    n = pconv_mod.native
    page = os.sysconf("SC_PAGESIZE")
    a = np.ones(64 * page, np.uint8)  # touched: every page present
    nodes = n.page_nodes(a.ctypes.data, a.nbytes)
    assert sum(nodes.values()) in (64, 65)  # an unaligned start spans one more page
    assert all(k >= 0 for k in nodes), nodes  # present pages report their node
    assert n.page_nodes(0, 0) == {}
