"""Test configuration.

Markers
  gpu  — needs a real MI355X (run with `-m gpu` on the GPU box).  Everything
         else runs on CPU (`-m "not gpu"`), including multi-process gloo tests.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
PKG = os.path.join(ROOT, "parallel-image-convolution-using-mpi-openmp-and-cuda_amd")
CONV_BIN = os.path.join(PKG, "bin", "conv")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def pconv_mod():
    import pconv

    assert pconv.native_available(), "native extension not built (run __graft_entry__.build())"
    # a native crash prints its C++ frames before faulthandler's; pytest
    # captures fd 2, so the report also goes to a file
    os.environ.setdefault("PCONV_CRASH_LOG", os.path.join(ROOT, "gpurun_out", f"native_crash_{os.getpid()}.log")
                          if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else "/tmp/pconv_native_crash.log")
    pconv.native.install_crash_handler()
    return pconv


@pytest.fixture(scope="session")
def native(pconv_mod):
    return pconv_mod.native


@pytest.fixture
def rng():
    import numpy as np

    return np.random.default_rng(12345)
