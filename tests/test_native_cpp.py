"""C++ unit runner (tests/cpp/test_native.cpp) for the host-side runtime,
built with AddressSanitizer + UndefinedBehaviorSanitizer and run here:
partitioner, filter exactness, CPU oracle vs a naive independent stencil,
the distributed schedule on CPU frames, raw I/O, CLI parsing, synthetic
images."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_native_unit_runner_asan_ubsan():
    csrc = os.path.join(PKG, "csrc")
    r = subprocess.run(["make", "-C", csrc, "test-native", "-j4"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "0 failures" in r.stdout
