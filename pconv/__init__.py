"""Importable name (`pconv`) for the package directory
``parallel-image-convolution-using-mpi-openmp-and-cuda_amd/``.

A hyphenated directory cannot be named in an ``import`` statement, so this
stub points the package's ``__path__`` at it and runs its ``__init__`` in this
namespace: ``import pconv`` / ``from pconv.ops import convolve`` load the real
modules (and the in-tree native extension) from that directory, exactly once.
"""
import os as _os

_PKG_DIR = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "parallel-image-convolution-using-mpi-openmp-and-cuda_amd",
)
__path__ = [_PKG_DIR]
_init = _os.path.join(_PKG_DIR, "__init__.py")
with open(_init, encoding="utf-8") as _f:
    exec(compile(_f.read(), _init, "exec"))  # noqa: S102 - trusted in-repo source
