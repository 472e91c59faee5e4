"""Loader for the in-tree native extension ``_pconv_native``.

``import torch`` comes first on purpose: torch ships its own
``libamdhip64.so.7`` / ``librccl.so.1``; loading them first makes the
extension (linked against the same sonames) bind to the copies torch already
mapped instead of pulling a second HIP runtime into the process.

The extension is REQUIRED: there is no silent Python fallback for the GPU
path.  If it is missing, build it with ``python -c "import __graft_entry__ as g;
g.build()"`` (or ``make -C <pkg>/csrc``).
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  -- see module docstring

# OpenMP workers of the CPU stencil sleep between parallel regions instead of
# spinning: CPU ranks of the MPI+OpenMP analog share a node's CPU quota, and
# spinning workers of one rank burn the quota the others' compute needs (a
# throttled cgroup stalls every rank for the rest of its 100 ms period: the
# round-2 hybrid table had 0.1-0.2 s outliers and got slower with more ranks;
# profiles/r03/hybrid/).  libgomp reads OMP_WAIT_POLICY once, when it is
# initialised, so the variable is set only around the extension's import and
# the caller's environment is restored right after: child processes and
# OpenMP runtimes initialised later keep the user's setting.  It takes effect
# only when the extension's import is what initialises the system libgomp
# (a libgomp already mapped by an earlier import keeps its own policy).  An
# explicit OMP_WAIT_POLICY or GOMP_SPINCOUNT wins.
_SET_POLICY = "OMP_WAIT_POLICY" not in os.environ and "GOMP_SPINCOUNT" not in os.environ
if _SET_POLICY:
    os.environ["OMP_WAIT_POLICY"] = "passive"

_ERR = None
try:
    native = importlib.import_module(__package__ + "._pconv_native")
except ImportError as e:  # pragma: no cover - exercised only on broken builds
    native = None
    _ERR = e
finally:
    if _SET_POLICY:
        os.environ.pop("OMP_WAIT_POLICY", None)


def native_available() -> bool:
    return native is not None


def require_native():
    """Return the extension module or raise a loud, actionable error."""
    if native is None:
        here = os.path.dirname(os.path.abspath(__file__))
        raise ImportError(
            f"pconv native extension not built (looked in {here}): run "
            f"`make -C {os.path.join(here, 'csrc')}` or __graft_entry__.build(). "
            f"Original error: {_ERR}"
        )
    return native


def conv_binary() -> str:
    """Path of the in-tree `conv` CLI binary (built with the extension)."""
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bin", "conv")
    if not os.path.exists(p):
        raise FileNotFoundError(f"conv binary not built: {p} (run __graft_entry__.build())")
    return p
