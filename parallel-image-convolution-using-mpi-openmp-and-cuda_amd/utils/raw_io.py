"""Raw 8-bit image files (headerless, row-major, interleaved channels).

Reference I/O: MPI-IO band reads/writes (``mpi/mpi_convolution.c:126-140,
244-262``) and POSIX ``read_info``/``write_info`` (``cuda/functions.c:31-45``).
The native layer does the real work (pread/pwrite at 64-bit offsets, size
validation, ``O_TRUNC``); these helpers return NumPy arrays shaped (H, W[, C]).
"""
from __future__ import annotations

import os

import numpy as np

from .._native import require_native

_CH = {"grey": 1, "rgb": 3, "rgba": 4}


def _shape(width: int, height: int, channels: str):
    c = _CH[channels]
    return (height, width) if c == 1 else (height, width, c)


def output_path_for(path: str, prefix: str = "blur_") -> str:
    """``dir/x.raw`` -> ``dir/blur_x.raw`` (reference: ``"blur_" + argv[1]``)."""
    d, b = os.path.split(path)
    return os.path.join(d, prefix + b) if d else prefix + b


def read_raw(path: str, width: int, height: int, channels: str = "grey") -> np.ndarray:
    out = np.empty(_shape(width, height, channels), dtype=np.uint8)
    require_native().read_raw(path, out.reshape(-1), width, height, channels)
    return out


def write_raw(path: str, img: np.ndarray) -> None:
    arr = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = arr.shape[:2]
    ch = {2: "grey"}.get(arr.ndim) or {1: "grey", 3: "rgb", 4: "rgba"}[arr.shape[2]]
    require_native().write_raw(path, arr.reshape(-1), w, h, ch)


def synthetic_image(width: int, height: int, channels: str = "grey", seed: int = 0, y0: int = 0,
                    rows: int | None = None) -> np.ndarray:
    """Deterministic random-byte image (or rows [y0, y0+rows) of it) — the
    same bytes the native ``--synthetic SEED`` generator produces."""
    rows = height - y0 if rows is None else rows
    out = np.empty(_shape(width, rows, channels), dtype=np.uint8)
    require_native().synth_rows(out.reshape(-1), width, height, channels, int(seed), int(y0), int(rows))
    return out
