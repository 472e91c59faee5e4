"""Independent pure-NumPy oracle.

Kept deliberately separate from the C++ oracle (``csrc/src/cpu_stencil.cpp``)
so the two check each other (SURVEY §4 "keeps the C++ oracle honest").

Semantics (reference ``mpi/mpi_convolution.c:301-322``): per
channel, ``out[y][x] = trunc(sum_{k,l} w[k][l] * in[y+k-1][x+l-1])`` with zero
padding, float32 multiply-then-add in row-major tap order starting from 0.0f.
NumPy's float32 elementwise ops round each multiply and add separately (no FMA),
which reproduces the reference bit for bit; integer-exact filters use
``(sum tap*p) >> shift`` directly.
"""
from __future__ import annotations

import numpy as np

from ..models.filters import get_filter


def _as_hwc(img: np.ndarray) -> np.ndarray:
    if img.ndim == 2:
        return img[:, :, None]
    if img.ndim == 3:
        return img
    raise ValueError("image must be (H, W) or (H, W, C)")


def numpy_step(img: np.ndarray, filt="gaussian") -> np.ndarray:
    f = get_filter(filt)
    x = _as_hwc(np.asarray(img, dtype=np.uint8))
    h, w, _ = x.shape
    p = np.pad(x, ((1, 1), (1, 1), (0, 0)))
    if f.int_exact:
        acc = np.zeros(x.shape, dtype=np.int64)
        for k in range(3):
            for l in range(3):
                t = f.taps[3 * k + l]
                if t:
                    acc += t * p[k : k + h, l : l + w].astype(np.int64)
        out = np.minimum(acc >> f.shift, 255).astype(np.uint8)
    else:
        acc = np.zeros(x.shape, dtype=np.float32)
        w32 = f.weights32
        for k in range(3):
            for l in range(3):
                prod = p[k : k + h, l : l + w].astype(np.float32) * w32[k, l]
                acc = (acc + prod).astype(np.float32)
        acc = np.where(acc > 0, acc, 0).astype(np.float32)
        out = np.minimum(np.trunc(acc), 255).astype(np.uint8)
    return out.reshape(img.shape)


def numpy_convolve(img: np.ndarray, reps: int = 1, filt="gaussian") -> np.ndarray:
    out = np.asarray(img, dtype=np.uint8).copy()
    for _ in range(int(reps)):
        out = numpy_step(out, filt)
    return out
