"""Filter zoo — the engine's "model family".

The reference defines three 3x3 kernels and selects one by (un)commenting
source (``mpi/mpi_convolution.c:90-101``):

* ``gaussian``  ``[[1,2,1],[2,4,2],[1,2,1]] / 16``  (active; also hard-coded in
  ``cuda/cuda_convolution.cu:12,29``)
* ``box``       all ones / 9                          (commented out, ``:90,98``)
* ``edge``      ``[[1,4,1],[4,8,4],[1,4,1]] / 28``  (``edge_detection``, ``:92,100``;
  despite the name a positive smoother)

Weights follow the reference construction ``(float)(tap / (double)divisor)``.
``int_exact`` marks filters whose float32 evaluation equals the integer formula
``(sum tap*p) >> log2(divisor)`` bit for bit (power-of-two divisor, non-negative
taps); those run on the packed-integer GPU kernels, the others on the float32
kernel that replays the reference's multiply-then-add order.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Sequence, Tuple

import numpy as np


@dataclass(frozen=True)
class Filter:
    name: str
    taps: Tuple[int, ...]
    divisor: int
    weights: Tuple[float, ...] = field(init=False)
    int_exact: bool = field(init=False)
    shift: int = field(init=False)

    def __post_init__(self):
        if len(self.taps) != 9:
            raise ValueError("a 3x3 filter needs 9 taps")
        if self.divisor <= 0:
            raise ValueError("divisor must be positive")
        w = tuple(float(np.float32(t / float(self.divisor))) for t in self.taps)
        object.__setattr__(self, "weights", w)
        pow2 = (self.divisor & (self.divisor - 1)) == 0
        nonneg = all(t >= 0 for t in self.taps)
        exact = pow2 and nonneg and sum(abs(t) for t in self.taps) * 255 < (1 << 24)
        object.__setattr__(self, "int_exact", exact)
        object.__setattr__(self, "shift", int(self.divisor).bit_length() - 1 if pow2 else 0)

    @property
    def matrix(self) -> np.ndarray:
        return np.array(self.taps, dtype=np.int64).reshape(3, 3)

    @property
    def weights32(self) -> np.ndarray:
        return np.array(self.weights, dtype=np.float32).reshape(3, 3)

    def to_native(self):
        from .._native import require_native

        return require_native().Filter.custom(list(self.taps), int(self.divisor), self.name)


_REGISTRY: Dict[str, Filter] = {
    "gaussian": Filter("gaussian", (1, 2, 1, 2, 4, 2, 1, 2, 1), 16),
    "box": Filter("box", (1, 1, 1, 1, 1, 1, 1, 1, 1), 9),
    "edge": Filter("edge", (1, 4, 1, 4, 8, 4, 1, 4, 1), 28),
}


def list_filters():
    return sorted(_REGISTRY)


def get_filter(f) -> Filter:
    """Accept a name, a Filter, or (taps, divisor)."""
    if isinstance(f, Filter):
        return f
    if isinstance(f, str):
        key = "edge" if f == "edge_detection" else f
        if key not in _REGISTRY:
            raise ValueError(f"unknown filter {f!r}; known: {list_filters()}")
        return _REGISTRY[key]
    if isinstance(f, (tuple, list)) and len(f) == 2:
        taps, div = f
        return Filter("custom", tuple(int(t) for t in np.asarray(taps).reshape(-1)), int(div))
    raise TypeError(f"cannot interpret {f!r} as a filter")


def register_filter(name: str, taps: Sequence[int], divisor: int) -> Filter:
    flt = Filter(name, tuple(int(t) for t in taps), int(divisor))
    _REGISTRY[name] = flt
    return flt
