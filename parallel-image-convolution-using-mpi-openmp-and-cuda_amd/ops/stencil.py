"""Stencil operators: the user-facing ``convolve`` and the persistent ``Engine``.

``convolve`` is the library form of the reference programs (repeated 3x3
convolution of an 8-bit grey/RGB image, zero padded): it dispatches to

* ``hip``   — the native CDNA4 kernels through a cached single-GPU
  :class:`Engine` (device-resident ping-pong frames, ``cuda/cuda_convolution.cu``
  analogue);
* ``omp`` / ``cpu`` — the native OpenMP / serial oracle (``open-mp/``, ``mpi/``);
* ``numpy`` — the independent pure-NumPy oracle (tests).

Images are ``(H, W)`` grey, ``(H, W, 3)`` RGB or ``(H, W, 4)`` RGBA uint8
arrays or tensors; CUDA tensors stay on the device (D2D copies on the
engine's stream, ordered after/before torch's current stream).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional, Tuple

import numpy as np
import torch

from .._native import require_native
from ..models.filters import get_filter
from .reference import numpy_convolve

_CHANNELS = {1: "grey", 3: "rgb", 4: "rgba"}


def image_geometry(shape) -> Tuple[int, int, str]:
    """(width, height, channels-name) of an (H, W[, C]) image."""
    if len(shape) == 2:
        return int(shape[1]), int(shape[0]), "grey"
    if len(shape) == 3 and int(shape[2]) in _CHANNELS:
        return int(shape[1]), int(shape[0]), _CHANNELS[int(shape[2])]
    raise ValueError(f"unsupported image shape {tuple(shape)}: expected (H, W) or (H, W, 1|3|4)")


class Engine:
    """Persistent single-GPU convolution engine for one image geometry.

    Device frames are allocated once; every call uploads, runs ``reps``
    repetitions with the fused kernels and downloads the newest buffer.
    """

    def __init__(self, width: int, height: int, channels: str = "grey", filter="gaussian", device: int = 0,
                 fuse: Optional[int] = None, graph: bool = False, variant: str = "auto"):
        n = require_native()
        self.filter = get_filter(filter)
        nf = self.filter.to_native()
        if fuse is None:
            ch = {"grey": 1, "rgb": 3, "rgba": 4}[channels]
            fuse = n.auto_fuse(nf, variant, int(width) * int(height) * ch, ch)
        self.width, self.height, self.channels = int(width), int(height), channels
        self.device = int(device)
        self._eng = n.BandEngine(self.width, self.height, channels, nf, 0, 1, self.device, halo=int(fuse),
                                 fuse=int(fuse), overlap=True, graph=bool(graph), variant=variant)
        self.row_bytes = self._eng.row_bytes

    @property
    def fuse(self) -> int:
        return self._eng.fuse

    @property
    def stats(self):
        return self._eng.stats

    def plan(self, reps: int):
        return self._eng.plan(reps)

    def run_numpy(self, img: np.ndarray, reps: int) -> np.ndarray:
        src = np.ascontiguousarray(img, dtype=np.uint8)
        out = np.empty_like(src)
        self._eng.upload(src.reshape(-1), 0, self.height)
        self._eng.run(int(reps))
        self._eng.download(out.reshape(-1), 0, self.height)
        self._eng.synchronize()
        return out

    def run_tensor(self, t: torch.Tensor, reps: int) -> torch.Tensor:
        if t.device.type != "cuda":
            return torch.from_numpy(self.run_numpy(t.numpy(), reps))
        src = t.contiguous()
        out = torch.empty_like(src)
        ts = torch.cuda.current_stream(src.device).cuda_stream
        self._eng.wait_stream(ts)
        self._eng.upload_ptr(src.data_ptr(), self.row_bytes, 0, self.height, device=True)
        self._eng.run(int(reps))
        self._eng.download_ptr(out.data_ptr(), self.row_bytes, 0, self.height, device=True)
        self._eng.signal_stream(ts)
        src.record_stream(torch.cuda.current_stream(src.device))
        return out

    def __call__(self, img, reps: int):
        if isinstance(img, torch.Tensor):
            return self.run_tensor(img, reps)
        return self.run_numpy(np.asarray(img), reps)


_ENGINES: "OrderedDict[tuple, Engine]" = OrderedDict()
_MAX_CACHED = 8


def _cached_engine(w, h, ch, flt, device, fuse, graph, variant) -> Engine:
    key = (w, h, ch, flt.taps, flt.divisor, device, fuse, graph, variant)
    eng = _ENGINES.get(key)
    if eng is None:
        eng = Engine(w, h, ch, flt, device=device, fuse=fuse, graph=graph, variant=variant)
        _ENGINES[key] = eng
        while len(_ENGINES) > _MAX_CACHED:
            _ENGINES.popitem(last=False)
    else:
        _ENGINES.move_to_end(key)
    return eng


def _default_backend() -> str:
    try:
        require_native()
    except ImportError:
        return "numpy"
    return "hip" if torch.cuda.is_available() else "omp"


def convolve(image, reps: int = 1, filter="gaussian", backend: str = "auto", device: Optional[int] = None,
             fuse: Optional[int] = None, graph: bool = False, variant: str = "auto", threads: int = 0):
    """Apply ``reps`` zero-padded 3x3 convolutions to an 8-bit image.

    Returns the same container type as the input (NumPy array or torch tensor
    on the same device).
    """
    if reps < 0:
        raise ValueError("reps must be >= 0")
    flt = get_filter(filter)
    is_tensor = isinstance(image, torch.Tensor)
    if is_tensor and image.dtype != torch.uint8:
        raise TypeError("image tensor must be uint8")
    w, h, ch = image_geometry(tuple(image.shape))
    if backend == "auto":
        backend = "hip" if (is_tensor and image.is_cuda) else _default_backend()

    if backend == "numpy":
        arr = image.cpu().numpy() if is_tensor else np.asarray(image)
        out = numpy_convolve(arr, reps, flt)
        return torch.from_numpy(out).to(image.device) if is_tensor else out

    if backend in ("cpu", "omp"):
        n = require_native()
        arr = np.ascontiguousarray(image.cpu().numpy() if is_tensor else image, dtype=np.uint8)
        out = np.empty_like(arr)
        n.cpu_convolve(arr.reshape(-1), out.reshape(-1), w, h, ch, int(reps), flt.to_native(), backend == "omp",
                       int(threads))
        return torch.from_numpy(out).to(image.device) if is_tensor else out

    if backend == "hip":
        if device is None:
            device = image.device.index if (is_tensor and image.is_cuda) else 0
        eng = _cached_engine(w, h, ch, flt, int(device or 0), fuse, graph, variant)
        return eng(image, reps)

    raise ValueError(f"unknown backend {backend!r} (hip|omp|cpu|numpy|auto)")


def convolve_file(path: str, width: int, height: int, reps: int, channels: str = "grey", filter="gaussian",
                  out: Optional[str] = None, backend: str = "auto", device: Optional[int] = None) -> str:
    """The reference program in one call (``cuda/main.c:10-53``): read the raw
    image, ``reps`` repetitions, write ``blur_<name>`` (or ``out``); returns the
    output path."""
    from ..utils.raw_io import output_path_for, read_raw, write_raw

    img = read_raw(path, width, height, channels)
    res = convolve(img, reps, filter, backend=backend, device=device)
    dst = out or output_path_for(path)
    write_raw(dst, res)
    return dst
