"""pconv — an MI355X-native 2-D image-convolution stencil engine.

Capabilities of theopaid/Parallel-Image-Convolution-using-MPI-OPENMP-and-CUDA
(reference at /root/reference), rebuilt for AMD Instinct MI355X:

* the reference CLI ``conv image.raw W H reps {grey,rgb}`` and its raw
  8-bit grey / interleaved-RGB files, output ``blur_<name>``
  (``cuda/main.c:10-53``, ``mpi/mpi_convolution.c:17-286``);
* repeated zero-padded 3x3 convolution with the gaussian (plus the
  reference's box and "edge" filters), bit-exact to the reference's float32
  arithmetic (``mpi/mpi_convolution.c:88-102, 288-322``);
* a serial / OpenMP CPU path that doubles as the test oracle
  (``open-mp/omp_convolution.c``);
* hand-written CDNA4 HIP kernels (packed 16-bit integer SIMD, temporal
  blocking), a HIP-stream/hipGraph runtime (``cuda/cuda_convolution.cu``);
* row-band domain decomposition over 1-8 GPUs, one process per GPU, halo rows
  exchanged with RCCL over xGMI overlapped with interior compute
  (``mpi/mpi_convolution.c:142-240``).

Layout: ``ops`` (kernels / operators), ``models`` (filters and convolution
pipelines), ``parallel`` (bootstrap, distributed engine, CPU emulator),
``utils`` (raw I/O, metrics, CLI), ``csrc`` (C++/HIP sources).
"""
from __future__ import annotations

__version__ = "0.1.0"

from ._native import native, native_available  # noqa: E402  (loads torch first)
from .models.filters import Filter, get_filter, list_filters  # noqa: E402
from .ops.stencil import convolve, convolve_file, Engine  # noqa: E402
from .models.pipeline import FilterPipeline  # noqa: E402
from .ops.reference import numpy_convolve  # noqa: E402
from .utils.raw_io import read_raw, write_raw, output_path_for, synthetic_image  # noqa: E402

__all__ = [
    "native",
    "native_available",
    "Filter",
    "get_filter",
    "list_filters",
    "convolve",
    "convolve_file",
    "Engine",
    "FilterPipeline",
    "numpy_convolve",
    "read_raw",
    "write_raw",
    "output_path_for",
    "synthetic_image",
]
