"""Command-line front end.

``python -m pconv image.raw W H reps {grey,rgb} [options]`` runs the native
``conv`` driver in-process (same argv contract and output as the reference
programs, ``cuda/main.c`` / ``mpi/mpi_convolution.c``).  ``--gpus N`` forks one
worker per GPU before any HIP call, like ``mpiexec -n N``.  Under
``torch.distributed.run`` use :mod:`pconv.parallel.run` instead.
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional

from .._native import require_native


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv if argv is None else argv)
    if argv:
        argv[0] = os.path.basename(argv[0]) if argv[0].endswith("__main__.py") else argv[0]
    sys.stdout.flush()
    return int(require_native().conv_main(argv))


if __name__ == "__main__":
    sys.exit(main())
