"""Halo transports besides the native RCCL one.

``GlooHostTransport`` stages ghost rows through pinned host memory and moves
them with ``torch.distributed`` (gloo) point-to-point messages.  It is the
reference's MPI_Isend/Irecv (``mpi/mpi_convolution.c:157-192``) done on the
host, and exists for environments where RCCL cannot run — notably several
ranks sharing ONE GPU (RCCL rejects duplicate devices in a communicator),
which is how the multi-process GPU engine is tested on a one-GPU box.  It is
synchronous (no overlap); the native RCCL transport is the production path.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .._native import require_native


class GlooHostTransport(require_native().HaloTransport):
    def __init__(self, group=None):
        super().__init__()
        self.group = group
        self.n = require_native()
        self._bufs = {}
        self.exchanges = 0

    def _buf(self, key, nbytes):
        b = self._bufs.get(key)
        if b is None or len(b) < nbytes:
            b = self.n.PinnedBuffer(nbytes)
            self._bufs[key] = b
        return b

    def exchange_rows(self, row0_ptr, pitch, rows, up, down, depth, stream):
        n = self.n
        nbytes = depth * pitch
        sends = []
        if up >= 0:
            b = self._buf("su", nbytes)
            n.memcpy_async(b.ptr, row0_ptr, nbytes, "d2h", stream)
            sends.append((b, up))
        if down >= 0:
            b = self._buf("sd", nbytes)
            n.memcpy_async(b.ptr, row0_ptr + (rows - depth) * pitch, nbytes, "d2h", stream)
            sends.append((b, down))
        n.stream_synchronize(stream)
        reqs, recvs = [], []
        for key, peer, dst in (("ru", up, row0_ptr - nbytes), ("rd", down, row0_ptr + rows * pitch)):
            if peer < 0:
                continue
            t = torch.empty(nbytes, dtype=torch.uint8)
            reqs.append(dist.irecv(t, src=peer, group=self.group))
            recvs.append((t, dst))
        for b, peer in sends:
            t = torch.from_numpy(np.asarray(b)[:nbytes].copy())
            reqs.append(dist.isend(t, dst=peer, group=self.group))
        for r in reqs:
            r.wait()
        for t, dst in recvs:
            n.memcpy_async(dst, t.data_ptr(), nbytes, "h2d", stream)
        n.stream_synchronize(stream)
        self.exchanges += 1
