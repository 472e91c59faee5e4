"""CPU emulator of the distributed engine (torch.distributed ``gloo``).

Runs EXACTLY the schedule the GPUs run (``native.plan_band`` — the same C++
planner the ``BandEngine`` executes) on NumPy frames with the native CPU
stencil (``cpu_fused_launch`` = the reference semantics of one fused launch),
moving halo rows with ``gloo`` point-to-point messages.  This is how the
multi-rank decomposition, deep-halo and overlap logic is tested without GPUs
(SURVEY §4 "distributed tests without 8 GPUs"); the reference's own
multi-rank runs disagree with serial at block corners, this
emulator must agree bit for bit.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .._native import require_native
from ..models.filters import get_filter


class CpuBandRunner:
    def __init__(self, width: int, height: int, channels: str, filter="gaussian", *, rank: int, world: int,
                 halo: int = 1, fuse: int = 1, overlap: bool = True, omp: bool = False):
        n = require_native()
        self.n = n
        self.width, self.height, self.channels = int(width), int(height), channels
        self.ch = {"grey": 1, "rgb": 3, "rgba": 4}[channels]
        self.row_bytes = self.width * self.ch
        self.filter = get_filter(filter).to_native()
        self.rank, self.world = int(rank), int(world)
        self.band = n.row_band(self.height, self.world, self.rank)
        min_rows = self.height // self.world if self.world > 1 else 0
        self.halo, self.fuse = n.normalize_plan(int(halo), int(fuse), min_rows)
        self.overlap = overlap
        self.omp = omp
        lay = n.frame_layout(self.row_bytes, self.band.rows, self.halo)
        self.pitch, self.frame_bytes, self.pad_left = lay["pitch"], lay["bytes"], lay["pad_left"]
        self.frames = [np.zeros(self.frame_bytes, np.uint8), np.zeros(self.frame_bytes, np.uint8)]
        self.cur = 0
        self.exchanges = 0

    # frame helpers ----------------------------------------------------
    def _row_slice(self, r0: int, r1: int) -> slice:
        """Byte range of whole pitched frame rows [r0, r1) (frame-local rows)."""
        a = (r0 + self.halo) * self.pitch
        return slice(a, a + (r1 - r0) * self.pitch)

    def _rows_view(self, frame: np.ndarray, r0: int, r1: int) -> np.ndarray:
        v = frame[self._row_slice(r0, r1)].reshape(r1 - r0, self.pitch)
        return v[:, self.pad_left : self.pad_left + self.row_bytes]

    def load(self, owned_rows: np.ndarray) -> None:
        self.frames = [np.zeros(self.frame_bytes, np.uint8), np.zeros(self.frame_bytes, np.uint8)]
        self.cur = 0
        self._rows_view(self.frames[0], 0, self.band.rows)[:] = owned_rows.reshape(self.band.rows, self.row_bytes)

    def result(self) -> np.ndarray:
        return self._rows_view(self.frames[self.cur], 0, self.band.rows).copy()

    # halo exchange over gloo -------------------------------------------
    def _exchange(self, depth: int, group) -> None:
        src = self.frames[self.cur]
        b = self.band
        reqs, recv = [], []
        if b.up >= 0:
            buf = torch.empty(depth * self.pitch, dtype=torch.uint8)
            reqs.append(dist.irecv(buf, src=b.up, group=group))
            recv.append((buf, self._row_slice(-depth, 0)))
            reqs.append(dist.isend(torch.from_numpy(src[self._row_slice(0, depth)].copy()), dst=b.up, group=group))
        if b.down >= 0:
            buf = torch.empty(depth * self.pitch, dtype=torch.uint8)
            reqs.append(dist.irecv(buf, src=b.down, group=group))
            recv.append((buf, self._row_slice(b.rows, b.rows + depth)))
            reqs.append(dist.isend(torch.from_numpy(src[self._row_slice(b.rows - depth, b.rows)].copy()),
                                   dst=b.down, group=group))
        for r in reqs:
            r.wait()
        for buf, sl in recv:
            src[sl] = buf.numpy()
        self.exchanges += 1

    def run(self, reps: int, group=None, halo_preloaded: bool = False) -> None:
        plan = self.n.plan_band(self.band, int(reps), self.halo, self.fuse, self.overlap, halo_preloaded)
        for ph in plan:
            if ph.exchange_depth:
                self._exchange(ph.exchange_depth, group)
            src, dst = self.frames[self.cur], self.frames[self.cur ^ 1]
            for l in ph.launches:
                self.n.cpu_fused_launch(self.filter, self.channels, self.row_bytes, self.band.rows, self.halo, src, dst,
                                        l.lo, l.hi, l.steps, self.band.y0, self.height, self.omp)
            self.cur ^= 1


def local_cpu_cluster_convolve(image: np.ndarray, reps: int, world: int, filter="gaussian", *, halo: int = 1,
                               fuse: int = 1, overlap: bool = True, preload_halo: bool = False,
                               channels: Optional[str] = None) -> np.ndarray:
    """All `world` bands in this process, halos copied between NumPy frames —
    the CPU twin of the native one-device ``LocalCluster``."""
    img = np.ascontiguousarray(image, dtype=np.uint8)
    h, w = img.shape[:2]
    if channels is None:
        channels = "grey" if img.ndim == 2 else {1: "grey", 3: "rgb", 4: "rgba"}[img.shape[2]]
    rows = img.reshape(h, -1)
    runs = [CpuBandRunner(w, h, channels, filter, rank=r, world=world, halo=halo, fuse=fuse, overlap=overlap)
            for r in range(world)]
    for r in runs:
        r.load(rows[r.band.y0 : r.band.y0 + r.band.rows])
        if preload_halo:
            a = min(r.halo, r.band.y0)
            b = min(r.halo, h - (r.band.y0 + r.band.rows))
            if a:
                r._rows_view(r.frames[0], -a, 0)[:] = rows[r.band.y0 - a : r.band.y0]
            if b:
                e = r.band.y0 + r.band.rows
                r._rows_view(r.frames[0], r.band.rows, r.band.rows + b)[:] = rows[e : e + b]
    plans = [r.n.plan_band(r.band, int(reps), r.halo, r.fuse, overlap, preload_halo and world > 1) for r in runs]
    for i in range(len(plans[0])):
        for k, r in enumerate(runs):
            d = plans[k][i].exchange_depth
            if not d:
                continue
            b = r.band
            src = r.frames[r.cur]
            if b.up >= 0:
                p = runs[b.up]
                src[r._row_slice(-d, 0)] = p.frames[p.cur][p._row_slice(p.band.rows - d, p.band.rows)]
            if b.down >= 0:
                p = runs[b.down]
                src[r._row_slice(b.rows, b.rows + d)] = p.frames[p.cur][p._row_slice(0, d)]
            r.exchanges += 1
        for k, r in enumerate(runs):
            src, dst = r.frames[r.cur], r.frames[r.cur ^ 1]
            for l in plans[k][i].launches:
                r.n.cpu_fused_launch(r.filter, channels, r.row_bytes, r.band.rows, r.halo, src, dst, l.lo, l.hi,
                                     l.steps, r.band.y0, h, False)
            r.cur ^= 1
    return np.concatenate([r.result() for r in runs], axis=0).reshape(img.shape)


def distributed_cpu_convolve(image: np.ndarray, reps: int, filter="gaussian", *, halo: int = 1, fuse: int = 1,
                             overlap: bool = True, group=None, channels: Optional[str] = None) -> np.ndarray:
    """Every rank passes the full image; returns the full result on every rank
    (bands gathered with all_gather)."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    img = np.ascontiguousarray(image, dtype=np.uint8)
    h, w = img.shape[:2]
    if channels is None:
        channels = "grey" if img.ndim == 2 else {1: "grey", 3: "rgb", 4: "rgba"}[img.shape[2]]
    run = CpuBandRunner(w, h, channels, filter, rank=rank, world=world, halo=halo, fuse=fuse, overlap=overlap)
    rows = img.reshape(h, -1)
    run.load(rows[run.band.y0 : run.band.y0 + run.band.rows])
    run.run(reps, group)
    mine = run.result()
    if world == 1:
        return mine.reshape(img.shape)
    parts = [None] * world
    dist.all_gather_object(parts, mine, group=group)
    return np.concatenate(parts, axis=0).reshape(img.shape)
