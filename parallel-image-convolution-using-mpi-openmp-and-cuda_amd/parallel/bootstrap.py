"""Process-group bootstrap (one process per GPU).

Reference: ``MPI_Init`` / ``MPI_Comm_size`` / ``MPI_Comm_rank``
(``mpi/mpi_convolution.c:23-25``) and six ``MPI_Bcast`` of the configuration
(``:65-70``).  Here the launcher is ``torch.distributed.run`` (RANK,
WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT in the environment); the control
plane is a ``gloo`` process group (CPU: barriers, config/unique-id broadcast,
max-reduction of timings) and the data plane is a native RCCL communicator
(halo rows over xGMI) created from a unique id broadcast over that group.
Every rank parses the same argv, so no configuration broadcast is needed.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .._native import require_native


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    initialized_here: bool = False

    @property
    def is_distributed(self) -> bool:
        return self.world > 1


def env_context() -> DistContext:
    return DistContext(
        rank=int(os.environ.get("RANK", "0")),
        world=int(os.environ.get("WORLD_SIZE", "1")),
        local_rank=int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))),
    )


def init_distributed(backend: str = "gloo", timeout_s: float = 600.0) -> DistContext:
    """Initialise torch.distributed from the environment if WORLD_SIZE > 1."""
    ctx = env_context()
    if ctx.world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        import datetime

        dist.init_process_group(backend=backend, rank=ctx.rank, world_size=ctx.world,
                                timeout=datetime.timedelta(seconds=timeout_s))
        ctx.initialized_here = True
    require_native().set_error_rank(ctx.rank)
    return ctx


def broadcast_bytes(data: Optional[bytes], src: int = 0, group=None) -> bytes:
    """Broadcast a small byte string from ``src`` over the (gloo) group."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        assert data is not None
        return data
    obj = [data]
    dist.broadcast_object_list(obj, src=src, group=group)
    return obj[0]


def single_node(world: int) -> bool:
    """All `world` ranks on this host (torchrun exports LOCAL_WORLD_SIZE)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", world)) >= world


def make_rccl_comm(device: int, group=None):
    """Create the native RCCL communicator for this rank (collective).

    On one node the communicator's bootstrap sockets go over loopback
    (NCCL_SOCKET_IFNAME=lo unless the user set it): the data moves over
    xGMI / P2P anyway, and a host whose only interfaces are loopback or
    unreachable container bridges then cannot stall the first RCCL call.
    librccl is loaded on that first call, so the variable is still unread."""
    n = require_native()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if single_node(world):
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    uid = n.rccl_unique_id() if rank == 0 else None
    uid = broadcast_bytes(uid, 0, group)
    return n.RcclComm(uid, rank, world, device)


def make_ipc_transports(engines, timeout_s: float = 30.0, group=None, pull: str = "grid"):
    """HIP-IPC halo transports for this rank's pipeline slots (collective).

    Rank 0 creates the job's shared flag segment and broadcasts its name;
    every rank maps it, exports its slot engines' frames with
    hipIpcGetMemHandle, the handles of all ranks are gathered, and each slot
    opens its neighbours' frames (slot k of rank r exchanges with slot k of
    ranks r-1 and r+1).  Once every rank has mapped the segment its name is
    unlinked, so nothing is left in /dev/shm whatever happens later.
    Replaces the reference's MPI_Isend/Irecv set-up of neighbour ranks
    (mpi/mpi_convolution.c:142-149) for ranks on one node."""
    import secrets

    n = require_native()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    slots = len(engines)
    name, err = None, None
    if rank == 0:
        name = f"/pconv_ipc_{os.getpid()}_{secrets.token_hex(4)}"
        try:
            n.ipc_create_segment(name, world, slots)
        except Exception as e:  # every rank must hear of it, not wait in the broadcast
            err, name = e, ""
    created = False
    try:
        # an empty name tells the other ranks that rank 0 could not create the segment
        name = broadcast_bytes(name.encode() if name is not None else None, 0, group).decode()
        if not name:
            raise RuntimeError(f"IPC halo segment creation failed on rank 0: {err}")
        created = True
        ts = [n.IpcHaloTransport(e, name, k, slots, float(timeout_s), pull) for k, e in enumerate(engines)]
    finally:
        barrier(group)
        if rank == 0 and created:
            n.ipc_unlink_segment(name)
    mine = [t.local_handles() for t in ts]
    if dist.is_initialized() and world > 1:
        every = [None] * world
        dist.all_gather_object(every, mine, group=group)
    else:
        every = [mine]
    for k, (t, e) in enumerate(zip(ts, engines)):
        b = e.band
        up = every[b.up][k] if b.up >= 0 else b""
        down = every[b.down][k] if b.down >= 0 else b""
        t.connect(up, down)
    barrier(group)
    # One exchange of sentinel rows per transport (slot order, like every
    # rank): a neighbour's stores or rows this rank cannot see raise a named
    # error now instead of timing out the first real exchange.
    for t in ts:
        t.self_test(min(5.0, float(timeout_s)))
    barrier(group)
    return ts


def max_over_ranks(value: float, group=None) -> float:
    """Max of a float over ranks (the reference's Send/Recv max-gather,
    ``mpi/mpi_convolution.c:264-275``)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sum_over_ranks(value: int, group=None) -> int:
    """Integer sum over ranks (mismatch counts of distributed checks)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())


def barrier(group=None) -> None:
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.barrier(group=group)


def shutdown(ctx: DistContext) -> None:
    if ctx.initialized_here and dist.is_initialized():
        dist.destroy_process_group()


def parse_cpulist(text: str) -> set:
    """Parse a sysfs cpulist ("0-3,8,10-11") into a set of CPU ids."""
    cpus = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def device_local_cpus(device: int, sysfs: str = "/sys/bus/pci/devices") -> Optional[set]:
    """CPUs on the NUMA node of GPU `device` (its PCIe root), or None if the
    platform does not say.  The pinned staging buffers of a rank are written
    by its host thread and read by its GPU's copy engines over that GPU's own
    PCIe link; keeping the thread (and so first-touch allocations) on the
    GPU's socket avoids crossing the inter-socket fabric on every copy."""
    try:
        bdf = require_native().device_pci_bus_id(device)
        with open(os.path.join(sysfs, bdf, "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
    except Exception:  # no device / no sysfs entry: leave the affinity alone
        return None
    return cpus or None


def bind_to_device_numa(device: int, enabled: bool = True) -> Optional[int]:
    """Restrict this process to the CPUs local to its GPU (intersected with
    the CPUs it may use); `enabled=False` (bench.py --numa-bind off) leaves
    the affinity alone.  Returns the number of CPUs kept, or None when
    nothing was changed."""
    if not enabled or not hasattr(os, "sched_setaffinity"):
        return None
    local = device_local_cpus(device)
    if not local:
        return None
    allowed = os.sched_getaffinity(0)
    keep = local & allowed
    if not keep or keep == allowed:
        return None
    os.sched_setaffinity(0, keep)
    return len(keep)


def cpu_rank_slice(local_rank: int, local_world: int, allowed, budget: int) -> list:
    """Disjoint CPU slice of one CPU rank of the MPI+OpenMP analog.

    The node's CPU budget (the CPUs this process may use, capped by the
    cgroup quota, one kept back for the launcher and the gloo threads) is
    split evenly between the ranks of the node; rank r gets the r-th block.
    More ranks than budget CPUs share (round-robin) rather than fail."""
    cpus = sorted(allowed)[:max(1, int(budget))]
    k = max(1, len(cpus) // max(1, int(local_world)))
    lo = (int(local_rank) * k) % len(cpus)
    return cpus[lo:lo + k]


def bind_cpu_rank(local_rank: int, local_world: int, bind: bool = False) -> Optional[list]:
    """Opt-in (`bind=True`, run.py --cpu-bind): bind this CPU rank to its slice
    (``cpu_rank_slice``) before its OpenMP team starts (team threads inherit
    the affinity of the thread that creates them).  Always: torch's own pools
    drop to one thread, so a rank runs its team and nothing else.

    Measured on the GPU box's CPU share (16 CPUs of a shared 256-CPU host,
    profiles/r03/hybrid/): binding to fixed CPUs puts the teams on CPUs other
    tenants also use (bound teams showed 14-190 ms stalls); unbound teams
    sized budget / ranks with passive waits (the package default, _native.py)
    were the steadiest, so binding is off by default.  Reference: one team
    per rank (open-mp/omp_convolution.c:292,297)."""
    torch.set_num_threads(1)
    if not bind or not hasattr(os, "sched_setaffinity"):
        return None
    n = require_native()
    budget = n.default_cpu_threads()
    mine = cpu_rank_slice(local_rank, local_world, os.sched_getaffinity(0), budget)
    os.sched_setaffinity(0, mine)
    return mine
