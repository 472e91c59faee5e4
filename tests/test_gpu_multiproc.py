"""Multi-process GPU engine on ONE GPU: N ranks (torch.distributed gloo) each
run a BandPipeline band on device 0; halos move through the host-staged gloo
transport (RCCL refuses two ranks on one device).  Exercises the real
multi-process band engine + pipeline + schedule with the HIP kernels; the
RCCL transport itself needs >= 2 GPUs (covered by the round-end 8-GPU run)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, ch, reps, halo, fuse, preload, slots, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from pconv.parallel.bootstrap import init_distributed, shutdown
    from pconv.parallel.dist_engine import DistributedBlur

    ctx = init_distributed("gloo")
    try:
        blur = DistributedBlur(w, h, ch, "gaussian", reps, rank=rank, world=world, device=0, halo=halo, fuse=fuse,
                               preload_halo=preload, slots=slots, transport="gloo-host")
        blur.load_synthetic(21)
        outs = []
        for _ in range(slots + 1):  # wrap the slot ring once
            k = blur.submit(reps)
            outs.append(k)
        blur.drain()
        res = [blur.outputs[k].copy() for k in outs[-slots:]]
        q.put((rank, blur.band.y0, res, blur.transport.exchanges))
    finally:
        shutdown(ctx)


@pytest.mark.parametrize("world,halo,fuse,preload,slots", [(2, 4, 4, False, 1), (2, 8, 4, True, 2),
                                                           (3, 6, 3, False, 3), (4, 16, 8, False, 2)])
def test_multiprocess_bands_one_gpu(pconv_mod, world, halo, fuse, preload, slots):
    w, h, ch, reps = 83, 97, "rgb", 19
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, ch, reps, halo, fuse, preload, slots, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = pconv_mod.numpy_convolve(pconv_mod.synthetic_image(w, h, ch, seed=21), reps)
    for i in range(slots):
        out = np.concatenate([r[2][i] for r in res]).reshape(ref.shape)
        assert np.array_equal(out, ref), (world, halo, fuse, preload, i)
    assert all(r[3] >= 1 for r in res)
