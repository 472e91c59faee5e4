"""Two ranks of the distributed engine with RCCL halo exchange.

Launch: python -m torch.distributed.run --nnodes=1 --nproc-per-node 2
        --master-addr 127.0.0.1 --master-port P tools/rccl_pair_test.py [--same-device]

--same-device puts both ranks on GPU 0 (a one-GPU box); RCCL may refuse
duplicate devices in one communicator, in which case this prints the error.
Checks the gathered result against the CPU oracle, with and without a
preloaded ghost zone (0 vs >= 1 RCCL exchanges in the timed loop).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch.distributed as dist

    import pconv
    from pconv.parallel.bootstrap import init_distributed, shutdown
    from pconv.parallel.dist_engine import DistributedBlur

    same = "--same-device" in sys.argv
    ctx = init_distributed("gloo")
    dev = 0 if same else ctx.local_rank
    W, H, reps = 97, 64, 13
    full = pconv.synthetic_image(W, H, "rgb", seed=11)
    ref = pconv.numpy_convolve(full, reps)
    ok = True
    for preload, halo, fuse in ((False, 4, 2), (True, 8, 4), (False, 16, 8)):
        blur = DistributedBlur(W, H, "rgb", "gaussian", reps, rank=ctx.rank, world=ctx.world, device=dev,
                               halo=halo, fuse=fuse, preload_halo=preload)
        blur.load_synthetic(11)
        blur.step(reps)
        parts = [None] * ctx.world
        dist.all_gather_object(parts, (blur.band.y0, blur.output.copy(), blur.stats.exchanges))
        if ctx.rank == 0:
            parts.sort(key=lambda p: p[0])
            out = np.concatenate([p[1] for p in parts]).reshape(full.shape)
            bad = int((out != ref).sum())
            print(f"preload={preload} halo={halo} fuse={fuse} exchanges={[p[2] for p in parts]} mismatches={bad}",
                  flush=True)
            ok = ok and bad == 0
        del blur
    if ctx.rank == 0:
        print("RCCL PAIR OK" if ok else "RCCL PAIR FAILED", flush=True)
    shutdown(ctx)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
