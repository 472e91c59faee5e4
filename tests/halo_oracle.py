"""Oracle of a self-neighbour band's run (shared by the GPU RCCL tests and the
CPU check of the oracle itself)."""
import numpy as np


def reflected_ghost_oracle(n, plan, halo, owned, y0, height, channels, filt="gaussian", pre_exchange=0):
    """NumPy/CPU model of a band's `plan` on a self-neighbour band: before
    every exchange phase the ghost zone is refreshed with the band's own rows
    (above: rows [0, d); below: rows [rows - d, rows)), exactly what RCCL
    send/recv-to-self delivers; launches are the CPU twin of a fused launch
    (`cpu_fused_launch`, reference tap order, per-step truncation, zeros
    outside the global image)."""
    rows, rb = owned.shape
    lay = n.frame_layout(rb, rows, halo)
    pitch, pad = lay["pitch"], lay["pad_left"]
    frames = [np.zeros(lay["bytes"], np.uint8), np.zeros(lay["bytes"], np.uint8)]

    def view(f, r0, r1):
        return f[(r0 + halo) * pitch:(r1 + halo) * pitch].reshape(r1 - r0, pitch)[:, pad:pad + rb]

    view(frames[0], 0, rows)[:] = owned
    cur = 0
    # pre_exchange: an exchange of that depth before the plan (a pipeline's
    # whole-zone exchange right after the upload)
    for ph in [None] + list(plan):
        if ph is None and not pre_exchange:
            continue
        src, dst = frames[cur], frames[cur ^ 1]
        d = pre_exchange if ph is None else ph.exchange_depth
        if d:
            top, bottom = view(src, 0, d).copy(), view(src, rows - d, rows).copy()
            view(src, -d, 0)[:] = top
            view(src, rows, rows + d)[:] = bottom
            # ghost rows outside the global image: the GPU kernels read them
            # as zeros whatever the frame holds; the CPU twin reads the frame
            a, b = max(-d, -y0), min(rows + d, height - y0)
            view(src, -d, a)[:] = 0
            view(src, b, rows + d)[:] = 0
        if ph is None:
            continue
        for l in ph.launches:
            n.cpu_fused_launch(filt, channels, rb, rows, halo, src, dst, l.lo, l.hi, l.steps, y0, height, False)
        cur ^= 1
    return view(frames[cur], 0, rows).copy()
