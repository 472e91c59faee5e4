"""Per-launch latency of the fused temporal kernel vs steps and tile shape.

Launches the kernel on a small region (one row-tile high) and a full image
back to back with hipEvents around each, to split a launch's cost into a
fixed part and a per-step part (fit t = a + b*steps).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import pconv

    n = pconv.native
    W, H = 1920, 2520
    rb = W * 3
    halo = 16
    lay = n.frame_layout(rb, H, halo)
    src = torch.randint(0, 256, (lay["bytes"],), dtype=torch.uint8, device="cuda")
    dst = torch.zeros_like(src)
    base = lay["pitch"] * halo + 16
    s = torch.cuda.current_stream()
    shapes = sys.argv[1].split(";") if len(sys.argv) > 1 else ["4,5,8", "4,4,8", "8,8,8", "4,8,8"]
    for shape in shapes:
        n.set_swar_shape(*map(int, shape.split(",")))
        for rows in (16, 100, 400, 2520):
            res = []
            for steps in (1, 2, 4, 8, 16):
                _, m, nw = map(int, shape.split(","))
                if m * nw <= 2 * steps:
                    continue
                times = []
                for it in range(12):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    n.launch_stencil("gaussian", "rgb", src.data_ptr() + base, dst.data_ptr() + base, lay["pitch"],
                                     rb, 0, rows, -halo, H + halo, steps, 0, H, s.cuda_stream, "temporal")
                    e1.record(s)
                    e1.synchronize()
                    times.append(e0.elapsed_time(e1) * 1000)
                res.append((steps, float(np.median(times[2:]))))
            if len(res) >= 2:
                st = np.array([r[0] for r in res], float)
                tt = np.array([r[1] for r in res])
                b, a = np.polyfit(st, tt, 1)
            else:
                a = b = float("nan")
            print(json.dumps({"shape": shape, "rows": rows, "us_by_steps": {str(k): round(v, 2) for k, v in res},
                              "fixed_us": round(float(a), 2), "per_step_us": round(float(b), 3)}), flush=True)


if __name__ == "__main__":
    main()
