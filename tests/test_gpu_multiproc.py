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


@pytest.mark.parametrize("world,extra", [(2, []), (3, ["--halo-mode", "exchange"]), (4, []), (8, []),
                                         (2, ["--slots", "1", "--no-overlap", "--halo-mode", "exchange"]),
                                         (2, ["--halo-select", "exchange"]), (3, ["--halo-select", "overlap"]),
                                         (2, ["--halo-select", "event"])])
def test_bench_torchrun_rehearsal(world, extra):
    """bench.py under torch.distributed.run with `world` ranks sharing the one
    GPU (gloo-host halos): the driver's N-GPU launch path with its default
    oracle check (no --check flag: every BENCH line is self-verifying), every
    halo mode timed after the headline and compared with the CPU oracle."""
    import json
    import subprocess
    import sys

    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "3", "--warmup", "1", "--transport", "gloo-host"] + extra
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    meta = json.loads(lines[0])
    assert meta["n_gpus"] == world and meta["mismatches"] == 0
    assert meta["value"] > 0 and meta["config"]["parallelism"] == f"rowband{world}"
    assert meta["runtime"]["hip_runtime_version"] > 0 and meta["runtime"]["hip_runtime_path"]
    assert len(meta["per_rank_ms_per_step"]) == world
    # PCIe bytes per rank: band (+ pre-loaded ghost rows) in, owned rows out; the bands tile the image
    assert len(meta["h2d_bytes_per_step"]) == world and len(meta["d2h_bytes_per_step"]) == world
    assert sum(meta["d2h_bytes_per_step"]) == 1920 * 2520 * 3
    assert all(i >= o for i, o in zip(meta["h2d_bytes_per_step"], meta["d2h_bytes_per_step"]))
    assert meta["config"]["ipc_pull"] == "grid" and meta["config"]["cu_mask_queues"] is True
    modes = meta["halo_modes"]
    head = "event" if "--halo-mode" in extra else "preload"
    assert set(modes) == {head, "slot_exchange", "slot_exchange_direct", "event", "overlap", "ipc"}, modes
    for m, r in modes.items():
        assert r["status"] == "ok", (m, r)
        assert r["ms_per_step"] > 0
        if m != head:
            assert len(r["per_rank_ms_per_step"]) == world and len(r["h2d_bytes_per_step"]) == world, (m, r)
        assert r["mismatches"] == 0, (m, r)  # every mode against the oracle, not only the headline's bytes
        if m != head:
            assert r["mismatches_vs_headline"] == 0 and r["exchanges_per_step"] >= 1, (m, r)
    # the reference's loop-only MPI timing on the resident bands, exchanges through the event mode's transport
    if head != "event":
        rl = meta["resident_loop"]
        assert rl == modes["event"]["resident_loop"] and rl["transport"] == "GlooHostTransport", rl
        assert rl["ms_per_image"] > 0 and rl["exchanges_per_image"] >= 40 // rl["halo_rows"], rl
        assert rl["one_graph_per_image"] is False  # host-staged halos cannot be captured
        g = rl["ghost_bytes_per_exchange"]  # per rank: one side at the image edges, two inside
        assert len(g) == world and g[0] == g[-1] and all(x == 2 * g[0] for x in g[1:-1]), g
        ri = meta["resident_loop_ipc"]  # the same loop with HIP-IPC pulls, captured
        assert ri == modes["ipc"]["resident_loop"] and ri["transport"] == "ipc-grid", ri
        assert ri["ms_per_image"] > 0 and ri["exchanges_per_image"] == rl["exchanges_per_image"], ri
        assert ri["one_graph_per_image"] is True and ri["ghost_bytes_per_exchange"] == g
    # overlap: a T-deep ghost zone, one exchange per fused launch (the reference's per-rep loop, T at a time)
    assert modes["overlap"]["halo_depth"] == modes["overlap"]["fuse"]
    assert modes["overlap"]["exchanges_per_step"] >= 40 // modes["overlap"]["fuse"]
    sel = meta["halo_select"]
    assert set(sel["candidates"]) == set(modes)
    if "--halo-select" in extra:  # forced adoption: the headline is the K timed steps of that mode
        want = extra[extra.index("--halo-select") + 1]
        want = "slot_exchange" if want == "exchange" else want
        assert sel["mode"] == want and meta["config"]["halo_mode"] == want
        assert meta["ms_per_step"] == modes[want]["ms_per_step"]
        assert meta["headline_transport"] == "gloo-host" and meta["config"]["exchanges_per_step"] >= 1
        assert meta["config"]["preload_halo"] is False
        assert "loop_only" not in meta and "loop_only" in modes["preload"]
    else:
        assert sel["mode"] in modes


def test_bench_exchange_watchdog():
    """A peer that never joins the secondary halo-mode measurement: the
    watchdog still prints the headline line (the mode marked timed out), so
    the driver's N-GPU run always yields its number, and the ranks exit with
    status 3 so that the stall is visible to whoever checks the exit code."""
    import json
    import subprocess
    import sys
    import time

    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--transport", "gloo-host", "--stall-exchange",
           "--watchdog", "8"]
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, "a fired watchdog must not look like a clean run"
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    meta = json.loads(lines[0])
    assert meta["n_gpus"] == 2 and meta["value"] > 0 and meta["mismatches"] == 0
    assert meta["halo_modes"]["slot_exchange"]["status"] == "watchdog timeout"
    assert meta["watchdog"].startswith("fired")
    assert meta["headline_transport"] == "none"
    assert time.time() - t0 < 250


@pytest.mark.parametrize("world,extra", [(2, []), (3, ["--exchange-halo", "--halo", "3", "--fuse", "3"]),
                                         (2, ["--filter", "box"])])
def test_torchrun_per_rank_program_hip(pconv_mod, tmp_path, world, extra):
    """`torch.distributed.run -m pconv.parallel.run --backend hip`: ranks share
    the GPU, halos via gloo-host; the written file equals the oracle."""
    import json
    import subprocess
    import sys

    img = np.random.default_rng(world).integers(0, 256, size=(61, 47, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "pic.raw"), img)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", "-m", "pconv.parallel.run",
           "pic.raw", "47", "61", "11", "rgb", "--transport", "gloo-host", "--json", "--check"] + extra
    r = subprocess.run(cmd, cwd=tmp_path, env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, text=True,
                       timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    assert meta["mismatches"] == 0 and meta["backend"] == "hip"
    filt = extra[extra.index("--filter") + 1] if "--filter" in extra else "gaussian"
    out = pconv_mod.read_raw(str(tmp_path / "blur_pic.raw"), 47, 61, "rgb")
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 11, filt))


def _slot_exchange_worker(rank, world, port, w, h, reps, halo, fuse, slots, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from pconv.parallel.bootstrap import init_distributed, shutdown
    from pconv.parallel.dist_engine import DistributedBlur

    ctx = init_distributed("gloo")
    try:
        blur = DistributedBlur(w, h, "rgb", "gaussian", reps, rank=rank, world=world, device=0, halo=halo, fuse=fuse,
                               slots=slots, transport="gloo-host", slot_exchange=True)
        assert blur.pipe.graphs and not blur.pipe.step_graphs
        blur.load_synthetic(5)
        ks = [blur.submit(reps) for _ in range(slots + 2)]
        blur.drain()
        q.put((rank, blur.band.y0, [blur.outputs[k].copy() for k in ks[-slots:]]))
    finally:
        shutdown(ctx)


@pytest.mark.parametrize("world,halo,fuse,reps,slots", [(2, 4, 4, 13, 2), (3, 6, 3, 19, 3), (4, 8, 8, 8, 2)])
def test_slot_exchange_pipeline_one_gpu(pconv_mod, world, halo, fuse, reps, slots):
    """Slot-stream pipeline that exchanges halos (one transport per slot, the
    exchange in stream order): every image of every band bit-exact."""
    w, h = 59, 83
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slot_exchange_worker, args=(r, world, port, w, h, reps, halo, fuse, slots, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    img = pconv_mod.synthetic_image(w, h, "rgb", seed=5)
    ref = pconv_mod.numpy_convolve(img, reps).reshape(h, -1)
    for rank, y0, outs in res:
        for o in outs:
            assert np.array_equal(o, ref[y0:y0 + o.shape[0]]), rank


@pytest.mark.parametrize("halo", ["preload", "event", "slot_exchange", "ipc"])
def test_bench_emulated_rank_halo_modes(halo):
    """`bench.py --emulate 8:3 --emulate-halo MODE`: one rank's step of the
    8-way split with its exchanges really issued (RCCL send/recv or IPC pulls
    to itself); with `event` also the resident MPI loop of its band through
    RCCL (resident_loop).  The pre-loaded proxy is oracle-checked."""
    import json
    import subprocess
    import sys

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--emulate", "8:3", "--emulate-halo", halo,
           "--steps", "10", "--warmup", "2"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["config"]["halo_mode"] == halo and d["ms_per_step"] > 0 and "8-way split" in d["emulated"]
    if halo == "preload":
        assert d["mismatches"] == 0
    if halo in ("event", "ipc"):
        rl = d["resident_loop" if halo == "event" else "resident_loop_ipc"]
        assert rl["transport"] == ("rccl" if halo == "event" else "ipc-grid"), rl
        assert rl["ms_per_image"] > 0 and rl["exchanges_per_image"] >= 1, rl
        assert rl["one_graph_per_image"] is True  # the exchange captured with the launches
        assert rl["ghost_bytes_per_exchange"] == [2 * rl["halo_rows"] * 1920 * 3], rl
    else:
        assert "resident_loop" not in d and "resident_loop_ipc" not in d
