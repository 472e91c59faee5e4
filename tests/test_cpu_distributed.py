"""Multi-process (torch.distributed gloo, world_size 2 and 3) run of the band
schedule with real point-to-point halo messages — CPU stand-in for RCCL."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, img, reps, halo, fuse, preload, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pconv.parallel.cpu_dist import CpuBandRunner

        h, w = img.shape[:2]
        ch = "grey" if img.ndim == 2 else "rgb"
        r = CpuBandRunner(w, h, ch, "gaussian", rank=rank, world=world, halo=halo, fuse=fuse)
        rows = img.reshape(h, -1)
        r.load(rows[r.band.y0 : r.band.y0 + r.band.rows])
        if preload:
            a = min(r.halo, r.band.y0)
            b = min(r.halo, h - (r.band.y0 + r.band.rows))
            if a:
                r._rows_view(r.frames[0], -a, 0)[:] = rows[r.band.y0 - a : r.band.y0]
            if b:
                e = r.band.y0 + r.band.rows
                r._rows_view(r.frames[0], r.band.rows, r.band.rows + b)[:] = rows[e : e + b]
        r.run(reps, halo_preloaded=preload)
        q.put((rank, r.band.y0, r.result(), r.exchanges))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,halo,fuse,preload", [(2, 1, 1, False), (2, 4, 2, True), (3, 5, 5, False)])
def test_gloo_bands_equal_serial(pconv_mod, world, halo, fuse, preload):
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, size=(29, 13, 3), dtype=np.uint8)
    reps = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, img, reps, halo, fuse, preload, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    out = np.concatenate([r[2] for r in res], axis=0).reshape(img.shape)
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps))
    assert all(r[3] >= (0 if preload else 1) for r in res)


def _torchrun(world, args, cwd, timeout=240):
    import subprocess
    import sys

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", "-m", "pconv.parallel.run"] + args
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    return subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("world,extra", [
    (1, []),
    (2, []),
    (3, ["--exchange-halo"]),
    (2, ["--filter", "box", "--halo", "2"]),
    (3, ["--filter", "edge", "--no-overlap", "--exchange-halo", "--halo", "1"]),
    (4, ["--backend", "cpu", "--fuse", "3", "--halo", "3"]),
])
def test_torchrun_per_rank_program(pconv_mod, tmp_path, world, extra):
    """`torch.distributed.run -m pconv.parallel.run` (the mpiexec analog): each
    rank reads its band (+ ghost rows), runs the schedule with gloo halos,
    pwrites its band; the file equals the oracle."""
    import json

    img = np.random.default_rng(world).integers(0, 256, size=(37, 29, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "pic.raw"), img)
    r = _torchrun(world, ["pic.raw", "29", "37", "7", "rgb", "--backend", "omp", "--json", "--check"] + extra,
                  tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    float(lines[-2])  # reference "%f" line
    meta = json.loads(lines[-1])
    assert meta["mismatches"] == 0 and meta["ranks"] == world
    filt = extra[extra.index("--filter") + 1] if "--filter" in extra else "gaussian"
    out = pconv_mod.read_raw(str(tmp_path / "blur_pic.raw"), 29, 37, "rgb")
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 7, filt))


def test_torchrun_usage_error(tmp_path):
    r = _torchrun(1, ["pic.raw", "29", "37", "7", "purple"], tmp_path)
    assert r.returncode != 0
    assert "Error Input!" in r.stderr


def test_parse_cpulist():
    from pconv.parallel.bootstrap import parse_cpulist

    assert parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert parse_cpulist("5") == {5}
    assert parse_cpulist("") == set()


def test_numa_bind_is_a_noop_without_a_gpu(pconv_mod):
    """No device (or enabled=False): binding changes nothing, raises nothing."""
    from pconv.parallel.bootstrap import bind_to_device_numa

    before = os.sched_getaffinity(0)
    assert bind_to_device_numa(0, enabled=False) is None
    assert bind_to_device_numa(0) is None  # this container has no GPU
    assert os.sched_getaffinity(0) == before


@pytest.mark.parametrize("world,extra", [(2, []), (3, ["--exchange-halo", "--backend", "cpu"])])
def test_torchrun_checkpoints(pconv_mod, tmp_path, world, extra):
    """--checkpoint-every K under torchrun: <out>.repK holds the whole image
    after K repetitions (every rank pwrites its band); resuming from a
    checkpoint with the remaining repetitions gives the final image."""
    img = np.random.default_rng(5).integers(0, 256, size=(41, 23, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "pic.raw"), img)
    r = _torchrun(world, ["pic.raw", "23", "41", "10", "rgb", "--backend", "omp", "--checkpoint-every", "4",
                          "--check", "--json"] + extra, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    for k in (4, 8):
        got = pconv_mod.read_raw(str(tmp_path / f"blur_pic.raw.rep{k}"), 23, 41, "rgb")
        assert np.array_equal(got, pconv_mod.numpy_convolve(img, k)), k
    assert not (tmp_path / "blur_pic.raw.rep12").exists()
    r = _torchrun(world, ["blur_pic.raw.rep8", "23", "41", "2", "rgb", "--backend", "omp", "--out", "resumed.raw"]
                  + extra, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert np.array_equal(pconv_mod.read_raw(str(tmp_path / "resumed.raw"), 23, 41, "rgb"),
                          pconv_mod.numpy_convolve(img, 10))


def test_preload_ghost_zone_covers_all_reps():
    """Pre-loaded ghost rows must carry every repetition (no exchange at all);
    bands shorter than `reps` fall back to the exchange cap."""
    from pconv.parallel.dist_engine import AUTO_HALO_CAP, auto_halo, preload_is_exchange_free

    assert auto_halo(8192, 8, 100, 8, preload=True) == 100
    assert auto_halo(32768, 8, 200, 8, preload=True) == 200
    assert auto_halo(32768, 8, 200, 8) == AUTO_HALO_CAP
    assert auto_halo(200, 4, 100, 8, preload=True) == 50
    assert preload_is_exchange_free(32768, 8, 200) and not preload_is_exchange_free(200, 4, 100)
    assert auto_halo(2520, 1, 40, 8, preload=True) == 8


def test_bench_metric_names():
    import importlib.util
    from types import SimpleNamespace

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a = SimpleNamespace(width=1920, height=2520, channels="rgb", reps=40, filter="gaussian")
    assert bench.metric_for(a) == bench.METRIC
    a = SimpleNamespace(width=8192, height=8192, channels="rgb", reps=100, filter="gaussian")
    assert bench.metric_for(a) == "Mpixels/sec (and wall-time) for 8192x8192 RGB, 100 reps at 1/2/4/8 MI355X"
    a = SimpleNamespace(width=1920, height=2520, channels="rgb", reps=40, filter="box")
    assert "box" in bench.metric_for(a) and bench.metric_for(a) != bench.METRIC


def test_bench_halo_mode_kwargs():
    """The N>1 pipelines bench.py times after the pre-loaded headline
    (slot_exchange, slot_exchange_direct, event, overlap, ipc) map to the
    intended DistributedBlur configurations and transports."""
    import importlib.util
    from types import SimpleNamespace

    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.HALO_MODES == ("slot_exchange", "slot_exchange_direct", "event", "overlap", "ipc")
    a = SimpleNamespace(slots=3, variant="auto", fuse=None, no_overlap=False, halo=None, concurrent="off")
    kw = {m: bench.mode_kwargs(a, m, 8) for m in bench.HALO_MODES}
    for m, k in kw.items():
        assert k["preload_halo"] is False, m  # every mode moves its ghost rows GPU-to-GPU
    assert kw["slot_exchange"]["slot_exchange"] and kw["slot_exchange"]["graph_capture"]
    assert kw["slot_exchange_direct"]["slot_exchange"] and not kw["slot_exchange_direct"]["graph_capture"]
    assert not kw["event"].get("slot_exchange") and kw["event"]["halo"] is None  # deep auto halo
    assert kw["overlap"]["halo"] == 8 and kw["overlap"]["overlap"]  # T-deep halo, split phases
    assert kw["ipc"]["slot_exchange"] and kw["ipc"]["graph_capture"]  # one captured graph per image
    assert bench.mode_transport("ipc", "rccl") == "ipc" and bench.mode_transport("event", "rccl") == "rccl"
    with pytest.raises(ValueError):
        bench.mode_kwargs(a, "nope", 8)


def test_omp_team_size_precedence():
    """--threads > a user's OMP_NUM_THREADS > bound CPUs > node budget / ranks;
    torchrun's injected OMP_NUM_THREADS=1 does not shrink the team."""
    from pconv.parallel.run import omp_team_size

    tr = {"TORCHELASTIC_RUN_ID": "x"}
    assert omp_team_size(5, {0, 1}, 16, 2, env=dict(tr, OMP_NUM_THREADS="3")) == 5
    assert omp_team_size(0, {0, 1}, 16, 2, env=dict(tr, OMP_NUM_THREADS="3")) == 3
    assert omp_team_size(0, {0, 1, 2}, 16, 2, env=dict(tr, OMP_NUM_THREADS="1")) == 3  # injected
    assert omp_team_size(0, None, 16, 4, env=dict(tr, OMP_NUM_THREADS="1")) == 4
    assert omp_team_size(0, None, 16, 1, env={"OMP_NUM_THREADS": "1"}) == 1  # a single process: the user's 1
    assert omp_team_size(0, None, 16, 2, env={"OMP_NUM_THREADS": "1"}) == 1  # not under torchrun: the user's
    assert omp_team_size(0, None, 16, 4, env={}) == 4
    assert omp_team_size(0, None, 2, 4, env={}) == 1


def test_import_leaves_omp_wait_policy_unset():
    """The passive wait policy is set only around the extension's import."""
    import subprocess
    import sys

    from conftest import ROOT

    code = f"import os, sys; sys.path.insert(0, {ROOT!r}); import pconv; print(os.environ.get('OMP_WAIT_POLICY'))"
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("OMP_WAIT_POLICY", "GOMP_SPINCOUNT")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "None"


def test_pcie_bytes_per_rank(pconv_mod):
    """h2d_bytes_per_step / d2h_bytes_per_step of the bench lines: band plus
    pre-loaded ghost rows in (clipped at the image edges), owned rows out;
    the 8-way headline's interior ranks upload 25 % more than their band."""
    from pconv.parallel.dist_engine import pcie_bytes_per_image

    n = pconv_mod.native
    rb = 1920 * 3
    tot_in = tot_out = 0
    for r in range(8):
        b = n.row_band(2520, 8, r)
        h2d, d2h = pcie_bytes_per_image(1920, 2520, "rgb", 8, r, 40, True)
        above, below = min(40, b.y0), min(40, 2520 - b.y0 - b.rows)
        assert (h2d, d2h) == ((b.rows + above + below) * rb, b.rows * rb)
        tot_in, tot_out = tot_in + h2d, tot_out + d2h
        assert pcie_bytes_per_image(1920, 2520, "rgb", 8, r, 40, False) == (b.rows * rb, b.rows * rb)
    assert tot_out == 2520 * rb
    assert pcie_bytes_per_image(1920, 2520, "rgb", 8, 3, 40, True)[0] == 395 * rb  # 315 + 2 x 40
    assert pcie_bytes_per_image(1920, 2520, "rgb", 1, 0, 40, True) == (2520 * rb, 2520 * rb)


def test_bench_policy_flags():
    """Pipeline policy is bench flags (echoed in the JSON config), not env vars."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_flags", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = bench.parse()
        assert (a.cu_mask_queues, a.head_on_slot_streams, a.ipc_pull, a.numa_bind) == (True, True, "grid", "on")
        assert a.stream_min_mb == 8.0 and a.stream_chunks == 4  # head streaming for images >= 8 MiB
        sys.argv = ["bench.py", "--pool-queues", "--head-pool-streams", "--ipc-pull", "sdma",
                    "--numa-bind", "off"]
        a = bench.parse()
    finally:
        sys.argv = old
    kw = bench.policy_kwargs(a)
    assert kw == dict(cu_mask_queues=False, head_on_slot_streams=False, head_alt_uploads=True, lazy_head=None,
                      ipc_pull="sdma")
    assert bench.mode_kwargs(a, "ipc", 8)["ipc_pull"] == "sdma"


def _floor_worker(rank, world, port, q):
    import importlib.util
    import sys
    import time

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec = importlib.util.spec_from_file_location("bench_floor", os.path.join(ROOT, "bench.py"))
        bench = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(bench)
        spans = []

        def run(n):  # a stand-in copy run: 0.2 s of "copying", returns ms per pair
            t0 = time.time()
            time.sleep(0.2)
            spans.append((t0, time.time(), n))
            return 200.0 + rank + (0.5 if len(spans) == 1 else 0.0)

        solo, conc = bench.copy_floors(run, world, rank)
        q.put((rank, solo, conc, spans))
    finally:
        dist.destroy_process_group()


def test_bench_copy_floors_solo_and_concurrent():
    """bench.py's copy floors at N > 1: every rank measures
    once ALONE (one rank at a time between barriers: no two solo spans
    overlap) and once with all ranks AT ONCE (the concurrent spans all
    overlap, one run long enough for the barrier skew not to matter); both
    come back as per-rank lists on every rank, the fields `pair_ms_solo` /
    `pair_ms_concurrent` of every N > 1 line."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_floor_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, solo, conc, spans in res:
        # solo: the better of two runs of 8; concurrent: one run, its own value
        assert solo == [200.0, 201.0, 202.0] and conc == [200.0, 201.0, 202.0]
        assert [s[2] for s in spans] == [8, 8, 8]  # >= 20 ms at a 202 ms "rate": the minimum 8
    solo_spans = sorted((r[3][0][0], r[3][1][1]) for r in res)
    for (a0, a1), (b0, b1) in zip(solo_spans, solo_spans[1:]):
        assert a1 <= b0, "solo floors overlapped"
    conc_spans = [r[3][2] for r in res]
    assert max(s[0] for s in conc_spans) < min(s[1] for s in conc_spans), "concurrent floors did not overlap"
