"""Resident service (`conv --serve` / `--server`): protocol, path handling
and results on the CPU backends (a `--device -1` server), plus the GPU
server under the gpu marker.  The server keeps the device context, engines,
pinned staging and tuned kernels between jobs; the client prints the
reference's timing lines with its own end-to-end clock."""
import json
import os
import socket
import struct
import subprocess
import time

import numpy as np
import pytest

from conftest import CONV_BIN


def _request(sock, *args):
    s = socket.socket(socket.AF_UNIX)
    s.connect(sock)
    msg = struct.pack("I", len(args))
    for a in args:
        b = a.encode()
        msg += struct.pack("I", len(b)) + b
    s.sendall(msg)
    n = struct.unpack("I", s.recv(4))[0]
    data = b""
    while len(data) < n:
        data += s.recv(n - len(data))
    s.close()
    return json.loads(data)


@pytest.fixture
def server(tmp_path, request):
    device = getattr(request, "param", -1)
    sock = str(tmp_path / "pconv.sock")
    p = subprocess.Popen([CONV_BIN, "--serve", sock, "--device", str(device), "--idle-timeout", "300"],
                         stderr=subprocess.PIPE, text=True)
    for _ in range(600):
        if os.path.exists(sock):
            break
        if p.poll() is not None:
            raise RuntimeError(p.stderr.read())
        time.sleep(0.05)
    yield sock
    try:
        _request(sock, "__shutdown__")
    finally:
        p.wait(timeout=60)


def test_service_cpu_jobs(pconv_mod, server, tmp_path, rng):
    img = rng.integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "in.raw"), img)
    for backend, reps in (("cpu", 3), ("omp", 7), ("cpu", 0)):
        r = subprocess.run([CONV_BIN, "in.raw", "53", "37", str(reps), "rgb", "--backend", backend, "--server",
                            server, "--json", "--check", "--format", "both"], cwd=tmp_path, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        lines = r.stdout.strip().splitlines()
        float(lines[0])
        assert lines[1].startswith("Execution time:")
        meta = json.loads(lines[2])
        assert meta["served"] and meta["mismatches"] == 0 and meta["client_e2e_s"] > 0
        # default output next to the input, resolved in the CLIENT's directory
        out = pconv_mod.read_raw(str(tmp_path / "blur_in.raw"), 53, 37, "rgb")
        assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps))
    assert _request(server, "__ping__")["jobs"] == 3


def test_service_errors_are_reported(server, tmp_path):
    r = subprocess.run([CONV_BIN, "missing.raw", "8", "8", "1", "grey", "--backend", "cpu", "--server", server],
                       cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "server:" in r.stderr
    r = subprocess.run([CONV_BIN, "x.raw", "8", "8", "1", "grey", "--synthetic", "1", "--server", server],
                       cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "no GPU" in r.stderr  # a --device -1 server runs the CPU backends only
    assert "error" in _request(server, "conv", "x.raw", "8")  # usage error comes back as JSON
    assert _request(server, "__ping__")["ok"]  # the server survives bad jobs


def test_client_without_server(tmp_path):
    r = subprocess.run([CONV_BIN, "x.raw", "8", "8", "1", "grey", "--synthetic", "1", "--server",
                        str(tmp_path / "none.sock")], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "conv --serve" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("server", [0], indirect=True)
def test_service_gpu_jobs_reuse_engines(pconv_mod, server, tmp_path, rng):
    """GPU jobs through one warm server: different geometries, repeated
    geometries (cached engine), checkpoints; every output exact."""
    jobs = [(61, 45, "rgb", 9), (200, 130, "grey", 40), (61, 45, "rgb", 13), (61, 45, "rgb", 9)]
    times = []
    for i, (w, h, ch, reps) in enumerate(jobs):
        c = 3 if ch == "rgb" else 1
        img = rng.integers(0, 256, size=(h, w, c) if c > 1 else (h, w), dtype=np.uint8)
        pconv_mod.write_raw(str(tmp_path / f"j{i}.raw"), img)
        r = subprocess.run([CONV_BIN, f"j{i}.raw", str(w), str(h), str(reps), ch, "--server", server, "--json",
                            "--check"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        meta = json.loads(r.stdout.strip().splitlines()[-1])
        assert meta["mismatches"] == 0 and "hip_init" not in meta["phases_s"]
        times.append(meta["client_e2e_s"])
        out = pconv_mod.read_raw(str(tmp_path / f"blur_j{i}.raw"), w, h, ch)
        assert np.array_equal(out, pconv_mod.numpy_convolve(img, reps))
    assert _request(server, "__ping__")["jobs"] == len(jobs)


def test_python_service_client(pconv_mod, tmp_path, rng):
    """pconv.utils.service: start a (CPU-only) server, run jobs through the
    Python client, errors raise ServiceError, shutdown stops the process."""
    from pconv.utils.service import ServiceClient, ServiceError, start_server

    sock = str(tmp_path / "py.sock")
    p = start_server(sock, device=-1, idle_timeout=120)
    try:
        c = ServiceClient(sock)
        img = rng.integers(0, 256, size=(29, 31), dtype=np.uint8)
        pconv_mod.write_raw(str(tmp_path / "g.raw"), img)
        meta = c.run(str(tmp_path / "g.raw"), 31, 29, 6, "grey", backend="omp", check=True)
        assert meta["mismatches"] == 0 and meta["output"].endswith("blur_g.raw")
        out = pconv_mod.read_raw(str(tmp_path / "blur_g.raw"), 31, 29, "grey")
        assert np.array_equal(out, pconv_mod.numpy_convolve(img, 6))
        meta = c.run("x.raw", 16, 16, 2, "rgb", out=str(tmp_path / "s.raw"), backend="cpu", synthetic=5)
        assert meta["mismatches"] == -1 and os.path.getsize(tmp_path / "s.raw") == 16 * 16 * 3
        with pytest.raises(ServiceError):
            c.run(str(tmp_path / "missing.raw"), 8, 8, 1, "grey", backend="cpu")
        assert c.ping()["jobs"] == 2
    finally:
        ServiceClient(sock).shutdown()
        p.wait(timeout=60)
    assert p.returncode == 0 and not os.path.exists(sock)


def test_service_pool_distributes_jobs(pconv_mod, tmp_path, rng):
    """ServicePool over two CPU-only servers: every job exact, all jobs served."""
    from pconv.utils.service import ServicePool

    pool = ServicePool.start([-1, -1], str(tmp_path / "pool"), idle_timeout=120)
    try:
        jobs, imgs = [], []
        for k in range(6):
            img = rng.integers(0, 256, size=(21, 17, 3), dtype=np.uint8)
            pconv_mod.write_raw(str(tmp_path / f"p{k}.raw"), img)
            imgs.append(img)
            jobs.append(dict(image=str(tmp_path / f"p{k}.raw"), width=17, height=21, reps=k + 1, channels="rgb",
                             backend="omp"))
        metas = pool.map(jobs)
        for k, (m, img) in enumerate(zip(metas, imgs)):
            out = pconv_mod.read_raw(m["output"], 17, 21, "rgb")
            assert np.array_equal(out, pconv_mod.numpy_convolve(img, k + 1)), k
        served = [c.ping()["jobs"] for c in pool.clients]
        assert sum(served) == 6
    finally:
        pool.close()


def test_serve_socket_path_safety(server, tmp_path):
    """`conv --serve PATH` never deletes a non-socket file at PATH, refuses a
    path a live server listens on, and replaces a dead server's socket."""
    regular = tmp_path / "not_a_socket"
    regular.write_text("keep me")
    r = subprocess.run([CONV_BIN, "--serve", str(regular), "--device", "-1"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "not a socket" in r.stderr
    assert regular.read_text() == "keep me"
    r = subprocess.run([CONV_BIN, "--serve", server, "--device", "-1"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "already listening" in r.stderr
    assert _request(server, "__ping__")["ok"]  # the live server is untouched
    stale = str(tmp_path / "stale.sock")
    s = socket.socket(socket.AF_UNIX)
    s.bind(stale)
    s.close()  # a socket file nobody listens on
    p = subprocess.Popen([CONV_BIN, "--serve", stale, "--device", "-1", "--idle-timeout", "60"],
                         stderr=subprocess.PIPE, text=True)
    try:
        for _ in range(600):
            try:
                if _request(stale, "__ping__")["ok"]:
                    break
            except OSError:
                time.sleep(0.05)
        assert _request(stale, "__shutdown__")["ok"]
    finally:
        p.wait(timeout=60)
    assert not os.path.exists(stale)
