"""Python client of the resident convolution service (``conv --serve``).

The server (``csrc/src/service.cpp``) keeps one GPU context, cached engines,
pinned staging and tuned kernels between jobs; a job is a ``conv`` argv.
This module speaks its wire format (u32 argc, then u32 length + bytes per
argument; reply u32 length + JSON) and starts servers for scripts and tests:

    from pconv.utils.service import start_server, ServiceClient
    srv = start_server("/tmp/pconv.sock", device=0)
    c = ServiceClient("/tmp/pconv.sock")
    meta = c.run("image.raw", 1920, 2520, 40, "rgb")   # -> blur_image.raw, report dict
    c.shutdown(); srv.wait()

The reference has no service: its CUDA program pays context creation in
every run (``cuda/main.c:20-49``).
"""
from __future__ import annotations

import json
import os
import socket
import struct
import subprocess
import time
from typing import Dict, List, Optional

from .._native import conv_binary


class ServiceError(RuntimeError):
    pass


class ServiceClient:
    def __init__(self, socket_path: str, timeout: float = 600.0):
        self.socket_path = socket_path
        self.timeout = float(timeout)

    def request(self, *args: str) -> Dict:
        """Send one argv (args[0] is the program name or a control word)."""
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(self.timeout)
        try:
            s.connect(self.socket_path)
            msg = [struct.pack("I", len(args))]
            for a in args:
                b = str(a).encode()
                msg.append(struct.pack("I", len(b)) + b)
            s.sendall(b"".join(msg))
            n = struct.unpack("I", _recv_exact(s, 4))[0]
            return json.loads(_recv_exact(s, n))
        finally:
            s.close()

    def ping(self) -> Dict:
        return self.request("__ping__")

    def shutdown(self) -> Dict:
        return self.request("__shutdown__")

    def run(self, image: str, width: int, height: int, reps: int, channels: str = "grey",
            out: Optional[str] = None, **flags) -> Dict:
        """One job with the CLI's contract; keyword flags map to `--flag value`
        (`check=True` -> `--check`).  Paths are resolved here, as the server's
        working directory is its own.  Raises ServiceError on a failed job."""
        synthetic = flags.get("synthetic") is not None
        argv: List[str] = ["conv", image if synthetic else os.path.abspath(image), str(width), str(height),
                           str(reps), channels]
        from .raw_io import output_path_for

        argv += ["--out", os.path.abspath(out if out is not None else output_path_for(image))]
        for k, v in flags.items():
            if v is None or v is False:
                continue
            argv.append("--" + k.replace("_", "-"))
            if v is not True:
                argv.append(str(v))
        argv.append("--json")
        meta = self.request(*argv)
        if "error" in meta:
            raise ServiceError(meta["error"])
        return meta


def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = b""
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            raise ServiceError("server closed the connection")
        buf += chunk
    return buf


def _drain_stderr(p: subprocess.Popen, keep: int = 40) -> List[str]:
    """Read the server's stderr on a daemon thread for as long as it runs
    (served jobs may write to it: --explain plans, reply errors, HIP runtime
    logs), so a full 64 KiB pipe can never block the server in a write and
    hang every client.  The first `keep` lines are kept for error messages."""
    import threading

    head: List[str] = []

    def pump():
        for line in p.stderr:
            if len(head) < keep:
                head.append(line)

    t = threading.Thread(target=pump, name="pconv-serve-stderr", daemon=True)
    t.start()
    p._pconv_stderr_thread = t  # type: ignore[attr-defined]
    return head


def start_server(socket_path: str, device: int = 0, idle_timeout: float = 0.0, max_engines: int = 8,
                 wait_s: float = 120.0) -> subprocess.Popen:
    """Start `conv --serve` as a child process and wait until it listens
    (device -1: a CPU-only server for the cpu / omp backends).  The server
    replaces a leftover socket of a dead server and refuses any other file
    or a live server at that path."""
    p = subprocess.Popen([conv_binary(), "--serve", socket_path, "--device", str(device), "--idle-timeout",
                          str(idle_timeout), "--max-engines", str(max_engines)], stderr=subprocess.PIPE, text=True)
    err_head = _drain_stderr(p)
    t0 = time.time()
    while time.time() - t0 < wait_s:
        if os.path.exists(socket_path):
            try:
                ServiceClient(socket_path, timeout=10).ping()
                return p
            except (OSError, ServiceError):
                pass
        if p.poll() is not None:
            p._pconv_stderr_thread.join(timeout=5)  # type: ignore[attr-defined]
            raise ServiceError(f"server exited: {''.join(err_head)}")
        time.sleep(0.05)
    p.kill()
    raise ServiceError("server did not start listening")


class ServicePool:
    """Data-parallel serving over several resident servers (one per GPU):
    independent images go to the servers round-robin by availability, each
    job whole on one GPU — no halos, so N servers give N x the image
    throughput of one (the row-band decomposition instead splits ONE image
    over N GPUs, trading halo work for latency; docs/ARCHITECTURE.md §5).

        pool = ServicePool.start(8, "/tmp/pconv")      # /tmp/pconv.0.sock ... .7.sock
        metas = pool.map([dict(image=p, width=1920, height=2520, reps=40, channels="rgb") for p in paths])
        pool.close()
    """

    def __init__(self, sockets: List[str], procs: Optional[List[subprocess.Popen]] = None, timeout: float = 600.0):
        if not sockets:
            raise ValueError("ServicePool needs at least one server socket")
        self.clients = [ServiceClient(s, timeout) for s in sockets]
        self.procs = list(procs or [])

    @classmethod
    def start(cls, devices, prefix: str, idle_timeout: float = 0.0) -> "ServicePool":
        """Start one server per device (an int n means devices 0..n-1)."""
        devs = list(range(devices)) if isinstance(devices, int) else list(devices)
        socks = [f"{prefix}.{i}.sock" for i in range(len(devs))]
        procs = []
        try:
            for d, s in zip(devs, socks):
                procs.append(start_server(s, device=d, idle_timeout=idle_timeout))
        except Exception:
            for p in procs:
                p.kill()
            raise
        return cls(socks, procs)

    def map(self, jobs: List[Dict]) -> List[Dict]:
        """Run every job (ServiceClient.run keyword arguments); results in job
        order.  Each server runs one job at a time; a free server takes the
        next job.  The first failing job's ServiceError is raised after all
        jobs finish."""
        import queue
        import threading

        todo: "queue.Queue" = queue.Queue()
        for i, j in enumerate(jobs):
            todo.put((i, j))
        out: List[Optional[Dict]] = [None] * len(jobs)
        errs: List[BaseException] = []

        def worker(c: ServiceClient):
            while True:
                try:
                    i, j = todo.get_nowait()
                except queue.Empty:
                    return
                try:
                    out[i] = c.run(**j)
                except BaseException as e:  # reported after the pool drains
                    errs.append(e)

        ts = [threading.Thread(target=worker, args=(c,)) for c in self.clients]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        return out  # type: ignore[return-value]

    def close(self) -> None:
        for c in self.clients:
            try:
                c.shutdown()
            except (OSError, ServiceError):
                pass
        for p in self.procs:
            p.wait(timeout=60)
