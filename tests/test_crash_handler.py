"""Native crash reporter (selftest.cpp install_crash_handler) on the CPU:
PCONV_CRASH_LOG is opened only when a fatal signal arrives, so processes
that exit normally leave no empty log file behind (VERDICT r03 hygiene)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = """
import os, signal, sys
sys.path.insert(0, {root!r})
import pconv
pconv.native.install_crash_handler()
if sys.argv[1] == "crash":
    os.kill(os.getpid(), signal.SIGSEGV)
"""


def _run(tmp_path, mode):
    log = tmp_path / "crash.log"
    env = dict(os.environ, PCONV_CRASH_LOG=str(log))
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT), mode], env=env, capture_output=True,
                       text=True, timeout=300)
    return r, log


def test_no_log_file_without_a_crash(tmp_path):
    r, log = _run(tmp_path, "ok")
    assert r.returncode == 0, r.stderr
    assert not log.exists()


def test_log_written_on_fatal_signal(tmp_path):
    r, log = _run(tmp_path, "crash")
    assert r.returncode != 0
    assert log.exists()
    text = log.read_text()
    assert "fatal signal 11 (Segmentation fault)" in text and "native backtrace" in text
