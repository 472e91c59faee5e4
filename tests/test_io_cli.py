"""Raw image I/O and the reference-compatible CLI (CPU backends)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import CONV_BIN


def test_output_naming(pconv_mod):
    assert pconv_mod.output_path_for("x.raw") == "blur_x.raw"
    assert pconv_mod.output_path_for("dir/sub/x.raw") == "dir/sub/blur_x.raw"
    assert pconv_mod.native.output_path_for("dir/x.raw") == "dir/blur_x.raw"


def test_raw_roundtrip_and_truncate(pconv_mod, tmp_path, rng):
    img = rng.integers(0, 256, size=(9, 7, 3), dtype=np.uint8)
    p = str(tmp_path / "a.raw")
    with open(p, "wb") as f:
        f.write(b"\xff" * 10_000)  # stale, longer file: must be truncated
    pconv_mod.write_raw(p, img)
    assert os.path.getsize(p) == img.size
    back = pconv_mod.read_raw(p, 7, 9, "rgb")
    assert np.array_equal(back, img)


def test_short_file_is_an_error(pconv_mod, tmp_path):
    p = str(tmp_path / "short.raw")
    with open(p, "wb") as f:
        f.write(b"\0" * 10)
    with pytest.raises(RuntimeError, match="needs"):
        pconv_mod.read_raw(p, 4, 4, "grey")


def test_synthetic_bands_consistent(pconv_mod):
    full = pconv_mod.synthetic_image(33, 17, "rgb", seed=5)
    part = pconv_mod.synthetic_image(33, 17, "rgb", seed=5, y0=6, rows=5)
    assert np.array_equal(full[6:11], part)
    assert not np.array_equal(full, pconv_mod.synthetic_image(33, 17, "rgb", seed=6))
    hist = np.bincount(pconv_mod.synthetic_image(256, 256, "grey", seed=1).reshape(-1), minlength=256)
    assert hist.min() > 0.5 * hist.mean()


def _run(args, cwd):
    return subprocess.run([CONV_BIN] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_cli_usage_contract(tmp_path):
    r = _run([], tmp_path)
    assert r.returncode == 1 and "Error Input!" in r.stderr and "image_name width height repetitions [rgb/grey]" in r.stderr
    r = _run(["a.raw", "4", "4", "1", "cmyk"], tmp_path)
    assert r.returncode == 1 and "Error Input!" in r.stderr
    r = _run(["a.raw", "4x", "4", "1", "grey"], tmp_path)
    assert r.returncode == 1 and "invalid width" in r.stderr
    r = _run(["a.raw", "4", "4", "-1", "grey"], tmp_path)
    assert r.returncode == 1 and "repetitions" in r.stderr
    r = _run(["missing.raw", "4", "4", "1", "grey", "--backend", "cpu"], tmp_path)
    assert r.returncode == 1 and "cannot open missing.raw" in r.stderr
    r = _run(["--help"], tmp_path)
    assert r.returncode == 0 and "--gpus" in r.stdout


@pytest.mark.parametrize("backend", ["cpu", "omp"])
@pytest.mark.parametrize("typ", ["grey", "rgb"])
def test_cli_cpu_end_to_end(pconv_mod, tmp_path, rng, backend, typ):
    c = 1 if typ == "grey" else 3
    img = rng.integers(0, 256, size=(21, 13, c) if c > 1 else (21, 13), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "img.raw"), img)
    r = _run(["img.raw", "13", "21", "6", typ, "--backend", backend, "--json", "--check"], tmp_path)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    float(lines[0])  # MPI-style "%f" loop time
    meta = json.loads(lines[-1])
    assert meta["mismatches"] == 0 and meta["reps"] == 6
    out = pconv_mod.read_raw(str(tmp_path / "blur_img.raw"), 13, 21, typ)
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 6))


def test_cli_checkpoint_resume(pconv_mod, tmp_path, rng):
    img = rng.integers(0, 256, size=(16, 16), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "i.raw"), img)
    r = _run(["i.raw", "16", "16", "10", "grey", "--backend", "cpu", "--checkpoint-every", "4"], tmp_path)
    assert r.returncode == 0, r.stderr
    ck = pconv_mod.read_raw(str(tmp_path / "blur_i.raw.rep8"), 16, 16, "grey")
    assert np.array_equal(ck, pconv_mod.numpy_convolve(img, 8))
    # resume: the iteration is Markov in the image -> 2 more reps from the checkpoint
    r = _run(["blur_i.raw.rep8", "16", "16", "2", "grey", "--backend", "cpu", "--out", "resumed.raw"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(pconv_mod.read_raw(str(tmp_path / "resumed.raw"), 16, 16, "grey"),
                          pconv_mod.read_raw(str(tmp_path / "blur_i.raw"), 16, 16, "grey"))


def test_cli_synthetic_and_filters(pconv_mod, tmp_path):
    for f in ("gaussian", "box", "edge"):
        r = _run(["s.raw", "40", "30", "3", "rgb", "--synthetic", "9", "--backend", "omp", "--filter", f, "--check",
                  "--quiet"], tmp_path)
        assert r.returncode == 0, r.stderr
        out = pconv_mod.read_raw(str(tmp_path / "blur_s.raw"), 40, 30, "rgb")
        ref = pconv_mod.numpy_convolve(pconv_mod.synthetic_image(40, 30, "rgb", seed=9), 3, f)
        assert np.array_equal(out, ref)


def test_python_module_cli(tmp_path, pconv_mod):
    import sys

    from conftest import ROOT

    r = subprocess.run([sys.executable, "-m", "pconv", "s.raw", "8", "8", "2", "grey", "--synthetic", "1",
                        "--backend", "cpu", "--format", "both"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr
    assert "Execution time:" in r.stdout


def test_cli_bench_flags(tmp_path):
    """`conv --bench K` (bench.py's serving step on the native stack) flags are
    validated like every other option; --help documents them."""
    r = _run(["a.raw", "64", "64", "4", "rgb", "--synthetic", "1", "--bench", "0"], tmp_path)
    assert r.returncode == 1 and "invalid --bench" in r.stderr
    r = _run(["a.raw", "64", "64", "4", "rgb", "--synthetic", "1", "--bench", "5", "--slots", "9"], tmp_path)
    assert r.returncode == 1 and "invalid --slots" in r.stderr
    r = _run(["a.raw", "64", "64", "4", "rgb", "--bench", "5", "--stream-chunks", "x"], tmp_path)
    assert r.returncode == 1 and "invalid --stream-chunks" in r.stderr
    r = _run(["--help"], tmp_path)
    assert "--bench K" in r.stdout and "--stream-chunks" in r.stdout


@pytest.mark.parametrize("typ", ["grey", "rgb"])
def test_cli_auto_backend_small_job_stays_on_cpu(pconv_mod, tmp_path, rng, typ):
    """`--backend auto`: a job whose CPU time (priced from its first, timed
    repetition) is below the GPU's start-up never touches the GPU; the output
    is the oracle's and the JSON says where every repetition ran."""
    c = 1 if typ == "grey" else 3
    img = rng.integers(0, 256, size=(37, 29, c) if c > 1 else (37, 29), dtype=np.uint8)
    pconv_mod.write_raw(str(tmp_path / "img.raw"), img)
    r = _run(["img.raw", "29", "37", "7", typ, "--backend", "auto", "--json", "--check"], tmp_path)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert lines[0].startswith("Execution time:")  # the one-shot (CUDA-style) line
    meta = json.loads(lines[-1])
    assert meta["backend"] == "auto" and meta["gpus"] == 0
    assert meta["cpu_reps"] == 7 and meta["gpu_reps"] == 0 and meta["mismatches"] == 0
    assert meta["auto_choice"].startswith("cpu only")
    out = pconv_mod.read_raw(str(tmp_path / "blur_img.raw"), 29, 37, typ)
    assert np.array_equal(out, pconv_mod.numpy_convolve(img, 7))


def test_cli_auto_backend_without_gpu_falls_back(pconv_mod, tmp_path):
    """Forced GPU choice (--auto-gpu-min 0) on a machine whose GPU cannot come
    up: the job finishes on the CPU, bit-exact, and says why."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")
    r = subprocess.run([CONV_BIN, "s.raw", "48", "40", "9", "rgb", "--synthetic", "5", "--backend", "auto", "--json",
                        "--check", "--quiet", "--auto-gpu-min", "0"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    meta = json.loads(r.stdout.strip().splitlines()[-1])
    assert meta["cpu_reps"] == 9 and meta["gpu_reps"] == 0 and meta["mismatches"] == 0 and meta["gpus"] == 0
    assert "failed" in meta["auto_choice"], meta["auto_choice"]
    out = pconv_mod.read_raw(str(tmp_path / "blur_s.raw"), 48, 40, "rgb")
    assert np.array_equal(out, pconv_mod.numpy_convolve(pconv_mod.synthetic_image(48, 40, "rgb", seed=5), 9))
