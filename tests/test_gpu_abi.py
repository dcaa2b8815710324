"""Build and run tests/abi/test_gpu_abi.cpp: the reference's 7 GPU tests (tests/test_gpu.cu) written
against this repository's C++ headers and linked against libmonotonic_rnnt_amd.so."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "monotonic-rnnt_amd")


def _build(out):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "abi", "test_gpu_abi.cpp"), "-L", PKG, "-lmonotonic_rnnt_amd",
           "-Wl,-rpath," + PKG, "-o", out]
    subprocess.run(cmd, check=True)


def test_abi_program_builds(tmp_path):
    _build(str(tmp_path / "test_gpu_abi"))


@pytest.mark.gpu
def test_abi_program_runs(tmp_path):
    exe = str(tmp_path / "test_gpu_abi")
    _build(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Tests pass" in r.stdout
