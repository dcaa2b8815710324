"""Build and run tests/abi/test_cpu_abi.cpp: the reference's CPU test program (tests/test_cpu.cpp: 7 tests)
written against this repository's C++ headers (cpu_rnnt.h, cpu_workspace_manager.h, rnnt_entrypoint.h), built
with plain g++ and linked against libmonotonic_rnnt_amd.so. Host only: runs without a GPU."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "monotonic-rnnt_amd")


def test_cpu_abi_program(tmp_path):
    exe = str(tmp_path / "test_cpu_abi")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "abi", "test_cpu_abi.cpp"), "-L", PKG, "-lmonotonic_rnnt_amd",
                    "-Wl,-rpath," + PKG, "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Tests pass" in r.stdout
