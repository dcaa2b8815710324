"""The GPU library's host orchestration under AddressSanitizer / UBSan (mrnnt_capi.cpp plans the
workspace and carves caller buffers with pointer arithmetic). `make asan-gpu` (an opt-in target that
__graft_entry__.build() also runs; the product build does not need clang's ASan runtime) compiles
mrnnt_capi.cpp with every -fsanitize behind -Xarch_host -- host code only, the kernels are the product's objects --
into libmonotonic_rnnt_amd_hostasan.so. The reference's 7 GPU tests in C++ (tests/abi/test_gpu_abi.cpp: the managers,
compute_rnnt_loss, the computer's getters) are linked against it, host code sanitized too, with clang's shared ASan
runtime linked first (no preload), and must pass with no sanitizer report.
"""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "monotonic-rnnt_amd")
LIB = os.path.join(PKG, "libmonotonic_rnnt_amd_hostasan.so")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-shared-libasan"]


def _runtime_dir():
    for pat in ("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so",
                "/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"):
        hits = sorted(glob.glob(pat))
        if hits:
            return os.path.dirname(hits[-1])
    return None


def _build(out):
    rt = _runtime_dir()
    if rt is None:
        pytest.skip("clang's ASan runtime (libclang_rt.asan-x86_64.so) not found under /opt/rocm")
    if not os.path.exists(LIB):
        pytest.skip("libmonotonic_rnnt_amd_hostasan.so not built (make -C monotonic-rnnt_amd asan-gpu)")
    cmd = (["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-g", "-std=c++17"] + SAN +
           ["-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "abi", "test_gpu_abi.cpp"),
            "-L", PKG, "-lmonotonic_rnnt_amd_hostasan", "-Wl,-rpath," + PKG, "-Wl,-rpath," + rt, "-o", out])
    subprocess.run(cmd, check=True)


def test_host_asan_abi_program_builds(tmp_path):
    _build(str(tmp_path / "test_gpu_abi_hostasan"))


@pytest.mark.gpu
def test_host_orchestration_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "test_gpu_abi_hostasan")
    _build(exe)
    env = dict(os.environ)
    # the ROCm runtime maps GPU memory where ASan's shadow gap would be; leaks of the process-lifetime runtime
    # objects are not this library's
    env["ASAN_OPTIONS"] = "detect_leaks=0:protect_shadow_gap=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "Tests pass" in r.stdout, out[-4000:]
