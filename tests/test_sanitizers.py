"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "race detection /
sanitizers"). `make -C monotonic-rnnt_amd asan` builds, with g++ and no GPU, the CPU implementation (mrnnt_cpu.cpp:
RNNT_CPU, cpu_monotonic_rnnt*, CpuRNNTWorkspaceManager / CpuRNNTComputer) and the host-only C ABI (mrnnt_entry.cpp:
error state, host lattice builder, compute_rnnt_loss) into build/asan/libmrnnt_host_asan.so, and the reference's CPU
test program against it. Then:

* tests/abi/test_cpu_abi.cpp (test_cpu.cpp's 7 cases through compute_rnnt_loss(RNNT_CPU)) runs under ASan with leak
  detection on;
* the CPU parity tests (every golden fixture, the oracle on random / alignment / padded cases, the reference's
  pytorch_binding/test.py assertions) and the reference-API C++ client (tests/abi/ref_client.cpp, built with the
  sanitizers too) run through the sanitized library (MRNNT_LIB_PATH, the runtimes preloaded into Python): numpy
  buffers come from the intercepted malloc, so a write past a caller's costs / grads / workspace is reported.

Any sanitizer report aborts the run (UBSan halt_on_error). Found and fixed when this was added: an out-of-range
`RNNTOptions.loc` read through the enum type (mrnnt_entry.cpp) and signed overflow / a negative left shift in the fp32
exp's exponent assembly on NaN input (mrnnt_cpu.cpp vexp)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "monotonic-rnnt_amd")
ASAN = os.path.join(PKG, "build", "asan")
SAN = "-fsanitize=address,undefined"


def _runtime(name):
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def asan_build():
    if not (_runtime("libasan.so") and _runtime("libubsan.so")):
        pytest.skip("g++ sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", PKG, "asan"], check=True, timeout=900)
    return os.path.join(ASAN, "libmrnnt_host_asan.so")


def _env(**extra):
    env = dict(os.environ)
    env.update(ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=87", **extra)
    return env


def test_reference_cpu_program_under_asan(asan_build):
    env = _env()
    env["ASAN_OPTIONS"] = "detect_leaks=1:exitcode=86"  # a standalone program: leaks count too
    r = subprocess.run([os.path.join(ASAN, "test_cpu_abi")], capture_output=True, text=True, timeout=300, env=env,
                       cwd="/tmp")
    assert r.returncode == 0 and "Tests pass" in r.stdout, r.stdout + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]


def test_cpu_parity_suite_under_asan(asan_build):
    # the sanitizer runtimes first in the initial library list; whatever the environment already preloads stays
    pre = ":".join([_runtime("libasan.so"), _runtime("libubsan.so")] + list(filter(None, [os.environ.get("LD_PRELOAD")])))
    env = _env(LD_PRELOAD=pre, MRNNT_LIB_PATH=asan_build, MRNNT_SAN_FLAGS=SAN)
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
           "-k", "not gpu_reference_client_builds",
           os.path.join(ROOT, "tests", "test_cpu_parity.py"), os.path.join(ROOT, "tests", "test_ref_client.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1200, env=env, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-6000:]
    assert " passed" in r.stdout and " failed" not in r.stdout, r.stdout[-2000:]
