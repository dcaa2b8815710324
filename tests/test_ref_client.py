"""Reference C++ clients against this library: the reference's own manager / computer API, as
its driver code uses it, compiled against include/ and linked against libmonotonic_rnnt_amd.so.

* tests/abi/ref_client.cpp -- the body of oracle/ref_driver.cpp (reference-API client code: the reference's
  CpuRNNTWorkspaceManager / CpuRNNTComputer lifecycle plus get_denom / get_alpha / get_beta per row), built with
  plain g++. Its costs, gradients, denominators and alpha / beta match the golden vectors that the reference itself
  produced (tests/golden, from cpu_rnnt.h<double>); plus every other public accessor of the reference's CPU
  manager (cpu_workspace_manager.h:63-205). Host only.
* tests/abi/gpu_ref_client.cpp -- GpuRNNTWorkspaceManager / GpuRNNTComputer plus every public host getter of the
  reference's GPU manager (gpu_workspace_manager.h:87-190) after cost_and_grad, against the same golden vectors.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from _parity import FIXTURES, assert_costs, assert_grads, assert_state

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "monotonic-rnnt_amd")
INC = os.path.join(ROOT, "include")
IDS = [os.path.basename(p)[:-4] for p in FIXTURES]


def _build(src, out, compiler):
    lib = os.environ.get("MRNNT_LIB_PATH")  # the host-only sanitizer build (tests/test_sanitizers.py)
    link = ([lib, "-Wl,-rpath," + os.path.dirname(lib)] + os.environ.get("MRNNT_SAN_FLAGS", "").split() if lib else
            ["-L", PKG, "-lmonotonic_rnnt_amd", "-Wl,-rpath," + PKG])
    cmd = [compiler, "-O2", "-std=c++17", "-fPIC", "-shared", "-I", INC, os.path.join(ROOT, "tests", "abi", src)] + \
        link + ["-o", out]
    if compiler.endswith("hipcc"):
        cmd.insert(1, "--offload-arch=gfx950")
    subprocess.run(cmd, check=True)
    return ctypes.CDLL(out)


@pytest.fixture(scope="module")
def cpu_client(tmp_path_factory):
    lib = _build("ref_client.cpp", str(tmp_path_factory.mktemp("refc") / "libref_client.so"), "g++")
    lib.client_rnnt_f32.restype = ctypes.c_int
    lib.client_accessors.restype = ctypes.c_int
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _tight(fx):
    """The reference's label row stride is max(S) (cpu_workspace_manager.h:44): hand it tight labels."""
    S = fx["S"]
    smax = int(S.max())
    lab = np.ascontiguousarray(fx["labels"][:, :smax]).astype(np.int32) if smax else np.zeros((len(S), 1), np.int32)
    al = fx.get("alignment")
    if al is not None:
        al = np.ascontiguousarray(al[:, :int(fx["T"].max())]).astype(np.int32)
    return lab, al


@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_reference_driver_compiles_and_matches_golden(cpu_client, path):
    fx = dict(np.load(path))
    lab, al = _tight(fx)
    acts = np.ascontiguousarray(fx["acts"], np.float32)
    N, V = acts.shape
    B = len(fx["T"])
    T = np.ascontiguousarray(fx["T"], np.int32)
    S = np.ascontiguousarray(fx["S"], np.int32)
    costs = np.zeros(B, np.float32)
    grads = np.zeros((N, V), np.float32)
    den, alpha, beta = (np.zeros(N, np.float32) for _ in range(3))
    rc = cpu_client.client_rnnt_f32(_p(acts), _p(lab), B, _p(T), _p(S), V, int(fx["blank"]), _p(al),
                                    int(fx.get("max_shift", 0)), int(fx["blank"]), _p(costs), _p(grads), _p(den),
                                    _p(alpha), _p(beta), 0)
    assert rc == 0
    assert_costs(costs, fx["costs_f64"])
    assert_grads(grads, fx["grads_f64"])
    # every row's denominator (get_denom reduces the rows the computation never read on first access), alpha / beta
    # with the reference's -inf outside the band; fp32 read-outs of fp64 state
    assert_state(den, alpha.astype(np.float64), beta.astype(np.float64), fx, window=np.ones(N, bool), rel=1e-4,
                 den_rel=1e-5)


@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_reference_cpu_manager_accessors(cpu_client, path):
    fx = dict(np.load(path))
    lab, al = _tight(fx)
    acts = np.ascontiguousarray(fx["acts"], np.float32)
    T = np.ascontiguousarray(fx["T"], np.int32)
    S = np.ascontiguousarray(fx["S"], np.int32)
    bad = cpu_client.client_accessors(_p(acts), _p(lab), len(T), _p(T), _p(S), acts.shape[1], int(fx["blank"]),
                                      _p(al), int(fx.get("max_shift", 0)))
    assert bad == 0


def test_gpu_reference_client_builds(tmp_path):
    _build("gpu_ref_client.cpp", str(tmp_path / "libgpu_ref_client.so"), "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def gpu_client(tmp_path_factory):
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    return _build("gpu_ref_client.cpp", str(tmp_path_factory.mktemp("gref") / "libgpu_ref_client.so"),
                  "/opt/rocm/bin/hipcc")


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_gpu_manager_getters_match_golden(gpu_client, path):
    lib = gpu_client
    fx = dict(np.load(path))
    lab, al = _tight(fx)
    acts = np.ascontiguousarray(fx["acts"], np.float32)
    N, V = acts.shape
    T = np.ascontiguousarray(fx["T"], np.int32)
    S = np.ascontiguousarray(fx["S"], np.int32)
    B, Tm = len(T), int(T.max())
    costs = np.zeros(B, np.float32)
    grads = np.zeros((N, V), np.float32)
    den, alpha, beta = (np.zeros(N, np.float32) for _ in range(3))
    llf, llb = np.zeros(B, np.float32), np.zeros(B, np.float32)
    mn, mx = np.zeros(B * Tm, np.int32), np.zeros(B * Tm, np.int32)
    voff = np.zeros(B, np.int32)
    sizes = np.zeros(4, np.int32)
    back = np.zeros((N, V), np.float32)
    k = int(fx.get("max_shift", 0))
    bad = lib.client_gpu_getters(_p(acts), _p(lab), B, _p(T), _p(S), V, int(fx["blank"]), _p(al), k, _p(costs),
                                 _p(grads), _p(den), _p(alpha), _p(beta), _p(llf), _p(llb), _p(mn), _p(mx), _p(voff),
                                 _p(sizes), _p(back))
    assert bad == 0
    assert_costs(costs, fx["costs_f64"])
    assert_grads(grads, fx["grads_f64"])
    assert_state(den, alpha.astype(np.float64), beta.astype(np.float64), fx, window=np.ones(N, bool), rel=1e-4,
                 den_rel=1e-5)
    rows = T.astype(np.int64) * (S + 1)
    np.testing.assert_array_equal(voff, np.concatenate([[0], np.cumsum(rows)[:-1]]))
    np.testing.assert_array_equal(sizes, [N, N, int(S.max()), Tm])
    np.testing.assert_array_equal(back, acts)
    # ll_forward = alpha(T-1, S) = -cost, ll_backward = beta(0, 0) (the reference's debug check, cpu_rnnt.h:257-259)
    fin = np.isfinite(fx["costs_f64"])
    np.testing.assert_allclose(-llf[fin], fx["costs_f64"][fin], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(llb[fin], llf[fin], rtol=1e-5, atol=1e-4)
    # the band in the reference's [B, max T] layout (gpu_workspace_manager.h:191-219, initial values :317-328)
    emn, emx = np.zeros((B, Tm), np.int32), np.repeat(S[:, None], Tm, 1).astype(np.int32)
    if al is not None:
        for b in range(B):
            m = np.concatenate([[0], np.cumsum(al[b, :T[b]] != int(fx["blank"]))])
            for t in range(T[b]):
                emn[b, t] = m[max(0, t + 1 - k)]
                emx[b, t] = m[min(T[b], t + 1 + k)]
    np.testing.assert_array_equal(mn.reshape(B, Tm), emn)
    np.testing.assert_array_equal(mx.reshape(B, Tm), emx)


@pytest.mark.gpu
def test_gpu_manager_band_members_are_output_only(gpu_client):
    """the band members are an output of the last computation, not an input (include/
    gpu_workspace_manager.h). A band written into them before cost() is ignored -- the costs equal a
    plain call's -- and the members hold [0, S_b] afterwards."""
    fx = dict(np.load(next(p for p in FIXTURES if os.path.basename(p) == "multibatch.npz")))
    lab, _ = _tight(fx)
    acts = np.ascontiguousarray(fx["acts"], np.float32)
    T = np.ascontiguousarray(fx["T"], np.int32)
    S = np.ascontiguousarray(fx["S"], np.int32)
    assert S.max() > 0
    bad = gpu_client.client_band_members_output_only(_p(acts), _p(lab), len(T), _p(T), _p(S), acts.shape[1],
                                                     int(fx["blank"]))
    assert bad == 0
