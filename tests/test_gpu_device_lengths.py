"""Device-resident lengths (ABI v7 lengths_on_device): the reference's GPU binding requires the
lengths on the device (pytorch_binding/monotonic_rnnt.cu:85-88) and its op passes them through (monotonic_rnnt_op.py:
39-50). Here they are never read back: the launch is planned from acts.size(0) and labels.size(1), the lattice is
built and validated on the device, and a failed validation makes the call's costs and gradients NaN and is
reported by the next call / check_lengths().

* bit-identical to the host-lengths path on every kernel family (packed f32 / bf16 / scalar-V, padded, alignment, a
  batch with more columns than the log-softmax's work-stealing grid);
* no host synchronisation (torch's sync debug mode set to "error" around forward + backward);
* a HIP graph captured with device lengths follows their content on replay (same total rows, other lengths);
* every invalid length set fails closed (NaN, nothing else touched) and is reported;
* the reference's pybind names take device lengths.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O
from _parity import FIXTURES, assert_costs, assert_grads, knobs, random_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def op():
    import monotonic_rnnt_op
    return monotonic_rnnt_op


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


def _t(x, dev=None, dt=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dev is None:
        return t
    return t.to(dev) if dt is None else t.to(dev, dt)


def _run(op, acts, labels, T, S, al=None, k=0, blank=0, scale=None):
    a = acts.detach().clone().requires_grad_(True)
    costs = op.monotonic_rnnt_loss(a, labels, T, S, al, k, blank)
    w = scale if scale is not None else torch.ones_like(costs)
    (costs * w).sum().backward()
    torch.cuda.synchronize()
    return costs.detach(), a.grad.detach()


def _alignment(labels, T, S):
    al = np.zeros((len(T), int(T.max())), np.int32)
    for b in range(len(T)):
        fr = ((np.arange(S[b]) + 0.5) * T[b] / max(S[b], 1)).astype(np.int64)
        al[b, fr] = labels[b, :S[b]]
    return al


CASES = {
    # name: (seed, B, T range, S max, V, dtype, layout, aligned)
    "packed_v128": (1, 6, (20, 90), 30, 128, torch.float32, "packed", False),
    "packed_v37_scalar": (2, 5, (10, 60), 20, 37, torch.float32, "packed", False),
    "packed_v256_row16": (3, 4, (30, 80), 40, 256, torch.float32, "packed", False),
    "packed_v1024": (4, 3, (20, 50), 20, 1024, torch.float32, "packed", False),
    "bf16_v512": (5, 4, (20, 70), 25, 512, torch.bfloat16, "packed", False),
    "padded_v64": (6, 5, (10, 40), 12, 64, torch.float32, "padded", False),
    "aligned_k2": (7, 5, (30, 100), 20, 96, torch.float32, "packed", True),
    "many_columns_b8": (8, 8, (600, 800), 6, 16, torch.float32, "packed", False),
    "steal_b80": (10, 80, (60, 90), 5, 16, torch.float32, "packed", False),  # > 64 utterances: setup kernel + stealing
    "long_labels_halo": (9, 2, (300, 320), 250, 8, torch.float32, "packed", False),
    # 9 <= B <= 64 on shapes the chase launch does not take: the lengths planned inside the log-softmax launch with
    # every lane of a wave holding an utterance (lane 63 = utterance 63), the headline's own kernels
    "fused_b64_v1024": (13, 64, (90, 110), 20, 1024, torch.float32, "packed", False),
    "fused_b64_v512": (14, 64, (60, 100), 40, 512, torch.float32, "packed", False),
    "fused_b64_bf16_v256": (15, 64, (150, 250), 60, 256, torch.bfloat16, "packed", False),
    "fused_b33_v1024": (16, 33, (40, 120), 30, 1024, torch.float32, "packed", False),
}


@pytest.mark.parametrize("separate_setup", [False, True], ids=["default", "setup_kernel"])
@pytest.mark.parametrize("name", list(CASES))
def test_device_lengths_bit_identical_to_host_lengths(op, dev, name, separate_setup):
    """default: batches of <= 64 utterances without an alignment plan inside the log-softmax launch; setup_kernel
    (development build, dyn_fused = 0): the separate setup kernel for every case."""
    if separate_setup:
        with knobs(dyn_fused=0):
            _bit_identical(op, dev, name, True)
    else:
        _bit_identical(op, dev, name, False)


def _bit_identical(op, dev, name, separate_setup):
    seed, B, Tr, Smax, V, dt, layout, aligned = CASES[name]
    rng = np.random.default_rng(seed)
    acts, labels, T, S = random_problem(rng, B, Tr, Smax, V)
    if layout == "padded":
        pad = np.zeros((B, int(T.max()), int(S.max()) + 1, V), np.float32)
        r = 0
        for b in range(B):
            n = T[b] * (S[b] + 1)
            pad[b, :T[b], :S[b] + 1] = acts[r:r + n].reshape(T[b], S[b] + 1, V)
            r += n
        acts_t = _t(pad, dev, dt)
    else:
        acts_t = _t(acts, dev, dt)
    lab = _t(labels, dev)
    al = _t(_alignment(labels, T, S), dev) if aligned else None
    k = 2 if aligned else 0
    scale = torch.linspace(0.5, 2.0, B, device=dev)
    c_host, g_host = _run(op, acts_t, lab, _t(T), _t(S), al, k, scale=scale)
    if name.startswith("fused_"):
        import _mrnnt_lib as L
        L.profile_enable(True)
        try:
            c_dev, g_dev = _run(op, acts_t, lab, _t(T, dev), _t(S, dev), al, k, scale=scale)
            prof = L.profile_read()
        finally:
            L.profile_enable(False)
        assert prof["chase"][1] == 0 and prof["log_softmax"][1] == 1, prof
        assert prof["setup"][1] == (1 if separate_setup else 0), prof
    else:
        c_dev, g_dev = _run(op, acts_t, lab, _t(T, dev), _t(S, dev), al, k, scale=scale)
    assert torch.equal(c_host, c_dev)
    assert torch.equal(g_host.view(torch.int16 if dt != torch.float32 else torch.int32),
                       g_dev.view(torch.int16 if dt != torch.float32 else torch.int32))
    if dt == torch.float32 and layout == "packed" and not aligned:
        cr, gr = O.oracle_rnnt(acts, labels, T, S)
        assert_costs(c_dev.cpu().numpy().astype(np.float64), cr)
        w = np.repeat(scale.cpu().numpy().astype(np.float64), T.astype(np.int64) * (S + 1))[:, None]
        assert_grads(g_dev.cpu().numpy(), gr * w)


def test_device_lengths_make_no_host_sync(op, dev):
    """torch raises on any synchronising call inside the block (the host-lengths path's read-back would)."""
    rng = np.random.default_rng(11)
    acts, labels, T, S = random_problem(rng, 4, (20, 60), 15, 64)
    a = _t(acts, dev).requires_grad_(True)
    lab, Td, Sd = _t(labels, dev), _t(T, dev).long(), _t(S, dev).long()  # int64 lengths: converted on the device
    op.monotonic_rnnt_loss(a, lab, Td, Sd).sum().backward()  # warm-up (allocations)
    torch.cuda.synchronize()
    a.grad = None
    torch.cuda.set_sync_debug_mode("error")
    try:
        costs = op.monotonic_rnnt_loss(a, lab, Td, Sd)
        costs.sum().backward()
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    assert_costs(costs.detach().cpu().numpy().astype(np.float64), cr)
    assert_grads(a.grad.cpu().numpy(), gr)
    with pytest.raises(RuntimeError):  # control: the debug mode does catch a synchronising call
        torch.cuda.set_sync_debug_mode("error")
        try:
            torch.zeros(1, device=dev).item()
        finally:
            torch.cuda.set_sync_debug_mode(0)


def test_graph_with_device_lengths_follows_their_content(op, dev):
    """The lattice is built from the device lengths at replay time: a graph captured with one length set replays
    another of the same total rows (and label width) correctly."""
    rng = np.random.default_rng(12)
    V = 48
    T1, S1 = np.array([10, 10], np.int32), np.array([3, 3], np.int32)  # 40 + 40 rows
    T2, S2 = np.array([16, 4], np.int32), np.array([3, 3], np.int32)   # 64 + 16 rows
    labels = rng.integers(1, V, (2, 3)).astype(np.int32)
    acts = rng.standard_normal((80, V)).astype(np.float32)
    a = _t(acts, dev).requires_grad_(True)
    lab, Td, Sd = _t(labels, dev), _t(T1, dev), _t(S1, dev)

    def step():
        c = op.monotonic_rnnt_loss(a, lab, Td, Sd)
        c.sum().backward()
        return c

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            a.grad = None
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    a.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        c_static = step()
    for T, S in ((T1, S1), (T2, S2)):
        Td.copy_(_t(T, dev))
        Sd.copy_(_t(S, dev))
        g.replay()
        torch.cuda.synchronize()
        cr, gr = O.oracle_rnnt(acts, labels, T, S)
        assert_costs(c_static.detach().cpu().numpy().astype(np.float64), cr)
        assert_grads(a.grad.cpu().numpy(), gr)


def _bad_cases():
    # name: (acts rows, labels width, T, S, padded (pad_T, pad_S1) or None, alignment width or None)
    return {
        "T_less_than_S": (8, 3, [2], [3], None, None),
        "rows_mismatch": (11, 2, [4], [2], None, None),
        "S_above_label_width": (12, 1, [4], [2], None, None),
        "T_zero": (3, 2, [0, 1], [0, 2], None, None),
        "S_negative": (4, 2, [4], [-1], None, None),
        "padded_T_above_pad": (0, 2, [5, 2], [1, 1], (4, 3), None),
        "alignment_narrower_than_T": (12, 2, [4], [2], None, 3),
        "b70_one_bad": (70 * 8, 2, [4] * 69 + [1], [1] * 69 + [2], None, None),
        "huge_T": (12, 2, [1 << 30], [2], None, None),
        "huge_T_b70": (70 * 8, 2, [4] * 69 + [1 << 30], [1] * 70, None, None),
    }


@pytest.mark.parametrize("name", list(_bad_cases()))
def test_invalid_device_lengths_fail_closed(op, dev, name):
    rows, lw, T, S, pad, alw = _bad_cases()[name]
    V, B = 5, len(T)
    acts = (torch.randn(B, pad[0], pad[1], V, device=dev) if pad else torch.randn(rows, V, device=dev))
    lab = torch.ones(B, lw, dtype=torch.int32, device=dev)
    al = torch.zeros(B, alw, dtype=torch.int32, device=dev) if alw else None
    a = acts.clone().requires_grad_(True)
    op.check_lengths()  # nothing pending
    costs = op.monotonic_rnnt_loss(a, lab, torch.tensor(T, device=dev), torch.tensor(S, device=dev), al, 1)
    costs.sum().backward()
    torch.cuda.synchronize()
    assert torch.isnan(costs).all(), costs
    assert torch.isnan(a.grad).all()
    # reported by the next call (no wait) ...
    ok_T, ok_S = torch.tensor([4], device=dev), torch.tensor([2], device=dev)
    good = torch.randn(12, V, device=dev)
    with pytest.raises(RuntimeError, match="failed validation"):
        op.monotonic_rnnt_loss(good, torch.ones(1, 2, dtype=torch.int32, device=dev), ok_T, ok_S)
    # ... once: the report is cleared, and a valid call is exact
    c = op.monotonic_rnnt_loss(good, torch.tensor([[1, 2]], dtype=torch.int32, device=dev), ok_T, ok_S)
    op.check_lengths()
    cr, _ = O.oracle_rnnt(good.cpu().numpy(), np.array([[1, 2]], np.int32), np.array([4], np.int32),
                          np.array([2], np.int32), grads=False)
    assert_costs(c.cpu().numpy().astype(np.float64), cr)


def test_check_lengths_sync_reports_the_failing_call(op, dev):
    acts = torch.randn(8, 5, device=dev)
    c = op.monotonic_rnnt_loss(acts, torch.ones(1, 3, dtype=torch.int32, device=dev), torch.tensor([2], device=dev),
                               torch.tensor([3], device=dev))
    with pytest.raises(RuntimeError, match="failed validation"):
        op.check_lengths()
    assert torch.isnan(c).all()
    op.check_lengths()


@pytest.mark.parametrize("path", [p for p in FIXTURES if "align" not in os.path.basename(p)][:6],
                         ids=lambda p: os.path.basename(p)[:-4])
def test_pybind_names_with_device_lengths(op, dev, path):
    fx = dict(np.load(path))
    acts = _t(fx["acts"], dev)
    costs = torch.zeros(len(fx["T"]))
    grads = torch.zeros_like(acts)
    rc = op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(acts, _t(fx["labels"], dev), _t(fx["T"], dev), _t(fx["S"], dev),
                                                  costs, grads, int(fx["blank"]), 0)
    assert rc == 0
    assert_costs(costs.numpy().astype(np.float64), fx["costs_f64"])
    assert_grads(grads.cpu().numpy(), fx["grads_f64"])


@pytest.mark.parametrize("B", [16, 70])
def test_device_lengths_launch_count(op, dev, B):
    """A batch of <= 64 utterances plans its lengths inside its first launch (no setup kernel at all) -- here the
    chase launch, which runs the whole forward (mrnnt_chase.hip); a larger one runs exactly one setup kernel per
    forward, then the log-softmax and the recursion -- never the host-lengths setup kernels."""
    import _mrnnt_lib as L
    rng = np.random.default_rng(B)
    acts, labels, T, S = random_problem(rng, B, (5, 12), 4, 16)
    a = _t(acts, dev).requires_grad_(True)
    L.profile_enable(True)
    try:
        op.monotonic_rnnt_loss(a, _t(labels, dev), _t(T, dev), _t(S, dev)).sum().backward()
        torch.cuda.synchronize()
        prof = L.profile_read()
    finally:
        L.profile_enable(False)
    assert prof["setup"][1] == (0 if B <= 64 else 1), prof
    if B <= 64:
        assert prof["chase"][1] == 1 and prof["log_softmax"][1] == 0 and prof["alpha_beta"][1] == 0, prof
    else:
        assert prof["chase"][1] == 0 and prof["log_softmax"][1] == 1 and prof["alpha_beta"][1] == 1, prof
    assert prof["grad"][1] == 1, prof


@pytest.mark.parametrize("device_lengths", [True, False])
def test_workspace_cache_follows_dtype_and_V(op, dev, device_lengths):
    """The op caches workspace sizes per shape; the size also depends on the acts element type and V (the chase
    launch, and with it the workspace's ready flags, applies to f32 rows of V <= 1024 only). Found by the round-5
    fuzz sweep (seed 150450: a bf16 call of the same shape before an f32 one left a size without the flags)."""
    rng = np.random.default_rng(150450)
    T, S = np.array([28], np.int32), np.array([0], np.int32)
    labels = _t(np.array([[65]], np.int32), dev)
    Tt, St = (_t(T, dev), _t(S, dev)) if device_lengths else (_t(T), _t(S))
    for dt, V in ((torch.bfloat16, 256), (torch.float32, 256), (torch.float32, 2048), (torch.float32, 256)):
        acts32 = rng.standard_normal((28, V)).astype(np.float32)
        acts = _t(acts32, dev, dt)
        c, g = _run(op, acts, labels, Tt, St, blank=160 % V)
        ref = acts.float().cpu().numpy()
        cr, gr = O.oracle_rnnt(ref, np.array([[65]], np.int32), T, S, blank=160 % V)
        assert_costs(c.cpu().numpy(), cr)
        tol = 1e-4 if dt == torch.float32 else 2e-2
        assert_grads(g.float().cpu().numpy(), gr, tol=tol)
