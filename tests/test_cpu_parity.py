"""Parity of the library's host implementation (RNNT_CPU: mrnnt_cpu_*, reached through the autograd op with CPU
tensors and through the reference's cpu_monotonic_rnnt extension functions) against the reference's golden
vectors and the oracle. Runs without a GPU.

Reference surfaces: pytorch_binding/monotonic_rnnt_op.py:63-88 (CPU dispatch), monotonic_rnnt.cu:16-77
(cpu_monotonic_rnnt[_align_restrict]), pytorch_binding/test.py:6-130 (its own assertions, below verbatim in
meaning). Tolerances: tests/_parity.py.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

import oracle as O
from _parity import FIXTURES, assert_costs, assert_grads, assert_state, random_problem, used_rows

import monotonic_rnnt_op as op
import _mrnnt_lib as L


def run_cpu(acts, labels, T, S, blank=0, alignment=None, k=0, scale=None, grads=True):
    a = torch.from_numpy(np.ascontiguousarray(acts, np.float32)).requires_grad_(grads)
    al = None if alignment is None else torch.from_numpy(np.asarray(alignment, np.int32))
    costs = op.monotonic_rnnt_loss(a, torch.from_numpy(np.ascontiguousarray(labels, np.int32)),
                                   torch.from_numpy(np.asarray(T, np.int32)), torch.from_numpy(np.asarray(S, np.int32)),
                                   al, k, blank)
    assert costs.device.type == "cpu" and costs.dtype == torch.float32
    g = None
    if grads:
        sc = torch.ones(len(T)) if scale is None else torch.as_tensor(scale, dtype=torch.float32)
        (costs * sc).sum().backward()
        g = a.grad.numpy()
    return costs.detach().numpy().astype(np.float64), g


def load(path):
    return dict(np.load(path if os.path.isabs(path) else os.path.join(os.path.dirname(FIXTURES[0]), path + ".npz")))


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_golden_cost_and_grad(path):
    fx = load(path)
    c, g = run_cpu(fx["acts"], fx["labels"], fx["T"], fx["S"], int(fx["blank"]), fx.get("alignment"),
                   int(fx.get("max_shift", 0)))
    assert_costs(c, fx["costs_f64"])
    assert_grads(g, fx["grads_f64"])
    c0, _ = run_cpu(fx["acts"], fx["labels"], fx["T"], fx["S"], int(fx["blank"]), fx.get("alignment"),
                    int(fx.get("max_shift", 0)), grads=False)
    assert_costs(c0, fx["costs_only_f64"])


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_golden_denominators_alpha_beta(path):
    """The workspace's per-row state (mrnnt_cpu_read_state) against the reference's own get_denom / get_alpha /
    get_beta at double precision (golden denom_f64 / alpha_f64 / beta_f64)."""
    fx = load(path)
    prep = op._Prepared(torch.from_numpy(fx["acts"]), torch.from_numpy(fx["labels"]), torch.from_numpy(fx["T"]),
                        torch.from_numpy(fx["S"]),
                        None if "alignment" not in fx else torch.from_numpy(fx["alignment"]),
                        int(fx.get("max_shift", 0)), int(fx["blank"]))
    _, ws = op._forward(prep, with_beta=True)
    n = fx["acts"].shape[0]
    den, al, be = np.zeros(n, np.float32), np.zeros(n), np.zeros(n)
    L.check(L.load().mrnnt_cpu_read_state(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                          den.ctypes.data, al.ctypes.data, be.ctypes.data), "read_state")
    assert_state(den, al, be, fx, window=used_rows(fx), rel=1e-6)


def test_reference_pytorch_binding_test_py():
    """pytorch_binding/test.py:6-130 on CPU tensors, its assertions unchanged."""
    p = torch.tensor([[0.6, 0.3, 0.1], [0.7, 0.1, 0.2], [0.5, 0.1, 0.4], [0.5, 0.4, 0.1], [0.5, 0.1, 0.4],
                      [0.8, 0.1, 0.1], [0.4, 0.3, 0.3], [0.5, 0.1, 0.4], [0.7, 0.2, 0.1], [0.8, 0.1, 0.1],
                      [0.3, 0.1, 0.6], [0.8, 0.1, 0.1]], dtype=torch.float32)
    acts = torch.log(p)
    labels = torch.tensor([[1, 2]], dtype=torch.int32)
    lengths = torch.tensor([4], dtype=torch.int32)
    label_lengths = torch.tensor([2], dtype=torch.int32)
    acts.requires_grad_(True)
    costs = op.monotonic_rnnt_loss(acts=acts, labels=labels, input_lengths=lengths, label_lengths=label_lengths,
                                   blank_label=0)
    cost = costs.detach().numpy()[0]
    costs.backward()
    expected = torch.tensor([[0.04, -0.14, 0.1], [0.0, 0.0, 0.0], [0.0, 0.0, 0.0], [0.13, -0.19, 0.06],
                             [-0.04, 0.04, -0.01], [0.0, 0.0, 0.0], [0.06, -0.1, 0.04], [0.01, 0.07, -0.08],
                             [-0.06, 0.04, 0.02], [0.0, 0.0, 0.0], [0.14, 0.05, -0.19], [-0.11, 0.05, 0.05]])
    assert abs(cost - 1.01) < 1e-02
    assert torch.allclose(acts.grad, expected, atol=1e-02)

    acts = torch.log(p).requires_grad_(True)
    costs = op.monotonic_rnnt_loss(acts=acts, labels=labels, input_lengths=lengths, label_lengths=label_lengths,
                                   alignment=torch.tensor([[0, 1, 0, 2]], dtype=torch.int32),
                                   max_distance_from_alignment=1, blank_label=0)
    assert abs(costs.detach().numpy()[0] - 1.22) < 1e-02
    costs = op.monotonic_rnnt_loss(acts=acts, labels=labels, input_lengths=lengths, label_lengths=label_lengths,
                                   alignment=torch.tensor([[1, 2, 0, 0]], dtype=torch.int32),
                                   max_distance_from_alignment=0, blank_label=0)
    assert abs(costs.detach().numpy()[0] - 2.7) < 1e-02
    # the module form (MonotonicRNNTLoss) and a grad_output of 2.5 (the reference's backward scaling, §8c)
    acts = torch.log(p).requires_grad_(True)
    (op.MonotonicRNNTLoss(blank_label=0)(acts, labels, lengths, label_lengths) * 2.5).sum().backward()
    assert torch.allclose(acts.grad[0], torch.tensor([0.1033, -0.3533, 0.2500]), atol=1e-3)


def test_reference_extension_functions_cpu():
    """monotonic_rnnt_cpp.cpu_monotonic_rnnt[_align_restrict] (reference monotonic_rnnt.cu:16-77): host costs
    and grads filled in place, return 0; grads = acts writes the gradient over the logits."""
    fx = load("multibatch")
    acts = torch.from_numpy(fx["acts"])
    args = (torch.from_numpy(fx["labels"]), torch.from_numpy(fx["T"]), torch.from_numpy(fx["S"]))
    costs, grads = torch.zeros(2), torch.zeros_like(acts)
    assert op.monotonic_rnnt_cpp.cpu_monotonic_rnnt(acts, *args, costs, grads, 0, 2) == 0
    assert_costs(costs.numpy(), fx["costs_f64"])
    assert_grads(grads.numpy(), fx["grads_f64"])
    inplace = acts.clone()
    assert op.monotonic_rnnt_cpp.cpu_monotonic_rnnt(inplace, *args, costs, inplace, 0, 0) == 0
    assert torch.equal(inplace, grads)
    fx = load("align_multibatch_k1")
    costs, grads = torch.zeros(2), torch.zeros_like(torch.from_numpy(fx["acts"]))
    rc = op.monotonic_rnnt_cpp.cpu_monotonic_rnnt_align_restrict(
        torch.from_numpy(fx["acts"]), torch.from_numpy(fx["labels"]), torch.from_numpy(fx["T"]),
        torch.from_numpy(fx["S"]), torch.from_numpy(fx["alignment"]), 1, costs, grads, 0, 0)
    assert rc == 0
    assert_costs(costs.numpy(), fx["costs_f64"])
    assert_grads(grads.numpy(), fx["grads_f64"])
    with pytest.raises(RuntimeError, match="GPU"):
        op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(acts, *args, costs, grads, 0, 0)


@pytest.mark.parametrize("seed", range(6))
def test_random_vs_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    V = [2, 3, 17, 64, 256, 1000][seed]
    acts, labels, T, S = random_problem(rng, 5, (1, 40), 12, V, dist="normal" if seed % 2 else "uniform")
    blank = int(rng.integers(0, V))
    scale = rng.standard_normal(5).astype(np.float32)
    c, g = run_cpu(acts, labels, T, S, blank=blank, scale=scale)
    cr, gr = O.oracle_rnnt(acts, labels, T, S, blank=blank)
    assert_costs(c, cr)
    assert_grads(g, gr * np.repeat(scale.astype(np.float64), T * (S + 1))[:, None])


@pytest.mark.parametrize("k", [0, 1, 3])
def test_random_alignment_vs_oracle(k):
    rng = np.random.default_rng(7 + k)
    acts, labels, T, S = random_problem(rng, 4, (8, 40), 10, 32)
    al = np.zeros((4, int(T.max()) + 3), np.int32)  # a wider row stride than max(T): the true stride is used
    for b in range(4):
        al[b, np.sort(rng.choice(T[b], S[b], replace=False))] = labels[b, :S[b]]
    c, g = run_cpu(acts, labels, T, S, alignment=al, k=k)
    cr, gr = O.oracle_rnnt(acts, labels, T, S, alignment=al, max_shift=k)
    assert_costs(c, cr)
    assert_grads(g, gr)


def test_configs1_full_vs_oracle():
    """configs[1] (B=16, T=200, S=40, V=256) on the host implementation, every utterance against the oracle."""
    B, T, S, V = 16, 200, 40, 256
    rows = B * T * (S + 1)
    acts = O.synth_acts(0, rows * V, seed=0).reshape(rows, V)
    labels = np.random.default_rng(1).integers(1, V, (B, S)).astype(np.int32)
    Tl, Sl = np.full(B, T, np.int32), np.full(B, S, np.int32)
    c, g = run_cpu(acts, labels, Tl, Sl)
    cr, gr = O.oracle_rnnt(acts, labels, Tl, Sl)
    assert_costs(c, cr)
    assert_grads(g, gr)


@pytest.mark.parametrize("V", [1, 5, 64])
def test_infeasible_alignment_inf_nan(V):
    """An alignment band no path satisfies: cost +inf and every gradient element of that utterance non-finite
    (exp(... - ll) with ll = -inf, cpu_rnnt.h:221-231); the other utterance unaffected."""
    rng = np.random.default_rng(V)
    acts, labels, T, S = random_problem(rng, 2, (12, 20), 6, max(V, 2), force={0: (15, 5), 1: (14, 4)})
    acts = np.ascontiguousarray(acts[:, :V])
    labels = np.where(labels >= V, 1, labels).astype(np.int32) if V > 1 else np.zeros_like(labels)
    al = np.zeros((2, 15), np.int32)
    al[0, [2, 7]] = 1 if V > 1 else 0
    al[1, np.sort(rng.choice(14, 4, replace=False))] = labels[1, :4] if V > 1 else 0
    c, g = run_cpu(acts, labels, T, S, alignment=al, k=0, scale=[1.0, -0.5])
    cr, gr = O.oracle_rnnt(acts, labels, T, S, alignment=al, max_shift=0)
    gr = gr * np.repeat(np.array([1.0, -0.5]), T * (S + 1))[:, None]
    assert np.isinf(cr[0]) and np.isinf(c[0])
    assert not np.isfinite(g[: 15 * 6]).any()
    assert_costs(c, cr)
    assert_grads(g, gr)


def test_cost_only_without_requires_grad():
    """acts.requires_grad=False: cost only (the reference's CPU path segfaults here, SURVEY §8b quirk i)."""
    fx = load("multibatch")
    costs = op.monotonic_rnnt_loss(torch.from_numpy(fx["acts"]), torch.from_numpy(fx["labels"]),
                                   torch.from_numpy(fx["T"]), torch.from_numpy(fx["S"]))
    assert costs.grad_fn is None
    assert_costs(costs.numpy(), fx["costs_only_f64"])


def test_backward_twice_with_retain_graph():
    rng = np.random.default_rng(3)
    acts, labels, T, S = random_problem(rng, 3, (5, 20), 6, 16)
    a = torch.from_numpy(acts).requires_grad_(True)
    costs = op.monotonic_rnnt_loss(a, torch.from_numpy(labels), torch.from_numpy(T), torch.from_numpy(S))
    costs.sum().backward(retain_graph=True)
    g1 = a.grad.clone()
    a.grad = None
    costs.sum().backward()
    assert torch.equal(a.grad, g1)
    with pytest.raises(RuntimeError):
        costs.sum().backward()  # the saved workspace was freed by the last backward


def test_broadcast_upstream_gradient():
    """costs.sum() / costs.mean() hand backward a stride-0 [B] gradient, read in place (grad_scale_broadcast, ABI
    v6): bit-identical to the same scale as a materialised [B] vector, and against the oracle."""
    rng = np.random.default_rng(5)
    acts, labels, T, S = random_problem(rng, 4, (5, 20), 6, 16)
    out = []
    for reduce in (lambda c: c.sum(), lambda c: c.mean(), lambda c: (c * torch.full_like(c, 1.0 / 4)).sum()):
        a = torch.from_numpy(acts).requires_grad_(True)
        reduce(op.monotonic_rnnt_loss(a, torch.from_numpy(labels), torch.from_numpy(T), torch.from_numpy(S))).backward()
        out.append(a.grad)
    assert torch.equal(out[1], out[2])
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    assert_grads(out[0].numpy(), gr)


def test_padded_layout_equals_packed():
    rng = np.random.default_rng(11)
    acts, labels, T, S = random_problem(rng, 3, (4, 15), 5, 9)
    pad_T, pad_S1 = int(T.max()) + 2, int(S.max()) + 3
    padded = np.full((3, pad_T, pad_S1, 9), np.nan, np.float32)
    r = 0
    for b in range(3):
        n = T[b] * (S[b] + 1)
        padded[b, :T[b], :S[b] + 1] = acts[r:r + n].reshape(T[b], S[b] + 1, 9)
        r += n
    c, g = run_cpu(acts, labels, T, S)
    cp, gp = run_cpu(padded, labels, T, S)
    assert np.array_equal(c, cp)
    r = 0
    for b in range(3):
        n = T[b] * (S[b] + 1)
        assert np.array_equal(gp[b, :T[b], :S[b] + 1].reshape(n, 9), g[r:r + n])
        rest = gp[b].copy()
        rest[:T[b], :S[b] + 1] = 0
        assert not rest.any()
        r += n


def test_thread_count_does_not_change_results():
    rng = np.random.default_rng(5)
    acts, labels, T, S = random_problem(rng, 6, (20, 60), 15, 128)
    out = []
    for nt in (1, 3, 8):
        costs, grads = torch.zeros(6), torch.zeros(acts.shape)
        op.monotonic_rnnt_cpp.cpu_monotonic_rnnt(torch.from_numpy(acts), torch.from_numpy(labels),
                                                 torch.from_numpy(T), torch.from_numpy(S), costs, grads, 0, nt)
        out.append((costs, grads))
    for c, g in out[1:]:
        assert torch.equal(c, out[0][0]) and torch.equal(g, out[0][1])


def test_validation_errors():
    fx = load("toy")
    acts, T, S = torch.from_numpy(fx["acts"]), torch.from_numpy(fx["T"]), torch.from_numpy(fx["S"])
    with pytest.raises(RuntimeError, match="outside"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1, 3]], dtype=torch.int32), T, S)  # V = 3
    with pytest.raises(RuntimeError, match="outside"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[-1, 2]], dtype=torch.int32), T, S)
    with pytest.raises(RuntimeError, match="stride"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1]], dtype=torch.int32), T, S)
    with pytest.raises(RuntimeError, match="stride"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1, 2]], dtype=torch.int32), T, S,
                               torch.tensor([[0, 1, 0]], dtype=torch.int32), 0)
    with pytest.raises(RuntimeError, match="invalid"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1, 2, 1]], dtype=torch.int32), torch.tensor([2]),
                               torch.tensor([3]))
    with pytest.raises(RuntimeError, match="rows"):
        op.monotonic_rnnt_loss(acts[:11], torch.tensor([[1, 2]], dtype=torch.int32), T, S)
    with pytest.raises(RuntimeError, match="float32"):
        op.monotonic_rnnt_loss(acts.double(), torch.tensor([[1, 2]], dtype=torch.int32), T, S)
