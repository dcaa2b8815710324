"""Parity of the HIP path (through the C ABI, via the autograd surface) against the oracle.

Oracle = oracle/rnnt_oracle.c at double precision = cpu_rnnt.h<double> on the same fp32 inputs
(pinned bit-exact to the reference in tests/test_oracle.py). Tolerances (north star):
    costs : |dc| <= 1e-4 * max(1, |c|)      (relative for large costs: 1e-4 abs is < 1 ulp at |c| ~ 1e3)
    grads : max |dg| <= 1e-4                 (absolute, fp32)
"""
import glob
import os

import numpy as np
import pytest
import torch

import oracle as O
from _parity import knobs as knobs_ctx

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(glob.glob(os.path.join(GOLD, "*.npz")))
COST_TOL = 1e-4
GRAD_TOL = 1e-4


@pytest.fixture(scope="module")
def op():
    import monotonic_rnnt_op
    return monotonic_rnnt_op


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


def run_gpu(op, dev, acts, labels, T, S, blank=0, alignment=None, k=0, scale=None, grads=True):
    a = torch.from_numpy(np.ascontiguousarray(acts, np.float32)).to(dev).requires_grad_(grads)
    lab = torch.from_numpy(np.ascontiguousarray(labels, np.int32)).to(dev)
    Tt = torch.from_numpy(np.asarray(T, np.int32)).to(dev)
    St = torch.from_numpy(np.asarray(S, np.int32)).to(dev)
    al = None if alignment is None else torch.from_numpy(np.asarray(alignment, np.int32)).to(dev)
    costs = op.monotonic_rnnt_loss(a, lab, Tt, St, al, k, blank)
    g = None
    if grads:
        sc = torch.ones(len(T), device=dev) if scale is None else torch.as_tensor(scale, dtype=torch.float32,
                                                                                  device=dev)
        (costs * sc).sum().backward()
        g = a.grad.detach().cpu().numpy()
    torch.cuda.synchronize()
    return costs.detach().cpu().numpy().astype(np.float64), g


def assert_costs(c, ref):
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(c), fin), (c, ref)
    if fin.any():
        err = np.abs(c[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))
        assert err.max() <= COST_TOL, (err.max(), c, ref)


def assert_grads(g, ref):
    assert g.shape == ref.shape
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(g), fin)
    err = np.abs(g[fin] - ref[fin]).max() if fin.any() else 0.0
    assert err <= GRAD_TOL, err


def random_problem(rng, B, Trange, Smax, V, dist="normal", force=None):
    T = rng.integers(Trange[0], Trange[1] + 1, B).astype(np.int32)
    S = np.array([rng.integers(0, min(t, Smax) + 1) for t in T], np.int32)
    for b, (t, s) in (force or {}).items():
        T[b], S[b] = t, s
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = (rng.standard_normal((rows, V)) if dist == "normal" else rng.random((rows, V))).astype(np.float32)
    labels = rng.integers(1, V, (B, max(1, int(S.max())))).astype(np.int32)
    return acts, labels, T, S


# ---------------------------------------------------------------------------------------------
# golden vectors from the reference (tests/golden)

@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_golden_cost_and_grad(op, dev, path):
    fx = dict(np.load(path))
    kw = dict(blank=int(fx["blank"]), alignment=fx.get("alignment"), k=int(fx.get("max_shift", 0)))
    c, g = run_gpu(op, dev, fx["acts"], fx["labels"], fx["T"], fx["S"], **kw)
    assert_costs(c, fx["costs_f64"])
    assert_grads(g, fx["grads_f64"])
    c_only, _ = run_gpu(op, dev, fx["acts"], fx["labels"], fx["T"], fx["S"], grads=False, **kw)
    assert_costs(c_only, fx["costs_only_f64"])


def test_reference_known_answers(op, dev):
    fx = dict(np.load(os.path.join(GOLD, "toy.npz")))
    c, g = run_gpu(op, dev, fx["acts"], fx["labels"], fx["T"], fx["S"])
    assert abs(c[0] - (-np.log(0.363))) < 1e-4  # tests/test_gpu.cu fwd_test
    # pytorch_binding/test.py:64-66 expected grads at 1e-2
    expected = np.array([0.04, -0.14, 0.1, 0, 0, 0, 0, 0, 0, 0.13, -0.19, 0.06, -0.04, 0.04, -0.01, 0, 0, 0,
                         0.06, -0.1, 0.04, 0.01, 0.07, -0.08, -0.06, 0.04, 0.02, 0, 0, 0, 0.14, 0.05, -0.19,
                         -0.11, 0.05, 0.05]).reshape(12, 3)
    assert np.abs(g - expected).max() < 1e-2
    # pytorch_binding/test.py:71-130
    c1, _ = run_gpu(op, dev, fx["acts"], fx["labels"], fx["T"], fx["S"], alignment=[[0, 1, 0, 2]], k=1)
    assert abs(c1[0] - 1.22) < 1e-2
    c2, _ = run_gpu(op, dev, fx["acts"], fx["labels"], fx["T"], fx["S"], alignment=[[1, 2, 0, 0]], k=0)
    assert abs(c2[0] - 2.7) < 1e-2


def test_out_of_band_rows_are_exact_zero(op, dev):
    fx = dict(np.load(os.path.join(GOLD, "toy.npz")))
    _, g = run_gpu(op, dev, fx["acts"], fx["labels"], fx["T"], fx["S"])
    for r in (1, 2, 5, 9):  # (t,s) = (0,1) (0,2) (1,2) (3,0)
        assert np.all(g[r] == 0.0)


# ---------------------------------------------------------------------------------------------
# random problems vs the oracle

@pytest.mark.parametrize("V", [3, 15, 16, 64, 100, 256, 512, 600, 1000, 1001, 1024, 2052])
def test_random_ragged_vs_oracle(op, dev, V):
    rng = np.random.default_rng(V)
    acts, labels, T, S = random_problem(rng, 5, (1, 40), 12, V, force={0: (1, 0), 1: (9, 9), 2: (17, 0)})
    blank = 0 if V % 2 else V - 1
    if blank:
        labels = np.where(labels == blank, 0, labels).astype(np.int32)
    c, g = run_gpu(op, dev, acts, labels, T, S, blank=blank)
    cr, gr = O.oracle_rnnt(acts, labels, T, S, blank=blank)
    assert_costs(c, cr)
    assert_grads(g, gr)


@pytest.mark.parametrize("k", [0, 1, 3])
def test_alignment_restricted_vs_oracle(op, dev, k):
    rng = np.random.default_rng(100 + k)
    acts, labels, T, S = random_problem(rng, 4, (10, 50), 10, 64)
    al = np.zeros((4, int(T.max()) + 3), np.int32)  # wider than max(T): true row stride is honoured
    for b in range(4):
        pos = np.sort(rng.choice(T[b], S[b], replace=False))
        al[b, pos] = labels[b, : S[b]]
    c, g = run_gpu(op, dev, acts, labels, T, S, alignment=al, k=k)
    cr, gr = O.oracle_rnnt(acts, labels, T, S, alignment=al, max_shift=k)
    assert_costs(c, cr)
    assert_grads(g, gr)


@pytest.mark.parametrize("V", [1, 5, 64])
def test_infeasible_alignment_matches_reference_inf_nan(op, dev, V):
    """An alignment band that no path satisfies (fewer aligned labels than S, k = 0): the reference's cost is +inf
    and every gradient element of that utterance is NaN/inf (exp(... - ll) with ll = -inf, cpu_rnnt.h:221-231),
    out-of-band rows included; the other utterance is unaffected. V = 1: blank only, labels parse as blanks."""
    rng = np.random.default_rng(V)
    acts, labels, T, S = random_problem(rng, 2, (12, 20), 6, max(V, 2), force={0: (15, 5), 1: (14, 4)})
    acts = np.ascontiguousarray(acts[:, :V])
    labels = np.where(labels >= V, 0, labels).astype(np.int32) if V > 1 else np.zeros_like(labels)
    if V > 1:
        labels = np.where(labels == 0, 1, labels).astype(np.int32)
    al = np.zeros((2, 15), np.int32)
    al[0, [2, 7]] = 1 if V > 1 else 0           # 2 (or 0) aligned labels for S = 5: infeasible
    al[1, np.sort(rng.choice(14, 4, replace=False))] = labels[1, :4] if V > 1 else 0
    c, g = run_gpu(op, dev, acts, labels, T, S, alignment=al, k=0, scale=[1.0, -0.5])
    cr, gr = O.oracle_rnnt(acts, labels, T, S, alignment=al, max_shift=0)
    gr = gr * np.repeat(np.array([1.0, -0.5]), T * (S + 1))[:, None]
    assert np.isinf(cr[0]) and np.isinf(c[0])
    assert not np.isfinite(g[: 15 * 6]).any()
    assert_costs(c, cr)
    assert_grads(g, gr)


def test_grad_output_scaling_fused(op, dev):
    rng = np.random.default_rng(5)
    acts, labels, T, S = random_problem(rng, 4, (5, 30), 8, 128)
    scale = np.array([2.5, -1.0, 0.0, 0.3], np.float32)
    c, g = run_gpu(op, dev, acts, labels, T, S, scale=scale)
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    gr = gr * np.repeat(scale.astype(np.float64), T * (S + 1))[:, None]
    assert_costs(c, cr)
    assert_grads(g, gr)


def test_reference_extension_functions(op, dev):
    """monotonic_rnnt_cpp.gpu_monotonic_rnnt[_align_restrict] (reference monotonic_rnnt.cu:81-152)."""
    fx = dict(np.load(os.path.join(GOLD, "multibatch.npz")))
    acts = torch.from_numpy(fx["acts"]).to(dev)
    labels = torch.from_numpy(fx["labels"]).to(dev)
    T = torch.from_numpy(fx["T"]).to(dev)
    S = torch.from_numpy(fx["S"]).to(dev)
    costs = torch.zeros(2)  # host tensor, as the reference passes it
    grads = torch.zeros_like(acts)
    assert op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(acts, labels, T, S, costs, grads, 0, 0) == 0
    assert_costs(costs.numpy().astype(np.float64), fx["costs_f64"])
    assert_grads(grads.cpu().numpy(), fx["grads_f64"])
    fx = dict(np.load(os.path.join(GOLD, "align_multibatch_k1.npz")))
    acts = torch.from_numpy(fx["acts"]).to(dev)
    costs = torch.zeros(2)
    grads = torch.zeros_like(acts)
    rc = op.monotonic_rnnt_cpp.gpu_monotonic_rnnt_align_restrict(
        acts, torch.from_numpy(fx["labels"]).to(dev), torch.from_numpy(fx["T"]).to(dev),
        torch.from_numpy(fx["S"]).to(dev), torch.from_numpy(fx["alignment"]).to(dev), 1, costs, grads, 0, 0)
    assert rc == 0
    assert_costs(costs.numpy().astype(np.float64), fx["costs_f64"])
    assert_grads(grads.cpu().numpy(), fx["grads_f64"])


def test_invalid_lengths_raise(op, dev):
    acts = torch.zeros(12, 3, device=dev)
    with pytest.raises(RuntimeError, match="invalid"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1, 2, 1]], dtype=torch.int32, device=dev),
                               torch.tensor([2], dtype=torch.int32), torch.tensor([3], dtype=torch.int32))
    with pytest.raises(RuntimeError, match="rows"):
        op.monotonic_rnnt_loss(acts[:11], torch.tensor([[1, 2]], dtype=torch.int32, device=dev),
                               torch.tensor([4], dtype=torch.int32), torch.tensor([2], dtype=torch.int32))


@pytest.mark.parametrize("poison", ["nan", "inf", "huge"])
def test_stale_workspace_contents_do_not_matter(op, dev, monkeypatch, poison):
    """The workspace comes from torch's caching allocator holding earlier data (the NaN padding of a padded acts
    tensor, say). Found by tests/test_gpu_fuzz.py: utterance 0's alpha(0, 0) read lpe[-1] from the lp pad."""
    orig = op._Prepared.workspace
    byte = {"nan": 0xFF, "huge": 0x7F}.get(poison)  # all-0xFF doubles are NaN, all-0x7F ones 1.4e306

    def poisoned(self):
        ws = orig(self)
        if byte is not None:
            ws.fill_(byte)
        else:  # +inf doubles over the 8-byte-aligned part
            ws[: ws.numel() // 8 * 8].view(torch.float64).fill_(float("inf"))
        return ws
    monkeypatch.setattr(op._Prepared, "workspace", poisoned)
    rng = np.random.default_rng(5)
    for Tr, Smax, V in (((20, 40), 7, 64), ((60, 90), 59, 33), ((150, 200), 120, 16)):  # 1 wave, 1 wave, halo
        acts, labels, T, S = random_problem(rng, 3, Tr, Smax, V, force={0: (Tr[1], Smax)})
        c, g = run_gpu(op, dev, acts, labels, T, S)
        cr, gr = O.oracle_rnnt(acts, labels, T, S)
        assert_costs(c, cr)
        assert_grads(g, gr)


def test_loglik_forward_equals_backward(op, dev):
    """beta(0,0) == alpha(T-1,S): the two recursions run independently (cpu_rnnt.h:257-259 check)."""
    import ctypes
    import _mrnnt_lib as L
    rng = np.random.default_rng(9)
    acts, labels, T, S = random_problem(rng, 6, (50, 300), 60, 96)
    a = torch.from_numpy(acts).to(dev)
    prep = op._Prepared(a, torch.from_numpy(labels), torch.from_numpy(T), torch.from_numpy(S), None, 0, 0)
    costs, ws = op._forward(prep, with_beta=True)
    llf = torch.empty(6, dtype=torch.float64, device=dev)
    llb = torch.empty(6, dtype=torch.float64, device=dev)
    L.check(L.load().mrnnt_read_loglik(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                       ctypes.c_void_p(llf.data_ptr()), ctypes.c_void_p(llb.data_ptr()),
                                       prep.stream()), "read_loglik")
    torch.cuda.synchronize()
    d = (llf - llb).abs().max().item()
    assert d < 1e-6 * max(1.0, llf.abs().max().item()), d
    assert np.allclose(-llf.cpu().numpy(), costs.cpu().numpy(), rtol=1e-6)


# ---------------------------------------------------------------------------------------------
# BASELINE.json configs

def synth_problem(B, T, S, V, seed=0):
    T = np.full(B, T, np.int32)
    S = np.full(B, S, np.int32)
    return T, S


def test_config_c2_vs_oracle(op, dev):
    """configs[1]: B=16, T=200, S=40, V=256 (grad check <= 1e-4), synthetic N(0,1) acts, seed 0."""
    import _mrnnt_lib as L
    import ctypes
    B, Tn, Sn, V = 16, 200, 40, 256
    T = np.full(B, Tn, np.int32)
    S = np.full(B, Sn, np.int32)
    rows = int(np.sum(T * (S + 1)))
    acts = O.synth_acts(0, rows * V, seed=0).reshape(rows, V)
    rng = np.random.default_rng(1)
    labels = rng.integers(1, V, (B, Sn)).astype(np.int32)
    # the device generator must reproduce the host twin bit for bit (bench parity relies on it)
    d = torch.empty(rows * V, dtype=torch.float32, device=dev)
    L.synth_acts(d.data_ptr(), 0, rows * V, 0, 1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), acts.reshape(-1))
    c, g = run_gpu(op, dev, acts, labels, T, S)
    cr, gr = O.oracle_rnnt(acts, labels, T, S, num_threads=16)
    assert_costs(c, cr)
    assert_grads(g, gr)


def test_accuracy_against_reference_fp32_noise(op, dev):
    """configs[1] shape: distance of this path and of cpu_rnnt.h<float> (its restatement, pinned bit-exact) to the
    fp64 golden. The HIP path (fp64 recursion state) must be at least as close as the reference's own
    fp32 CPU computation."""
    B, Tn, Sn, V = 16, 200, 40, 256
    T = np.full(B, Tn, np.int32)
    S = np.full(B, Sn, np.int32)
    rows = int(np.sum(T * (S + 1)))
    acts = O.synth_acts(0, rows * V, seed=0).reshape(rows, V)
    labels = np.random.default_rng(1).integers(1, V, (B, Sn)).astype(np.int32)
    c, g = run_gpu(op, dev, acts, labels, T, S)
    c64, g64 = O.oracle_rnnt(acts, labels, T, S, num_threads=16)
    c32, g32 = O.oracle_rnnt(acts, labels, T, S, precision="f32", num_threads=16)
    ours = (float(np.max(np.abs(c - c64) / np.abs(c64))), float(np.max(np.abs(g - g64))))
    ref32 = (float(np.max(np.abs(c32 - c64) / np.abs(c64))), float(np.max(np.abs(g32 - g64))))
    print(f"\naccuracy vs cpu_rnnt.h<double>: HIP path costs rel {ours[0]:.3e} grads abs {ours[1]:.3e}; "
          f"cpu_rnnt.h<float> costs rel {ref32[0]:.3e} grads abs {ref32[1]:.3e}")
    assert ours[0] <= max(ref32[0], 1e-6) and ours[1] <= max(ref32[1], 1e-6), (ours, ref32)


@pytest.mark.parametrize("knob_set", [
    {"softmax_variant": 0, "grad_variant": 0, "grid_per_cu": 8, "nt_store": 1},
    {"softmax_variant": 2, "grad_variant": 2, "grid_per_cu": 0, "nt_store": 0},
    {"softmax_variant": 0, "grad_variant": 0, "grid_per_cu": 3, "nt_store": 1},
    {"softmax_variant": 0, "grad_variant": 0, "softmax_grid_per_cu": 0, "grad_grid_per_cu": 32},
    {"softmax_variant": 2, "grad_variant": 2, "softmax_grid_per_cu": 0, "grad_grid_per_cu": 32},
    {"softmax_variant": 0, "grad_variant": 2, "nt_load": 0, "nt_store": 0},
    {"softmax_variant": 2, "grad_variant": 3, "softmax_grid_per_cu": 5, "grad_grid_per_cu": 7},
    {"softmax_variant": 0, "grad_variant": 3, "grid_per_cu": 16, "nt_store": 1, "nt_load": 0},
    {"softmax_variant": 2, "grad_variant": 6, "softmax_grid_per_cu": 3, "grad_grid_per_cu": 5},
    {"softmax_variant": 13},
    {"softmax_variant": 14, "softmax_grid_per_cu": 2, "nt_load": 0},
    {"softmax_variant": 15},
    {"col_scatter": 3},
    {"dp_halo": 0},
    {"dp_halo": 1},
    {"dp_halo": 2},
    {"col_scatter": 0, "grad_variant": 6},
    {"col_scatter": 3, "grad_grid_per_cu": 0, "softmax_grid_per_cu": 4},
    {"grad_variant": 5},
    {"grad_variant": 6, "grad_grid_per_cu": 3, "nt_load": 0, "nt_store": 0},
])
def test_every_kernel_variant_matches_oracle(op, dev, knob_set):
    """All launch variants selectable through mrnnt_tune (development build) compute the same result (alignment
    included)."""
    with knobs_ctx(**knob_set):
        rng = np.random.default_rng(77)
        for V, S_max, extra in ((1024, 40, 60), (260, 300, 60), (64, 12, 60), (32, 100, 200), (16, 200, 150)):
            acts, labels, T, S = random_problem(rng, 3, (S_max, S_max + extra), S_max, V, force={0: (S_max + extra, S_max)})
            c, g = run_gpu(op, dev, acts, labels, T, S)
            cr, gr = O.oracle_rnnt(acts, labels, T, S)
            assert_costs(c, cr)
            assert_grads(g, gr)
        for Tr, S_max, V, k in (((20, 60), 10, 128, 2), ((160, 220), 150, 32, 5)):  # 1 wave / halo recursion
            acts, labels, T, S = random_problem(rng, 3, Tr, S_max, V, force={0: (Tr[1], S_max)})
            al = np.zeros((3, int(T.max())), np.int32)
            for b in range(3):
                al[b, np.sort(rng.choice(T[b], S[b], replace=False))] = labels[b, : S[b]]
            c, g = run_gpu(op, dev, acts, labels, T, S, alignment=al, k=k)
            cr, gr = O.oracle_rnnt(acts, labels, T, S, alignment=al, max_shift=k)
            assert_costs(c, cr)
            assert_grads(g, gr)


@pytest.mark.parametrize("S_len,T_len,V", [(1100, 1200, 16), (64, 64, 8), (128, 300, 12), (511, 530, 8),
                                           (2047, 2060, 4)])
def test_long_label_sequences_vs_oracle(op, dev, S_len, T_len, V):
    """Label lengths across the recursion's wave/cell sizing boundaries (S+1 = 65, 129, 512, 1101)."""
    rng = np.random.default_rng(S_len)
    T = np.array([T_len, max(S_len, T_len - 7)], np.int32)
    S = np.array([S_len, S_len - 1], np.int32)
    rows = int(np.sum(T * (S + 1)))
    acts = rng.standard_normal((rows, V)).astype(np.float32)
    labels = rng.integers(1, V, (2, S_len)).astype(np.int32)
    c, g = run_gpu(op, dev, acts, labels, T, S)
    cr, gr = O.oracle_rnnt(acts, labels, T, S, num_threads=2)
    assert_costs(c, cr)
    assert_grads(g, gr)


# ---------------------------------------------------------------------------------------------
# extensions: padded [B, pad_T, pad_S1, V] acts read in place; bf16 / fp16 acts

def pack_to_padded(acts, T, S, pad_T, pad_S1, fill=np.nan):
    """Scatter packed rows into the padded joint-network layout; padding rows hold `fill`."""
    B, V = len(T), acts.shape[1]
    out = np.full((B, pad_T, pad_S1, V), fill, np.float32)
    r = 0
    for b in range(B):
        n = int(T[b]) * (int(S[b]) + 1)
        out[b, : T[b], : S[b] + 1] = acts[r:r + n].reshape(T[b], S[b] + 1, V)
        r += n
    return out


def padded_to_packed(x, T, S):
    return np.concatenate([x[b, : T[b], : S[b] + 1].reshape(-1, x.shape[-1]) for b in range(len(T))])


@pytest.mark.parametrize("V", [7, 64, 1024])
def test_padded_layout_bit_identical_to_packed(op, dev, V):
    """The padded layout reads the same logits in place: costs and lattice grads are bit-identical to the
    packed run, padding rows of grads are exactly 0 (NaN-filled padding of acts is never read)."""
    rng = np.random.default_rng(300 + V)
    acts, labels, T, S = random_problem(rng, 4, (1, 30), 9, V, force={0: (30, 9), 1: (1, 0)})
    pad_T, pad_S1 = int(T.max()) + 2, int(S.max()) + 3
    scale = np.array([1.0, -2.0, 0.5, 3.0], np.float32)
    c, g = run_gpu(op, dev, acts, labels, T, S, scale=scale)
    xp = torch.from_numpy(pack_to_padded(acts, T, S, pad_T, pad_S1)).to(dev).requires_grad_(True)
    cp = op.monotonic_rnnt_loss(xp, torch.from_numpy(labels).to(dev), torch.from_numpy(T), torch.from_numpy(S))
    (cp * torch.from_numpy(scale).to(dev)).sum().backward()
    gp = xp.grad.cpu().numpy()
    assert np.array_equal(cp.detach().cpu().numpy().astype(np.float64), c)
    assert np.array_equal(padded_to_packed(gp, T, S), g)
    mask = np.ones(gp.shape[:3], bool)
    for b in range(4):
        mask[b, : T[b], : S[b] + 1] = False
    assert np.all(gp[mask] == 0.0)
    # the reference-named extension function takes the padded layout too
    costs = torch.zeros(4)
    grads = torch.empty_like(xp)
    assert op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(xp.detach(), torch.from_numpy(labels).to(dev),
                                                    torch.from_numpy(T), torch.from_numpy(S), costs, grads, 0) == 0
    assert np.array_equal(costs.numpy().astype(np.float64), c)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("V", [15, 256, 1000, 1024])
def test_reduced_precision_acts_vs_oracle(op, dev, dtype, V):
    """bf16 / fp16 acts, fp32/fp64 math: parity against the double oracle on the upcast inputs.
    Tolerance: costs as fp32 (1e-4 relative); grads 1e-4 absolute + one rounding of the output type
    (2^-8 relative for bf16, 2^-11 for fp16), since grads are stored in the acts element type."""
    rng = np.random.default_rng(400 + V)
    acts, labels, T, S = random_problem(rng, 4, (1, 40), 12, V, force={0: (40, 12)})
    a = torch.from_numpy(acts).to(dev).to(dtype).requires_grad_(True)
    up = a.detach().float().cpu().numpy()  # the exact values the kernels read
    scale = np.array([1.0, 0.5, -1.0, 2.0], np.float32)
    costs = op.monotonic_rnnt_loss(a, torch.from_numpy(labels).to(dev), torch.from_numpy(T), torch.from_numpy(S))
    assert costs.dtype == torch.float32
    (costs * torch.from_numpy(scale).to(dev)).sum().backward()
    assert a.grad.dtype == dtype
    g = a.grad.float().cpu().numpy()
    cr, gr = O.oracle_rnnt(up, labels, T, S)
    gr = gr * np.repeat(scale.astype(np.float64), T * (S + 1))[:, None]
    assert_costs(costs.detach().cpu().numpy().astype(np.float64), cr)
    rel = 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11
    err = np.abs(g - gr) - rel * np.abs(gr)
    assert err.max() <= GRAD_TOL, err.max()


def test_reduced_precision_padded_and_aligned(op, dev):
    """bf16 + padded layout + alignment band together, against the oracle on the upcast packed inputs."""
    rng = np.random.default_rng(555)
    acts, labels, T, S = random_problem(rng, 3, (20, 60), 10, 128)
    al = np.zeros((3, int(T.max())), np.int32)
    for b in range(3):
        al[b, np.sort(rng.choice(T[b], S[b], replace=False))] = labels[b, : S[b]]
    pad = pack_to_padded(acts, T, S, int(T.max()), int(S.max()) + 1, fill=0.0)
    x = torch.from_numpy(pad).to(dev).to(torch.bfloat16).requires_grad_(True)
    up = padded_to_packed(x.detach().float().cpu().numpy(), T, S)
    costs = op.monotonic_rnnt_loss(x, torch.from_numpy(labels).to(dev), torch.from_numpy(T), torch.from_numpy(S),
                                   torch.from_numpy(al).to(dev), 2)
    costs.sum().backward()
    g = padded_to_packed(x.grad.float().cpu().numpy(), T, S)
    cr, gr = O.oracle_rnnt(up, labels, T, S, alignment=al, max_shift=2)
    assert_costs(costs.detach().cpu().numpy().astype(np.float64), cr)
    assert (np.abs(g - gr) - 2.0 ** -8 * np.abs(gr)).max() <= GRAD_TOL


# ---------------------------------------------------------------------------------------------
# occupancy skip: rows whose fp32 gradient is exactly zero are stored without reading acts

def _live_rows(op, dev, acts, labels, T, S, alignment=None, k=0):
    import ctypes
    import _mrnnt_lib as L
    a = torch.from_numpy(acts).to(dev)
    al = None if alignment is None else torch.from_numpy(alignment).to(dev)
    prep = op._Prepared(a, torch.from_numpy(labels), torch.from_numpy(T), torch.from_numpy(S), al, k, 0)
    _, ws = op._forward(prep, with_beta=True)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    L.check(L.load().mrnnt_grad_live_rows(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                          ctypes.c_void_p(cnt.data_ptr()), prep.stream()), "live_rows")
    return int(cnt.item())


@pytest.mark.parametrize("grad_variant", [0, 2, 3, 5, 6])
def test_occupancy_skip_is_bit_identical(op, dev, grad_variant):
    """With occ_skip the gradient kernel does not read acts rows whose occupancy is < e^-110; their fp32
    gradient is exactly 0 either way, so grads must be bit-identical with the skip on and off (and match the
    oracle), while the live-row count drops below the in-band row count on long utterances."""
    import _mrnnt_lib as L
    rng = np.random.default_rng(606)
    T = np.array([400, 300, 37, 250], np.int32)
    S = np.array([80, 120, 5, 0], np.int32)
    V = 64
    rows = int(np.sum(T * (S + 1)))
    acts = (3.0 * rng.standard_normal((rows, V))).astype(np.float32)
    labels = rng.integers(1, V, (4, int(S.max()))).astype(np.int32)
    scale = np.array([1.0, -0.5, 2.0, 0.0], np.float32)
    n_band = int(np.sum((S.astype(np.int64) + 1) * (T - S + 1) - 1))
    with knobs_ctx(grad_variant=grad_variant):
        out = {}
        for skip in (0, 1):
            with knobs_ctx(occ_skip=skip):
                out[skip] = run_gpu(op, dev, acts, labels, T, S, scale=scale)
                live = _live_rows(op, dev, acts, labels, T, S)
                if skip:
                    assert live < 0.9 * n_band, (live, n_band)
                else:
                    assert live == n_band
        assert np.array_equal(out[0][0], out[1][0])
        assert np.array_equal(out[0][1].view(np.uint32), out[1][1].view(np.uint32))  # signed zeros included
        cr, gr = O.oracle_rnnt(acts, labels, T, S, num_threads=4)
        gr = gr * np.repeat(scale.astype(np.float64), T * (S + 1))[:, None]
        assert_costs(out[1][0], cr)
        assert_grads(out[1][1], gr)


@pytest.mark.parametrize("grad_variant", [0, 5])
def test_alignment_window_with_and_without_occupancy_skip(op, dev, grad_variant):
    """Alignment-restricted calls reduce only the rows of each column's alignment window; rows outside it get
    zero lp/den. With the occupancy skip off the gradient kernel reads those rows too: the result must still be
    bit-identical to the skip-on run (every such row meets alpha or beta = -inf) and match the oracle."""
    import _mrnnt_lib as L
    rng = np.random.default_rng(707)
    T = np.array([300, 220, 90], np.int32)
    S = np.array([110, 60, 30], np.int32)
    V = 48
    rows = int(np.sum(T * (S + 1)))
    acts = rng.standard_normal((rows, V)).astype(np.float32)
    labels = rng.integers(1, V, (3, int(S.max()))).astype(np.int32)
    al = np.zeros((3, int(T.max())), np.int32)
    for b in range(3):
        al[b, np.sort(rng.choice(T[b], S[b], replace=False))] = labels[b, : S[b]]
    scale = np.array([1.0, -2.0, 0.5], np.float32)
    k = 3
    with knobs_ctx(grad_variant=grad_variant):
        out = {}
        for skip in (0, 1):
            with knobs_ctx(occ_skip=skip):
                out[skip] = run_gpu(op, dev, acts, labels, T, S, alignment=al, k=k, scale=scale)
        assert np.array_equal(out[0][0], out[1][0])
        assert np.array_equal(out[0][1].view(np.uint32), out[1][1].view(np.uint32))
        cr, gr = O.oracle_rnnt(acts, labels, T, S, alignment=al, max_shift=k, num_threads=4)
        gr = gr * np.repeat(scale.astype(np.float64), T * (S + 1))[:, None]
        assert_costs(out[1][0], cr)
        assert_grads(out[1][1], gr)


@pytest.mark.parametrize("B,T,S,V", [(1, 150, 20, 50), (1, 150, 20, 5000), (16, 150, 20, 50), (16, 150, 20, 5000),
                                     (2, 391, 300, 79)])
def test_reference_size_cases_vs_oracle(op, dev, B, T, S, V):
    """The shape list of the reference's size tests (tensorflow_binding/test.py:159-176: uniform [0,1) acts like
    tests/random.cpp:4-20, labels U[1, V-1] with a forced repeat at S/2 like tests/random.cpp:22-37), here
    checked against the oracle rather than only for inf/NaN."""
    rng = np.random.default_rng(B * 1000 + S)
    Tn = np.full(B, T, np.int32)
    Sn = np.full(B, S, np.int32)
    rows = int(np.sum(Tn * (Sn + 1)))
    acts = rng.random((rows, V), dtype=np.float32)
    labels = rng.integers(1, V, (B, S)).astype(np.int32)
    labels[:, S // 2] = labels[:, S // 2 - 1]
    c, g = run_gpu(op, dev, acts, labels, Tn, Sn)
    assert np.all(np.isfinite(c)) and np.all(np.isfinite(g))
    cr, gr = O.oracle_rnnt(acts, labels, Tn, Sn, num_threads=8)
    assert_costs(c, cr)
    assert_grads(g, gr)


def test_gradient_in_place_over_acts(op, dev):
    """mrnnt_backward with grads == acts (the reference extension's output-buffer form, used to fit batches whose
    acts + grads exceed HBM): every element of a row is read before it is written and the log-softmax pass is
    complete, so the in-place result equals the out-of-place one bit for bit."""
    rng = np.random.default_rng(808)
    acts, labels, T, S = random_problem(rng, 4, (20, 120), 30, 1024)
    a = torch.from_numpy(acts).to(dev)
    lab = torch.from_numpy(labels).to(dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    c1, g1 = torch.zeros(4), torch.empty_like(a)
    assert op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(a, lab, Tt, St, c1, g1, 0) == 0
    c2 = torch.zeros(4)
    assert op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(a, lab, Tt, St, c2, a, 0) == 0  # grads written over acts
    torch.cuda.synchronize()
    assert torch.equal(c1, c2)
    assert torch.equal(g1.view(torch.int32), a.view(torch.int32))
