"""Parity of the fused joint network + loss (monotonic_rnnt_joint.py / mrnnt_joint.hip) against a host reference.

Reference = the composition the fused op replaces, evaluated on the host in fp64 from the same bf16 inputs:
  h    = bf16(tanh(enc + pred))                  (fp32 tanh, round-to-nearest-even to bf16, like the kernel)
  acts = h @ weight.T + bias  (fp64, then fp32)  -> the oracle (cpu_rnnt.h<double> restatement) for costs, dacts
  dweight = dacts^T h, dbias = sum dacts, dpre = (dacts weight) (1 - h^2), denc/dpred = dpre summed over s / t.

Tolerances (floating-point extension on bf16 matrix cores, stated here):
  costs : |dc| <= 1e-5 * max(1, |c|)   (fp32 accumulation of exact bf16 products; the kernel's fast tanh can land on
                                         the other side of a bf16 rounding boundary than the host's for rare elements)
  grads : max |dg| <= 1.5e-2 * max |g_ref| + 1e-5 per tensor (the logit gradient is stored as bf16, 2^-9 relative,
                                         and dH = G weight runs as a bf16 GEMM)
"""
import os

import numpy as np
import pytest
import torch

import oracle as O
from _parity import knobs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jop():
    import monotonic_rnnt_joint
    # sweeps through another launch variant (development build): MRNNT_FUZZ_TUNE="joint_bwd_mfma=32,joint_reduce_sparse=2"
    kv = dict(x.split("=") for x in filter(None, os.environ.get("MRNNT_FUZZ_TUNE", "").split(",")))
    if not kv:
        yield monotonic_rnnt_joint
        return
    with knobs(**kv):
        yield monotonic_rnnt_joint


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def make_case(seed, B, Trange, Smax, H, V, scale_in=1.0):
    rng = np.random.default_rng(seed)
    T = rng.integers(Trange[0], Trange[1] + 1, B).astype(np.int32)
    S = np.array([rng.integers(0, min(t, Smax) + 1) for t in T], np.int32)
    Tm, Sm = int(T.max()), int(S.max())
    enc = torch.from_numpy(scale_in * rng.standard_normal((B, Tm + 1, H)).astype(np.float32)).to(torch.bfloat16)
    pred = torch.from_numpy(scale_in * rng.standard_normal((B, Sm + 2, H)).astype(np.float32)).to(torch.bfloat16)
    w = torch.from_numpy((rng.standard_normal((V, H)) / np.sqrt(H) * 2.0).astype(np.float32)).to(torch.bfloat16)
    bias = torch.from_numpy(0.1 * rng.standard_normal(V).astype(np.float32))
    labels = rng.integers(1, V, (B, max(1, Sm))).astype(np.int32)
    return enc, pred, w, bias, labels, T, S


def host_reference(enc, pred, w, bias, labels, T, S, blank=0, scale=None, alignment=None, k=0, extra=None):
    B = len(T)
    W64 = w.double()
    hs, rows = [], []
    for b in range(B):
        e = enc[b, : T[b]].float()
        p = pred[b, : S[b] + 1].float()
        h = torch.tanh(e[:, None, :] + p[None, :, :]).to(torch.bfloat16).double()  # [T, S+1, H]
        hs.append(h)
        rows.append((h @ W64.T + bias.double()).reshape(-1, w.shape[0]))
    acts = torch.cat(rows).float().numpy()
    costs, dz = O.oracle_rnnt(acts, labels, T, S, blank=blank, alignment=alignment, max_shift=k, num_threads=4)
    if scale is not None:
        dz = dz * np.repeat(np.asarray(scale, np.float64), T * (S + 1))[:, None]
    dz = torch.from_numpy(dz)
    if extra is not None:  # column sums of |dz|: what d_bias = sum_rows dz cancels from
        extra["dz_abs_colsum"] = dz.abs().sum(0)
    d_enc = torch.zeros(enc.shape, dtype=torch.float64)
    d_pred = torch.zeros(pred.shape, dtype=torch.float64)
    d_w = torch.zeros(w.shape, dtype=torch.float64)
    r = 0
    for b in range(B):
        n = int(T[b]) * (int(S[b]) + 1)
        g = dz[r:r + n]
        h = hs[b].reshape(n, -1)
        d_w += g.T @ h
        dpre = ((g @ W64) * (1 - h * h)).reshape(T[b], S[b] + 1, -1)
        d_enc[b, : T[b]] = dpre.sum(1)
        d_pred[b, : S[b] + 1] = dpre.sum(0)
        r += n
    return costs, d_enc, d_pred, d_w, dz.sum(0)


def close(x, ref, rel=1.5e-2, name=""):
    x = x.double().cpu()
    ref = ref.double()
    err = (x - ref).abs().max().item()
    lim = rel * ref.abs().max().item() + 1e-5
    assert err <= lim, (name, err, lim)


def run_joint(jop, dev, enc, pred, w, bias, labels, T, S, blank=0, scale=None, alignment=None, k=0):
    e = enc.to(dev).requires_grad_(True)
    p = pred.to(dev).requires_grad_(True)
    ww = w.to(dev).requires_grad_(True)
    bb = None if bias is None else bias.to(dev).requires_grad_(True)
    al = None if alignment is None else torch.from_numpy(alignment).to(dev)
    costs = jop.monotonic_rnnt_joint_loss(e, p, ww, bb, torch.from_numpy(labels).to(dev), torch.from_numpy(T),
                                          torch.from_numpy(S), blank, al, k)
    sc = torch.ones(len(T), device=dev) if scale is None else torch.tensor(scale, dtype=torch.float32, device=dev)
    (costs * sc).sum().backward()
    torch.cuda.synchronize()
    return costs.detach().cpu().double().numpy(), e.grad, p.grad, ww.grad, None if bb is None else bb.grad


@pytest.mark.parametrize("H,V", [(128, 64), (256, 100), (256, 1000), (512, 256), (384, 96), (640, 130)])
def test_joint_loss_and_grads_vs_host(jop, dev, H, V):
    enc, pred, w, bias, labels, T, S = make_case(H + V, 3, (1, 24), 8, H, V)
    scale = [1.0, -0.5, 2.0]
    c, de, dp, dw, db = run_joint(jop, dev, enc, pred, w, bias, labels, T, S, scale=scale)
    cr, de_r, dp_r, dw_r, db_r = host_reference(enc, pred, w, bias, labels, T, S, scale=scale)
    assert np.all(np.abs(c - cr) <= 1e-5 * np.maximum(1.0, np.abs(cr))), (c, cr)
    close(de, de_r, name="d_enc")
    close(dp, dp_r, name="d_pred")
    close(dw, dw_r, name="d_weight")
    close(db, db_r, name="d_bias")
    # padding frames / label slots beyond the lengths get exactly zero gradient
    for b in range(len(T)):
        assert torch.all(de[b, T[b]:] == 0) and torch.all(dp[b, S[b] + 1:] == 0)


def test_joint_blank_last_and_long_utterance(jop, dev):
    """blank = V-1, an utterance long enough that the occupancy skip removes rows from the backward pass."""
    H, V = 256, 64
    enc, pred, w, bias, labels, T, S = make_case(7, 2, (150, 200), 40, H, V, scale_in=2.0)
    labels = np.where(labels == V - 1, 1, labels).astype(np.int32)
    c, de, dp, dw, db = run_joint(jop, dev, enc, pred, w, bias, labels, T, S, blank=V - 1)
    cr, de_r, dp_r, dw_r, db_r = host_reference(enc, pred, w, bias, labels, T, S, blank=V - 1)
    assert np.all(np.abs(c - cr) <= 1e-5 * np.maximum(1.0, np.abs(cr))), (c, cr)
    close(de, de_r, name="d_enc")
    close(dp, dp_r, name="d_pred")
    close(dw, dw_r, name="d_weight")
    close(db, db_r, name="d_bias")


def test_joint_matches_materialised_acts_path(jop, dev):
    """The fused op equals monotonic_rnnt_loss on the logits it never materialises (costs; same bf16 h up to
    rare tanh rounding flips), cost-only forward included."""
    import monotonic_rnnt_op as op
    H, V = 256, 256
    enc, pred, w, bias, labels, T, S = make_case(11, 4, (5, 40), 12, H, V)
    c_fused = jop.monotonic_rnnt_joint_loss(enc.to(dev), pred.to(dev), w.to(dev), bias.to(dev),
                                            torch.from_numpy(labels).to(dev), torch.from_numpy(T),
                                            torch.from_numpy(S)).cpu().double().numpy()
    rows = []
    for b in range(len(T)):
        e = enc[b, : T[b]].to(dev).float()
        p = pred[b, : S[b] + 1].to(dev).float()
        h = torch.tanh(e[:, None] + p[None]).to(torch.bfloat16).float()
        rows.append((h @ w.to(dev).float().T + bias.to(dev)).reshape(-1, V))
    acts = torch.cat(rows).contiguous()
    c_acts = op.monotonic_rnnt_loss(acts, torch.from_numpy(labels).to(dev), torch.from_numpy(T),
                                    torch.from_numpy(S)).cpu().double().numpy()
    assert np.all(np.abs(c_fused - c_acts) <= 1e-3 * np.maximum(1.0, np.abs(c_acts))), (c_fused, c_acts)


def random_joint_case(seed):
    rng = np.random.default_rng(7000 + seed)
    H = int(rng.choice([128, 256, 384, 512, 640]))
    V = int(rng.choice([2, 3, 17, 32, 64, 100, 130, 256, 1000, 1030]))
    B = int(rng.integers(1, 5))
    big = os.environ.get("MRNNT_JOINT_BIG") == "1"  # long utterances: occupancy skip, many row tiles
    t_caps, s_caps = ([100, 200], [20, 60, 90]) if big else ([8, 30, 60], [0, 4, 12, 30])
    enc, pred, w, bias, labels, T, S = make_case(int(rng.integers(1 << 30)), B, (1, int(rng.choice(t_caps))),
                                                 int(rng.choice(s_caps)), H, V,
                                                 scale_in=float(rng.choice([0.5, 1.0, 2.0])))
    if rng.random() < 0.3:  # T = S somewhere
        T[0] = max(int(S[0]), 1)
    blank = int(rng.integers(0, V))
    labels = rng.integers(0, V, labels.shape).astype(np.int32)
    if rng.random() < 0.7:
        labels[labels == blank] = (blank + 1) % V
    if rng.random() < 0.25:
        bias = None
    scale = rng.choice([1.0, -0.5, 0.0, 2.0], B).tolist()
    al, k = None, 0
    if rng.random() < 0.3:
        k = int(rng.integers(0, 4))
        al = np.full((B, int(T.max())), blank, np.int32)
        for b in range(B):
            fr = np.sort(rng.choice(int(T[b]), int(S[b]), replace=False))
            al[b, fr] = np.where(labels[b, : S[b]] == blank, (blank + 1) % V, labels[b, : S[b]])
    return enc, pred, w, bias, labels, T, S, blank, scale, al, k


@pytest.mark.parametrize("seed", range(int(os.environ.get("MRNNT_FUZZ_FIRST", "0")),
                                  int(os.environ.get("MRNNT_FUZZ_FIRST", "0")) + int(os.environ.get("MRNNT_JOINT_CASES", "32"))))
def test_joint_random_cases(jop, dev, seed):
    """Seeded sweep over the fused path's switches: every supported H, V with and without a tail chunk (V < 32
    included), blank anywhere, labels that may equal the blank, no bias, ragged lengths with S = 0 and T = S,
    alignment restriction, negative / zero gradient scales."""
    enc, pred, w, bias, labels, T, S, blank, scale, al, k = random_joint_case(seed)
    B, V = len(T), w.shape[0]
    c, de, dp, dw, db = run_joint(jop, dev, enc, pred, w, bias, labels, T, S, blank=blank, scale=scale,
                                  alignment=al, k=k)
    bias_ref = torch.zeros(V) if bias is None else bias
    ex = {}
    cr, de_r, dp_r, dw_r, db_r = host_reference(enc, pred, w, bias_ref, labels, T, S, blank=blank, scale=scale,
                                                alignment=al, k=k, extra=ex)
    fin = np.isfinite(cr)
    assert np.array_equal(np.isfinite(c), fin), (c, cr)
    assert np.all(np.abs(c[fin] - cr[fin]) <= 1e-5 * np.maximum(1.0, np.abs(cr[fin]))), (c, cr)
    close(de, de_r, name="d_enc")
    close(dp, dp_r, name="d_pred")
    close(dw, dw_r, name="d_weight")
    if bias is not None:
        # d_bias sums G (stored as bf16) over rows: with V = 2 or 3 it can cancel to ~1 % of sum |G|, so the bound
        # adds two bf16 roundings of that sum (found by the 400-case sweep, seeds 223 / 334: V = 2)
        lim = 1.5e-2 * db_r.abs().max().item() + 2.0 ** -8 * ex["dz_abs_colsum"].max().item() + 1e-5
        err = (db.double().cpu() - db_r).abs().max().item()
        assert err <= lim, ("d_bias", err, lim)
    for b in range(B):
        assert torch.all(de[b, T[b]:] == 0) and torch.all(dp[b, S[b] + 1:] == 0)


@pytest.mark.parametrize("k", [0, 2])
def test_joint_alignment_restricted(jop, dev, k):
    """alignment / max_distance_from_alignment on the fused path, against the oracle's restricted loss."""
    H, V = 256, 64
    enc, pred, w, bias, labels, T, S = make_case(50 + k, 3, (10, 40), 8, H, V)
    rng = np.random.default_rng(k)
    al = np.zeros((3, int(T.max())), np.int32)
    for b in range(3):
        al[b, np.sort(rng.choice(T[b], S[b], replace=False))] = labels[b, : S[b]]
    c, de, dp, dw, db = run_joint(jop, dev, enc, pred, w, bias, labels, T, S, alignment=al, k=k)
    cr, de_r, dp_r, dw_r, db_r = host_reference(enc, pred, w, bias, labels, T, S, alignment=al, k=k)
    assert np.all(np.abs(c - cr) <= 1e-5 * np.maximum(1.0, np.abs(cr))), (c, cr)
    close(de, de_r, name="d_enc")
    close(dp, dp_r, name="d_pred")
    close(dw, dw_r, name="d_weight")
    close(db, db_r, name="d_bias")


@pytest.mark.parametrize("H,V", [(512, 256), (256, 1000), (128, 64), (384, 130), (640, 64)])
def test_joint_gradients_bitwise_reproducible(dev, H, V):
    """Two calls on the same inputs give the same bits in the costs and in every gradient: the
    column sums of d_bias and the d_pred sums over frames are fixed-order reductions (per-workgroup partials, then
    one ordered pass), not float atomics, as the reference's own op is deterministic."""
    import monotonic_rnnt_joint as jm
    enc, pred, w, bias, labels, T, S = make_case(7 + H, 5, (10, 60), 20, H, V)
    ref = run_joint(jm, dev, enc, pred, w, bias, labels, T, S)
    for _ in range(2):
        got = run_joint(jm, dev, enc, pred, w, bias, labels, T, S)
        assert np.array_equal(ref[0], got[0])
        for a, b in zip(ref[1:], got[1:]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("tile", ["joint_bwd_mfma=32"])
@pytest.mark.parametrize("H,V,blank", [(512, 1024, 517), (512, 1000, 0), (256, 17, 16), (128, 64, 37), (384, 130, 129),
                                       (256, 2, 1)])
def test_joint_tile_variants_vs_host(dev, H, V, blank, tile):
    """The launch variant of the development build against the host reference at this file's tolerances:
    joint_bwd_mfma = 32 (the backward on the 32x32x16 tile, which H = 640 runs anyway). Blank and labels in every lane
    group and vocabulary tile, tail chunks (V = 1000, 130, 17, 2), ragged rows past the list end."""
    import monotonic_rnnt_joint as jm
    enc, pred, w, bias, labels, T, S = make_case(31 + H + V, 4, (10, 50), 16, H, V)
    labels = np.where(labels == blank, (blank + 1) % V, labels).astype(np.int32)
    scale = [1.0, -0.5, 2.0, 0.25]
    k, v = tile.split("=")
    with knobs(**{k: int(v)}):
        c, de, dp, dw, db = run_joint(jm, dev, enc, pred, w, bias, labels, T, S, blank=blank, scale=scale)
    cr, de_r, dp_r, dw_r, db_r = host_reference(enc, pred, w, bias, labels, T, S, blank=blank, scale=scale)
    assert np.all(np.abs(c - cr) <= 1e-5 * np.maximum(1.0, np.abs(cr))), (c, cr)
    close(de, de_r, name="d_enc")
    close(dp, dp_r, name="d_pred")
    close(dw, dw_r, name="d_weight")
    close(db, db_r, name="d_bias")
    for b in range(len(T)):
        assert torch.all(de[b, T[b]:] == 0) and torch.all(dp[b, S[b] + 1:] == 0)


@pytest.mark.parametrize("H,V,ld", [(512, 1024, 512), (256, 1000, 256), (512, 1000, 520), (256, 1024, 288)])
def test_joint_dpre_kernel_vs_torch(jop, dev, H, V, ld):
    """mrnnt_joint_dpre (hand-written MFMA GEMM, mrnnt_joint_gemm.hip) against torch on the same bf16 operands:
    dpre = (G W) * (1 - Hact^2) over 3,000 rows (11+ row tiles, the last partial), V with and without a partial last
    k-chunk, Hact with a wider row stride. Tolerance: the bf16 rounding of the output (2^-8 relative) plus fp32
    accumulation-order noise, stated as |d - ref| <= 2^-7 |ref| + 1e-3 max|ref|."""
    enc, pred, w, _, labels, T, S = make_case(7, 4, (150, 200), 60, H, V)
    prep = jop._JointPrepared(enc.to(dev), pred.to(dev), w.to(dev), None, torch.from_numpy(labels).to(dev),
                              torch.from_numpy(T), torch.from_numpy(S), 0)
    n = 3000
    g = torch.Generator(device=dev).manual_seed(H + V + ld)
    G = (torch.randn(n, V, device=dev, generator=g) * 1e-2).to(torch.bfloat16)
    Hw = torch.tanh(torch.randn(n, ld, device=dev, generator=g)).to(torch.bfloat16)
    prep.problem.hact_ld = ld
    out = prep.dpre(G, Hw)
    torch.cuda.synchronize()
    h = Hw[:, :H].float()
    ref = (G.float() @ prep.weight.float()) * (1.0 - h * h)
    err = (out.float() - ref).abs()
    lim = 2.0 ** -7 * ref.abs() + 1e-3 * ref.abs().max()
    assert bool((err <= lim).all()), (err.max().item(), ref.abs().max().item())
    # bit-for-bit repeatable
    assert torch.equal(prep.dpre(G, Hw), out)


@pytest.mark.parametrize("nw", [0, 1, 2, 8, 81, 42, 421, 431, 851, 160, 161, 162, 163, 164, 165, 166, 167])
@pytest.mark.parametrize("H,V,ld", [(512, 1024, 512), (256, 1000, 288)])
def test_joint_dpre_variants_vs_torch(jop, dev, nw, H, V, ld):
    """Every launch variant of mrnnt_joint_dpre (development build, knob joint_dpre_nw: tile shapes, LDS stages, the
    LDS-staged epilogue, the 16x16x32 forms) against torch on the same operands, as above, over 5,000 rows (a partial
    last row tile of every tile height); the 32x32x16 staged forms equal each other bit for bit (same fragments, same
    k order)."""
    enc, pred, w, _, labels, T, S = make_case(9, 4, (150, 200), 60, H, V)
    prep = jop._JointPrepared(enc.to(dev), pred.to(dev), w.to(dev), None, torch.from_numpy(labels).to(dev),
                              torch.from_numpy(T), torch.from_numpy(S), 0)
    n = 5000
    g = torch.Generator(device=dev).manual_seed(H + V + ld + 1)
    G = (torch.randn(n, V, device=dev, generator=g) * 1e-2).to(torch.bfloat16)
    Hw = torch.tanh(torch.randn(n, ld, device=dev, generator=g)).to(torch.bfloat16)
    prep.problem.hact_ld = ld
    with knobs(joint_dpre_nw=nw):
        out = prep.dpre(G, Hw)
        again = prep.dpre(G, Hw)
    with knobs(joint_dpre_nw=8):
        staged = prep.dpre(G, Hw)
    torch.cuda.synchronize()
    h = Hw[:, :H].float()
    ref = (G.float() @ prep.weight.float()) * (1.0 - h * h)
    err = (out.float() - ref).abs()
    lim = 2.0 ** -7 * ref.abs() + 1e-3 * ref.abs().max()
    assert bool((err <= lim).all()), (nw, err.max().item(), ref.abs().max().item())
    assert torch.equal(again, out)
    if nw in (8, 81, 42, 421, 431, 851):
        assert torch.equal(staged, out)


def test_joint_dpre_path_matches_library_gemm_path(jop, dev, monkeypatch):
    """The backward through mrnnt_joint_dpre + the reduce on dpre equals the hipBLASLt dH + reduce-with-Hact path
    within the bf16 rounding of dH / dpre (both against the same fp64 host reference: test above; here path vs path)."""
    enc, pred, w, bias, labels, T, S = make_case(11, 3, (40, 70), 20, 512, 256)
    outs = []
    for blas in (False, True):
        monkeypatch.setattr(jop, "_DH_BLAS", blas)
        outs.append(run_joint(jop, dev, enc, pred, w, bias, labels, T, S, scale=[1.0, 0.5, -1.0]))
    (c0, de0, dp0, dw0, db0), (c1, de1, dp1, dw1, db1) = outs
    assert np.array_equal(c0, c1)
    assert torch.equal(dw0, dw1) and torch.equal(db0, db1)  # dW / dbias do not depend on the dH path
    for x, y, name in ((de0, de1, "d_enc"), (dp0, dp1, "d_pred")):
        err = (x.float() - y.float()).abs().max().item()
        assert err <= 1e-2 * y.float().abs().max().item() + 1e-6, (name, err)


@pytest.mark.parametrize("H,V", [(512, 256), (256, 1000), (128, 64), (640, 130)])
def test_joint_reduce_recomputed_activation_is_bit_identical(jop, dev, H, V):
    """The reduce recomputes tanh(enc + pred) with the gradient pass's own function instead of reading Hact (halving
    its bytes): d_enc / d_pred equal the Hact-reading form (development build, joint_reduce_hact = 1) bit for bit."""
    enc, pred, w, bias, labels, T, S = make_case(H + 3 * V, 3, (30, 60), 20, H, V)
    with knobs(joint_reduce_hact=0):
        _, de0, dp0, dw0, _ = run_joint(jop, dev, enc, pred, w, bias, labels, T, S)
    with knobs(joint_reduce_hact=1):
        _, de1, dp1, dw1, _ = run_joint(jop, dev, enc, pred, w, bias, labels, T, S)
    assert torch.equal(de0, de1) and torch.equal(dp0, dp1) and torch.equal(dw0, dw1)


@pytest.mark.parametrize("H,V,S_max", [(512, 256, 100), (256, 1000, 20), (640, 130, 90), (128, 64, 5)])
def test_joint_reduce_padded_pitch_bit_identical(jop, dev, H, V, S_max):
    """The reduce's accumulators at LDS pitch HS + 1 (default, bank-conflict-free) equal pitch HS (development build,
    joint_reduce_pad = 0) bit for bit: only the layout differs, every sum keeps its order."""
    enc, pred, w, bias, labels, T, S = make_case(H + V + S_max, 3, (max(30, S_max - 10), S_max + 31), S_max, H, V)
    with knobs(joint_reduce_pad=0):
        _, de0, dp0, dw0, _ = run_joint(jop, dev, enc, pred, w, bias, labels, T, S)
    with knobs(joint_reduce_pad=1):
        _, de1, dp1, dw1, _ = run_joint(jop, dev, enc, pred, w, bias, labels, T, S)
    assert torch.equal(de0, de1) and torch.equal(dp0, dp1) and torch.equal(dw0, dw1)



def _check_vs_host(jop, dev, enc, pred, w, bias, labels, T, S, blank=0, cost_rel=1e-5):
    scale = [1.0, -0.5, 2.0][: len(T)]
    c, de, dp, dw, db = run_joint(jop, dev, enc, pred, w, bias, labels, T, S, blank=blank, scale=scale)
    cr, de_r, dp_r, dw_r, db_r = host_reference(enc, pred, w, bias, labels, T, S, blank=blank, scale=scale)
    assert np.all(np.isfinite(c)), c
    assert np.all(np.abs(c - cr) <= cost_rel * np.maximum(1.0, np.abs(cr))), (c, cr)
    close(de, de_r, name="d_enc")
    close(dp, dp_r, name="d_pred")
    close(dw, dw_r, name="d_weight")
    if bias is not None:
        close(db, db_r, name="d_bias")


@pytest.mark.parametrize("H,V", [(512, 1000), (256, 130)])
def test_joint_unbounded_weights_take_the_running_max(jop, dev, H, V):
    """The forward sums exp(z) without a running max only when the device-side weight bound max_v (sum |W_v| + |b_v|)
    is <= 64 (every |z| <= 64 since |tanh| <= 1: no fp32 overflow). Weights 50 / sqrt(H) put logits near +-170 --
    e^170 overflows fp32 -- so the bound fails and the online log-sum-exp must run: costs finite and on the host
    reference. Tolerance: costs 1e-5 relative (as above; the costs here are O(1e3))."""
    enc, pred, w, bias, labels, T, S = make_case(H + V + 5, 3, (10, 40), 12, H, V)
    w = (w.float() * 25.0).to(torch.bfloat16)
    _check_vs_host(jop, dev, enc, pred, w, bias, labels, T, S)


@pytest.mark.parametrize("over", [False, True])
def test_joint_weight_bound_edge(jop, dev, over):
    """Logits at exactly +-64 (saturated tanh, weight rows of +-1/8 at H = 512: sum |W_v| = 64, the bound's edge, the
    plain exp-sum path) and the same weights with |bias| = 0.5 (bound 64.5: the running-max path): both on the host
    reference (costs 1e-5 relative)."""
    H, V = 512, 1024
    enc, pred, w, bias, labels, T, S = make_case(3 + over, 3, (10, 30), 10, H, V)
    enc = torch.full_like(enc, 8.0)  # tanh(8 + pred) rounds to 1 in bf16 for |pred| < ~4
    pred = pred.clamp(-3.0, 3.0)
    sign = torch.where(torch.arange(V) % 3 == 0, 1.0, -1.0)
    w = (sign[:, None] * torch.full((V, H), 0.125)).to(torch.bfloat16)
    bias = torch.full((V,), 0.5 if over else 0.0)
    _check_vs_host(jop, dev, enc, pred, w, bias, labels, T, S)


@pytest.mark.parametrize("H,V", [(512, 1024), (256, 1000), (640, 130)])
def test_joint_plain_exp_sum_matches_running_max(dev, H, V):
    """Bounded weights: the plain exp-sum forward (product) against the running-max epilogue forced on (development
    build, joint_probe bit 3) on the same inputs: costs within 1e-6 relative (the two fp32 sums differ only in
    rounding), gradients within 2^-7 of their max (bf16 logit-gradient rounding can flip)."""
    import monotonic_rnnt_joint as jm
    enc, pred, w, bias, labels, T, S = make_case(H * 3 + V, 3, (20, 60), 20, H, V)
    a = run_joint(jm, dev, enc, pred, w, bias, labels, T, S, scale=[1.0, -0.5, 2.0])
    with knobs(joint_probe=8):
        b = run_joint(jm, dev, enc, pred, w, bias, labels, T, S, scale=[1.0, -0.5, 2.0])
    assert np.all(np.abs(a[0] - b[0]) <= 1e-6 * np.maximum(1.0, np.abs(b[0]))), (a[0], b[0])
    for x, y, name in zip(a[1:], b[1:], ("d_enc", "d_pred", "d_weight", "d_bias")):
        err = (x.float() - y.float()).abs().max().item()
        assert err <= 2.0 ** -7 * y.float().abs().max().item() + 1e-6, (name, err)


def _joint_step(jm, enc, pred, w, bias, labels, T, S, capturable):
    """costs.sum().backward() of the fused op on leaf tensors; returns (costs, d_enc, d_pred, d_weight, d_bias)."""
    for x in (enc, pred, w, bias):
        x.grad = None
    costs = jm.monotonic_rnnt_joint_loss(enc, pred, w, bias, labels, T, S, capturable=capturable)
    costs.sum().backward()
    return (costs.detach().clone(), enc.grad.clone(), pred.grad.clone(), w.grad.clone(), bias.grad.clone())


@pytest.mark.parametrize("H,V", [(256, 128), (512, 256), (128, 64), (640, 130)])
def test_joint_step_graph_capture_replay(dev, H, V):
    """the joint backward reads no live-row count back to the host when capturable (row buffers
    and GEMMs sized by mrnnt_joint_row_bound, the kernels take the count from the device, rows past it zero), so a
    training step captures in torch.cuda.graph. Replays on new inputs equal an eager capturable step bit for bit;
    the capturable step agrees with the default (count read back) one at the fp32 rounding of the weight GEMM's
    split-K order; and it makes no device-to-host synchronisation at all."""
    import monotonic_rnnt_joint as jm
    enc0, pred0, w0, bias0, labels, T, S = make_case(31 + H, 4, (20, 50), 12, H, V)
    enc = enc0.to(dev).requires_grad_(True)
    pred = pred0.to(dev).requires_grad_(True)
    w = w0.to(dev).requires_grad_(True)
    bias = bias0.to(dev).requires_grad_(True)
    lab, Tt, St = torch.from_numpy(labels).to(dev), torch.from_numpy(T), torch.from_numpy(S)
    # the capturable step against the default one
    eager_cap = _joint_step(jm, enc, pred, w, bias, lab, Tt, St, True)
    eager = _joint_step(jm, enc, pred, w, bias, lab, Tt, St, False)
    assert torch.equal(eager_cap[0], eager[0])
    for a, b, name in zip(eager_cap[1:], eager[1:], ("d_enc", "d_pred", "d_weight", "d_bias")):
        close(a, b.double().cpu(), rel=1e-5, name=name)
    torch.cuda.synchronize()
    prev = torch.cuda.get_sync_debug_mode()
    torch.cuda.set_sync_debug_mode("error")  # any device-to-host read in the step raises
    try:
        _joint_step(jm, enc, pred, w, bias, lab, Tt, St, True)
    finally:
        torch.cuda.set_sync_debug_mode(prev)
    # capture (warm-up on a side stream first, as torch.cuda.graph asks), then replay on new inputs
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            _joint_step(jm, enc, pred, w, bias, lab, Tt, St, None)
    torch.cuda.current_stream().wait_stream(s)
    for x in (enc, pred, w, bias):
        x.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        costs = jm.monotonic_rnnt_joint_loss(enc, pred, w, bias, lab, Tt, St)  # capturable inside capture
        costs.sum().backward()
    gen = torch.Generator(device=dev).manual_seed(3)
    for i in range(3):
        with torch.no_grad():
            enc.copy_(torch.randn(enc.shape, device=dev, generator=gen).to(enc.dtype))
            pred.copy_(torch.randn(pred.shape, device=dev, generator=gen).to(pred.dtype))
        g.replay()
        torch.cuda.synchronize()
        got = (costs.detach().clone(), enc.grad.clone(), pred.grad.clone(), w.grad.clone(), bias.grad.clone())
        e2, p2 = enc.detach().clone().requires_grad_(True), pred.detach().clone().requires_grad_(True)
        w2, b2 = w.detach().clone().requires_grad_(True), bias.detach().clone().requires_grad_(True)
        ref = _joint_step(jm, e2, p2, w2, b2, lab, Tt, St, True)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)
