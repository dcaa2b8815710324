"""Seeded random sweep of the HIP path against the oracle (cpu_rnnt.h<double> restatement), across the shapes the
kernel variants switch on: V (vector width, chunking, FULL / ragged rows, V < 4, odd V), S+1 (single-wave /
halo / per-step-barrier recursion, gradient segments of 256 rows), blank anywhere in [0, V), labels that may equal
the blank, alignment restriction with random k, per-utterance gradient scales (negative and zero included),
packed and padded layouts, f32 / bf16 / f16 acts, host or device-resident lengths (round 4); then the same
generator through the other launch variants.
Tolerances as tests/test_gpu_parity.py (reduced precision: the grads tolerance adds one rounding of the acts type).
The sweep found the stale-workspace bug pinned by test_gpu_parity.py::test_stale_workspace_contents_do_not_matter.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O
from _parity import knobs

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("MRNNT_FUZZ_CASES", "160"))  # round-end suite: 160; long sweeps: set it higher
FIRST = int(os.environ.get("MRNNT_FUZZ_FIRST", "0"))
V_CHOICES = [int(v) for v in os.environ.get("MRNNT_FUZZ_V", "2,3,5,16,31,64,100,255,256,257,1000,1024,1030,2048").split(",")]
ACT_SCALES = [float(v) for v in os.environ.get("MRNNT_FUZZ_SCALE", "0.5,1,3").split(",")]  # logit spread
T_EXTRA = int(os.environ.get("MRNNT_FUZZ_T_EXTRA", "40"))  # frames beyond the label cap


@pytest.fixture(scope="module")
def op():
    import monotonic_rnnt_op
    # long sweeps through another launch variant (development build): MRNNT_FUZZ_TUNE="dp_halo=0,grad_variant=3"
    kv = dict(x.split("=") for x in filter(None, os.environ.get("MRNNT_FUZZ_TUNE", "").split(",")))
    if not kv:
        yield monotonic_rnnt_op
        return
    with knobs(**kv):
        yield monotonic_rnnt_op


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


def make_case(seed):
    rng = np.random.default_rng(1000 + seed)
    V = int(rng.choice(V_CHOICES))
    B = int(rng.integers(1, 5))
    # label lengths across the recursion's shapes: <= 63, halo (64 .. 447), per-step barrier (>= 448)
    s_cap = int(rng.choice([8, 60, 130, 250, 460]))
    if V >= 1000:
        s_cap = min(s_cap, 130)  # keep the oracle's work small
    if V >= 4000:
        s_cap = min(s_cap, 40)
    T = rng.integers(1, s_cap + T_EXTRA, B).astype(np.int32)
    S = np.array([rng.integers(0, min(int(t), s_cap) + 1) for t in T], np.int32)
    blank = int(rng.integers(0, V))
    L = max(1, int(S.max()))
    labels = rng.integers(0, V, (B, L)).astype(np.int32)
    if rng.random() < 0.7:  # mostly labels != blank, as in training data
        labels[labels == blank] = (blank + 1) % V if V > 1 else blank
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = (rng.standard_normal((rows, V)) * rng.choice(ACT_SCALES)).astype(np.float32)
    scale = rng.choice([1.0, -0.5, 0.0, 2.0, 0.25], B).astype(np.float32)
    align, k = None, 0
    if rng.random() < 0.3:
        k = int(rng.integers(0, 6))
        align = np.full((B, int(T.max())), blank, np.int32)
        for b in range(B):
            fr = np.sort(rng.choice(int(T[b]), int(S[b]), replace=False))
            align[b, fr] = labels[b, : S[b]]
            # the alignment's labels are parsed by != blank: keep them distinct from the blank
            align[b, fr[align[b, fr] == blank]] = (blank + 1) % V
    dtype = rng.choice(["f32"] * 6 + ["bf16", "f16"])
    padded = bool(rng.random() < 0.25)
    # the reference's calling convention (lengths on the device, monotonic_rnnt.cu:85-88): planned from bounds and
    # validated on the GPU, the chase launch included (drawn last: earlier fields keep their seeds' values)
    dev_lengths = bool(rng.random() < 0.4)
    return dict(V=V, T=T, S=S, blank=blank, labels=labels, acts=acts, scale=scale, align=align, k=k,
                dtype=str(dtype), padded=padded, dev_lengths=dev_lengths)


def pad(acts, T, S, pad_T, pad_S1):
    B, V = len(T), acts.shape[1]
    out = np.full((B, pad_T, pad_S1, V), np.nan, np.float32)
    r = 0
    for b in range(B):
        n = int(T[b]) * (int(S[b]) + 1)
        out[b, : T[b], : S[b] + 1] = acts[r: r + n].reshape(T[b], S[b] + 1, V)
        r += n
    return out


def unpad(x, T, S):
    return np.concatenate([x[b, : T[b], : S[b] + 1].reshape(-1, x.shape[-1]) for b in range(len(T))])


@pytest.mark.parametrize("seed", range(FIRST, FIRST + N_CASES))
def test_random_case_vs_oracle(op, dev, seed):
    check_case(op, dev, make_case(seed), cost_only_too=(seed % 4 == 0))


KNOB_SETS = [
    {"dp_halo": 0},                                  # per-step-barrier recursion at every S
    {"dp_halo": 2},                                  # log-domain halo recursion
    {"softmax_variant": 0, "grad_variant": 2},       # first log-softmax, per-row gradient
    {"grad_variant": 3, "nt_load": 0, "nt_store": 0},  # row-sweep gradient, plain loads / stores
    {"softmax_variant": 14, "grad_variant": 6, "col_scatter": 0},
    {"occ_skip": 0, "softmax_variant": 15},
]


@pytest.mark.parametrize("knob_set", range(len(KNOB_SETS)))
@pytest.mark.parametrize("seed", range(1000, 1024))
def test_random_case_other_kernels(op, dev, knob_set, seed):
    """The same sweep through the other launch variants (development build, mrnnt_tune), 24 cases each."""
    with knobs(**KNOB_SETS[knob_set]):
        check_case(op, dev, make_case(seed))


@pytest.mark.parametrize("B,V,dtype", [(300, 16, "f32"), (1000, 33, "f32"), (257, 64, "bf16")])
def test_many_utterances(op, dev, B, V, dtype):
    """Batches wider than the setup scan's 64-lane chunks, with T = 1 / S = 0 utterances among them."""
    rng = np.random.default_rng(B)
    T = rng.integers(1, 30, B).astype(np.int32)
    T[:3] = 1
    S = np.array([rng.integers(0, t + 1) for t in T], np.int32)
    S[1] = 0
    labels = rng.integers(1, V, (B, max(1, int(S.max())))).astype(np.int32)
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = rng.standard_normal((rows, V)).astype(np.float32)
    c = dict(V=V, T=T, S=S, blank=0, labels=labels, acts=acts, scale=rng.choice([1.0, -0.5], B).astype(np.float32),
             align=None, k=0, dtype=dtype, padded=False)
    check_case(op, dev, c, cost_only_too=True)


def test_more_utterances_than_grid_y_with_alignment(op, dev):
    """B = 70000 > 65535 (the largest grid y dimension, which the alignment band kernel walks) with alignment."""
    rng = np.random.default_rng(70000)
    B, V = 70000, 4
    T = rng.integers(1, 4, B).astype(np.int32)
    S = np.array([rng.integers(0, t + 1) for t in T], np.int32)
    labels = rng.integers(1, V, (B, max(1, int(S.max())))).astype(np.int32)
    align = np.zeros((B, int(T.max())), np.int32)
    for b in range(B):
        align[b, np.sort(rng.choice(int(T[b]), int(S[b]), replace=False))] = labels[b, : S[b]]
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = rng.standard_normal((rows, V)).astype(np.float32)
    c = dict(V=V, T=T, S=S, blank=0, labels=labels, acts=acts, scale=np.ones(B, np.float32), align=align, k=1,
             dtype="f32", padded=False)
    check_case(op, dev, c)


def test_more_columns_than_a_32bit_dispatch(op, dev):
    """17 M lattice columns: one 256-thread workgroup per column would be 4.4 G work-items, past the 32-bit
    dispatch size; the streaming kernels cap their grid and walk the columns grid-stride."""
    rng = np.random.default_rng(17)
    B, V = 17000, 4
    T = np.full(B, 1000, np.int32)
    S = (rng.random(B) < 0.01).astype(np.int32)  # mostly S = 0, a few S = 1
    labels = rng.integers(1, V, (B, 1)).astype(np.int32)
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = rng.standard_normal((rows, V)).astype(np.float32)
    c = dict(V=V, T=T, S=S, blank=0, labels=labels, acts=acts, scale=np.ones(B, np.float32), align=None, k=0,
             dtype="f32", padded=False)
    check_case(op, dev, c)


@pytest.mark.parametrize("V,dtype", [(65539, "f32"), (100000, "f32"), (131072, "bf16")])
def test_very_large_vocabulary(op, dev, V, dtype):
    """Vocabularies far past the benchmark's 10000 (many chunks per row; V odd: the scalar kernels)."""
    rng = np.random.default_rng(V)
    T = np.array([7, 4, 1], np.int32)
    S = np.array([3, 4, 0], np.int32)
    blank = int(rng.integers(0, V))
    labels = rng.integers(0, V, (3, 4)).astype(np.int32)
    labels[labels == blank] = (blank + 1) % V
    rows = int(np.sum(T * (S + 1)))
    acts = (rng.standard_normal((rows, V)) * 2.0).astype(np.float32)
    c = dict(V=V, T=T, S=S, blank=blank, labels=labels, acts=acts, scale=np.array([1.0, -0.5, 2.0], np.float32),
             align=None, k=0, dtype=dtype, padded=False)
    check_case(op, dev, c, cost_only_too=True)


def check_case(op, dev, c, cost_only_too=False):
    T, S, V = c["T"], c["S"], c["V"]
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[c["dtype"]]
    a = torch.from_numpy(c["acts"]).to(tdt)
    host = a.float().numpy()  # the exact values the kernels read
    if c["padded"]:
        a = torch.from_numpy(pad(host, T, S, int(T.max()) + 2, int(S.max()) + 3)).to(tdt)
    a = a.to(dev).requires_grad_(True)
    lab = torch.from_numpy(c["labels"]).to(dev)
    al = None if c["align"] is None else torch.from_numpy(c["align"]).to(dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    if c.get("dev_lengths"):
        Tt, St = Tt.to(dev), St.to(dev)
    costs = op.monotonic_rnnt_loss(a, lab, Tt, St, al, c["k"], c["blank"])
    (costs * torch.from_numpy(c["scale"]).to(dev)).sum().backward()
    g = a.grad.float().cpu().numpy()
    if c["padded"]:
        pad_rows = np.ones(g.shape[:3], bool)
        for b in range(len(T)):
            pad_rows[b, : T[b], : S[b] + 1] = False
        assert np.all(g[pad_rows] == 0.0)  # padding rows of the gradient are zero
        g = unpad(g, T, S)
    cr, gr = O.oracle_rnnt(host, c["labels"], T, S, blank=c["blank"], alignment=c["align"], max_shift=c["k"],
                           num_threads=8)
    gr = gr * np.repeat(c["scale"].astype(np.float64), T.astype(np.int64) * (S + 1))[:, None]
    cc = costs.detach().float().cpu().numpy().astype(np.float64)
    fin = np.isfinite(cr)
    assert np.array_equal(np.isfinite(cc), fin), (cc, cr)
    if fin.any():
        err = np.abs(cc[fin] - cr[fin]) / np.maximum(1.0, np.abs(cr[fin]))
        assert err.max() <= 1e-4, (err.max(), cc, cr)
    gfin = np.isfinite(gr)
    assert np.array_equal(np.isfinite(g), gfin)
    rel = {"f32": 0.0, "bf16": 2.0 ** -8, "f16": 2.0 ** -11}[c["dtype"]]
    tol = 1e-4 + rel * np.abs(gr[gfin])
    assert np.all(np.abs(g[gfin] - gr[gfin]) <= tol), np.abs(g[gfin] - gr[gfin]).max()
    if cost_only_too:  # the cost-only forward (no beta pass) gives the same costs bit for bit
        c2 = op.monotonic_rnnt_loss(a.detach(), lab, Tt, St, al, c["k"], c["blank"])
        assert np.array_equal(c2.float().cpu().numpy().astype(np.float64), cc)
