"""The chase launch (mrnnt_chase.hip): log-softmax and alpha / beta recursion in one launch, the
recursion workgroups consuming each lattice column as its log-softmax workgroup publishes it (write-through rows +
a ready flag per column, Guideline 16 R1). The reference runs the two back to back (gpu_rnnt.h:99-191).

Every value the chase computes is the one the two-kernel path computes, so the tests compare bit for bit against
the development build with the chase off (chase = 0), over every log-softmax body the chase carries (16-lane rows,
single-chunk U = 2 / 4, full and partial chunks), both recursion shapes (one wave, 4-wave halo with idle waves),
both prefetch depths, both acts load policies, ragged / odd / T = 1 / S = 0 lattices, the padded layout, forward
only (alpha alone), HIP-graph replay (flags cleared by the memset node each replay) and two streams at once.
"""
import numpy as np
import pytest
import torch

import oracle as O
from _parity import assert_costs, assert_grads, knobs, random_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def op():
    import monotonic_rnnt_op
    return monotonic_rnnt_op


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


def _run(op, acts, labels, T, S, grad=True, scale=None):
    if not grad:
        with torch.no_grad():
            c = op.monotonic_rnnt_loss(acts, labels, T, S)
        torch.cuda.synchronize()
        return c, None
    a = acts.detach().clone().requires_grad_(True)
    c = op.monotonic_rnnt_loss(a, labels, T, S)
    w = scale if scale is not None else torch.ones_like(c)
    (c * w).sum().backward()
    torch.cuda.synchronize()
    return c.detach(), a.grad.detach()


def _launches(fn):
    import _mrnnt_lib as L
    L.profile_enable(True)
    try:
        fn()
        prof = L.profile_read()
    finally:
        L.profile_enable(False)
    return {k: n for k, (_, n) in prof.items()}


CASES = {
    # name: (seed, B, T range, S max, V, force {b: (T, S)})
    "c2_row16_one_wave": (1, 16, (200, 200), 40, 256, {b: (200, 40) for b in range(16)}),
    "ragged_row16_t1_s0": (2, 7, (1, 90), 50, 128, {0: (1, 0), 3: (1, 1), 5: (37, 0)}),
    "v100_row16_odd_t": (3, 5, (21, 61), 30, 100, {1: (21, 21), 2: (61, 3)}),
    "halo_u2_full_idle_waves": (4, 3, (150, 260), 200, 512, {0: (259, 200), 1: (151, 30), 2: (200, 120)}),
    "halo_u2_partial": (5, 3, (100, 140), 150, 400, {0: (140, 150 - 11)}),
    "halo_u4_full": (6, 2, (120, 180), 180, 1024, {0: (179, 180 - 1)}),
    "u4_partial_one_wave": (7, 4, (30, 70), 60, 800, {}),
    "u4_partial_v1000": (8, 3, (40, 80), 63, 1000, {2: (80, 63)}),
}


def _problem(name, dev):
    seed, B, Tr, Smax, V, force = CASES[name]
    rng = np.random.default_rng(seed)
    acts, labels, T, S = random_problem(rng, B, Tr, Smax, V, force=force)
    return acts, labels, T, S, torch.from_numpy(acts).to(dev), torch.from_numpy(labels).to(dev)


def _assert_same(a, b):
    ca, ga = a
    cb, gb = b
    assert torch.equal(ca.view(torch.int32), cb.view(torch.int32))
    if ga is not None:
        assert torch.equal(ga.view(torch.int32), gb.view(torch.int32))


@pytest.mark.parametrize("depth", [16, 8])
@pytest.mark.parametrize("name", list(CASES))
def test_chase_bit_identical_to_two_kernels(op, dev, name, depth):
    acts, labels, T, S, a, lab = _problem(name, dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    scale = torch.linspace(0.5, 2.0, len(T), device=dev)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St, scale=scale)
    with knobs(chase=1, chase_depth=depth):
        n = _launches(lambda: _run(op, a, lab, Tt, St, scale=scale))
        got = _run(op, a, lab, Tt, St, scale=scale)
    assert n["chase"] == 1 and n["log_softmax"] == 0 and n["alpha_beta"] == 0, n
    _assert_same(got, ref)
    if name.startswith("c2") or name.startswith("ragged"):
        cr, gr = O.oracle_rnnt(acts, labels, T, S)
        assert_costs(got[0].cpu().numpy().astype(np.float64), cr)
        w = np.repeat(scale.cpu().numpy().astype(np.float64), T.astype(np.int64) * (S + 1))[:, None]
        assert_grads(got[1].cpu().numpy(), gr * w)


@pytest.mark.parametrize("nt_load", [0, 1])
def test_chase_both_acts_load_policies(op, dev, nt_load):
    _, _, T, S, a, lab = _problem("halo_u2_full_idle_waves", dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=0, nt_load=nt_load):
        ref = _run(op, a, lab, Tt, St)
    with knobs(chase=1, nt_load=nt_load):
        got = _run(op, a, lab, Tt, St)
    _assert_same(got, ref)


def test_chase_forward_only_alpha_alone(op, dev):
    """No gradient wanted: B recursion workgroups (alpha), production in frame order."""
    _, _, T, S, a, lab = _problem("ragged_row16_t1_s0", dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St, grad=False)
    n = _launches(lambda: _run(op, a, lab, Tt, St, grad=False))
    got = _run(op, a, lab, Tt, St, grad=False)
    assert n["chase"] == 1, n
    _assert_same(got, ref)


def test_chase_padded_layout(op, dev):
    acts, labels, T, S, _, lab = _problem("v100_row16_odd_t", dev)
    B, V = len(T), acts.shape[1]
    pad = np.zeros((B, int(T.max()), int(S.max()) + 1, V), np.float32)
    r = 0
    for b in range(B):
        n = T[b] * (S[b] + 1)
        pad[b, :T[b], :S[b] + 1] = acts[r:r + n].reshape(T[b], S[b] + 1, V)
        r += n
    a = torch.from_numpy(pad).to(dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St)
    n = _launches(lambda: _run(op, a, lab, Tt, St))
    got = _run(op, a, lab, Tt, St)
    assert n["chase"] == 1, n
    _assert_same(got, ref)


def test_chase_not_taken_outside_its_shapes(op, dev):
    """S + 1 > 224 (the halo recursion of more than 4 waves) and bf16 acts run the two-kernel path."""
    rng = np.random.default_rng(11)
    acts, labels, T, S = random_problem(rng, 2, (300, 320), 250, 8, force={0: (310, 250)})
    a, lab = torch.from_numpy(acts).cuda(), torch.from_numpy(labels).cuda()
    n = _launches(lambda: _run(op, a, lab, torch.from_numpy(T), torch.from_numpy(S)))
    assert n["chase"] == 0 and n["log_softmax"] == 1, n
    _, _, T2, S2, a2, lab2 = _problem("c2_row16_one_wave", dev)
    n = _launches(lambda: _run(op, a2.bfloat16(), lab2, torch.from_numpy(T2), torch.from_numpy(S2)))
    assert n["chase"] == 0 and n["log_softmax"] == 1, n


def test_chase_graph_replay_follows_new_acts(op, dev):
    """A captured step replays the flag memset + the chase launch: every replay waits for its own producers (a
    replay reading the previous replay's flags would return the previous acts' costs)."""
    _, _, T, S, a0, lab = _problem("c2_row16_one_wave", dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    static = a0.clone().requires_grad_(True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            static.grad = None
            op.monotonic_rnnt_loss(static, lab, Tt, St).sum().backward()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    static.grad = None
    with torch.cuda.graph(g):
        costs = op.monotonic_rnnt_loss(static, lab, Tt, St)
        costs.sum().backward()
    gen = torch.Generator(device=dev).manual_seed(5)
    for i in range(4):
        new = torch.randn(a0.shape, device=dev, generator=gen) * (1 + i)
        with torch.no_grad():
            static.copy_(new)
        g.replay()
        torch.cuda.synchronize()
        with knobs(chase=0):
            ref = _run(op, new, lab, Tt, St)
        _assert_same((costs.detach(), static.grad), ref)


def test_chase_two_streams_at_once(op, dev):
    """Two forward + backward passes in flight on two streams: flags live in each call's workspace."""
    _, _, T, S, a, lab = _problem("c2_row16_one_wave", dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    b = torch.flip(a, [1]).contiguous()
    with knobs(chase=0):
        ra, rb = _run(op, a, lab, Tt, St), _run(op, b, lab, Tt, St)
    outs = {}
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    for _ in range(3):
        for key, x, st in (("a", a, streams[0]), ("b", b, streams[1])):
            with torch.cuda.stream(st):
                xx = x.detach().clone().requires_grad_(True)
                c = op.monotonic_rnnt_loss(xx, lab, Tt, St)
                c.sum().backward()
                outs[key] = (c.detach(), xx.grad)
    torch.cuda.synchronize()
    _assert_same(outs["a"], ra)
    _assert_same(outs["b"], rb)
