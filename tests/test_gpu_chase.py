"""The chase launch (mrnnt_chase.hip): log-softmax and alpha / beta recursion in
one launch, the recursion workgroups consuming each lattice column as its log-softmax workgroup publishes it
(write-through rows + a ready flag per column, Guideline 16 R1). The reference runs the two back to back
(gpu_rnnt.h:99-191).

Every value the chase computes is the one the two-kernel path computes, so the tests compare bit for bit against
the development build with the chase off (chase = 0). The development build also carries round 6's frame-pair walks
(chase_pair = 2: two frames per dependent log-sum-exp, a three-term step; 3: the same with the first frame of each
pair formed by a side wave), measured and not taken by the product; they round differently and are
checked within fp64-rounding tolerance (_assert_same with the case's S) and against the oracle. Covered: every
log-softmax body the chase carries (16-lane rows,
single-chunk U = 2 / 4, full and partial chunks), both recursion shapes (one wave with its frames staged in LDS by a
loader wave, or read directly; 4-wave halo with idle waves), both acts load policies, ragged / odd / T = 1 / S = 0
lattices, the padded layout, forward only (alpha alone), host and device-resident lengths, HIP-graph replay (ready
tags derived per launch from the dispatch id: no flag is ever cleared), two streams at once, and the progress
guarantee: a recursion wave that waits too long for a column computes it itself (budget 0: every column; producers
held back; a kernel holding the CUs on another stream) -- still the same bits.
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


def _assert_same(a, b, S=None, stage=1):
    """Bit for bit, unless S (the case's label lengths) puts the chase on the staged one-wave walk (S + 1 <= 64, stage
    1) with its default frame pairs: then within the paired step's rounding (costs 1e-6 relative, gradients 1e-5
    absolute -- ~100x the measured differences and ~10x below the oracle tolerance of _parity)."""
    ca, ga = a
    cb, gb = b
    if S is not None and stage == 1 and int(np.max(S)) + 1 <= 64:
        ca64, cb64 = ca.double(), cb.double()
        assert torch.equal(torch.isnan(ca64), torch.isnan(cb64)) and torch.equal(torch.isinf(ca64), torch.isinf(cb64))
        fin = torch.isfinite(cb64)
        assert torch.all((ca64[fin] - cb64[fin]).abs() <= 1e-6 * cb64[fin].abs().clamp(min=1.0)), (ca, cb)
        if ga is not None:
            assert torch.equal(torch.isnan(ga), torch.isnan(gb))
            d = (ga.double() - gb.double()).abs()
            d[torch.isnan(gb)] = 0
            assert float(d.max()) <= 1e-5, float(d.max())
        return
    assert torch.equal(ca.view(torch.int32), cb.view(torch.int32))
    if ga is not None:
        assert torch.equal(ga.view(torch.int32), gb.view(torch.int32))


@pytest.mark.parametrize("stage", [1, 0])
@pytest.mark.parametrize("name", list(CASES))
def test_chase_bit_identical_to_two_kernels(op, dev, name, stage):
    """stage: the one-wave recursion's frames staged in LDS by a loader wave (the product) or read directly."""
    acts, labels, T, S, a, lab = _problem(name, dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    scale = torch.linspace(0.5, 2.0, len(T), device=dev)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St, scale=scale)
    with knobs(chase=1, chase_stage=stage, chase_pair=1):  # one log-sum-exp per frame: the two-kernel path's bits
        n = _launches(lambda: _run(op, a, lab, Tt, St, scale=scale))
        got = _run(op, a, lab, Tt, St, scale=scale)
    assert n["chase"] == 1 and n["log_softmax"] == 0 and n["alpha_beta"] == 0, n
    _assert_same(got, ref)
    with knobs(chase=1, chase_stage=stage, chase_pair=2):  # frame pairs, the side step on the walk
        paired = _run(op, a, lab, Tt, St, scale=scale)
    _assert_same(paired, ref, S, stage)
    with knobs(chase=1, chase_stage=stage, chase_pair=3):  # the product: chain-only walk, side steps on wave 2
        side = _run(op, a, lab, Tt, St, scale=scale)
    _assert_same(side, paired)  # the same operations on the same values, split over two waves
    if name.startswith("c2"):  # the product library takes the same launch
        n = _launches(lambda: _run(op, a, lab, Tt, St, scale=scale))
        assert n["chase"] == 1, n
        _assert_same(_run(op, a, lab, Tt, St, scale=scale), ref)
    if name.startswith("c2") or name.startswith("ragged"):
        cr, gr = O.oracle_rnnt(acts, labels, T, S)
        w = np.repeat(scale.cpu().numpy().astype(np.float64), T.astype(np.int64) * (S + 1))[:, None]
        for r in (got, paired):
            assert_costs(r[0].cpu().numpy().astype(np.float64), cr)
            assert_grads(r[1].cpu().numpy(), gr * w)


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


@pytest.mark.parametrize("lengths", ["host", "device"])
def test_chase_graph_replay_follows_new_acts(op, dev, lengths):
    """A captured step replays the chase launch with the kernel arguments frozen at capture: every replay derives its
    own ready tag from its dispatch id, so it waits for its own producers (a replay matching the previous replay's
    flags would return the previous acts' costs)."""
    _, _, T, S, a0, lab = _problem("c2_row16_one_wave", dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    if lengths == "device":
        Tt, St = Tt.to(dev), St.to(dev)
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
            ref = _run(op, new, lab, Tt.cpu(), St.cpu())
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


def test_dispatch_ids_are_unique_per_replay(dev):
    """The ready tags rest on this: every launch -- each kernel of each HIP-graph replay included -- sees its own
    dispatch id (the AQL packet index on its queue)."""
    import ctypes

    import _mrnnt_lib as L
    t = L.devtools()
    out = torch.zeros(16, dtype=torch.int64, device=dev)
    ptr = ctypes.c_void_p(out.data_ptr())
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            cs = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            assert t.mrnnt_dispatch_probe(ptr, 0, cs) == 0
            assert t.mrnnt_dispatch_probe(ptr, 1, cs) == 0
    seen = []
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        v = out[:4].tolist()
        seen += [v[0], v[2]]
    assert len(set(seen)) == len(seen), seen


@pytest.mark.parametrize("name", ["c2_row16_one_wave", "ragged_row16_t1_s0", "halo_u2_full_idle_waves",
                                  "u4_partial_v1000"])
def test_chase_device_lengths_bit_identical_to_host_lengths(op, dev, name):
    """The reference's calling convention (lengths on the GPU, monotonic_rnnt.cu:85-88) takes the chase launch too:
    the launch plans from acts.size(0) / labels.size(1), locates columns from the lengths in registers and publishes
    the lattice for the gradient pass -- the same bits as host lengths and as the two-kernel path."""
    acts, labels, T, S, a, _ = _problem(name, dev)
    lab = torch.from_numpy(labels[:, :max(1, int(S.max()))].copy()).to(dev)  # tight label rows: the S_b bound
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    Td, Sd = Tt.to(dev), St.to(dev)
    scale = torch.linspace(0.5, 2.0, len(T), device=dev)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St, scale=scale)
    host = _run(op, a, lab, Tt, St, scale=scale)
    n = _launches(lambda: _run(op, a, lab, Td, Sd, scale=scale))
    got = _run(op, a, lab, Td, Sd, scale=scale)
    _assert_same(host, ref)
    _assert_same(got, host)  # host and device lengths: the same launch, the same bits
    if name == "c2_row16_one_wave":
        assert n["chase"] == 1 and n["setup"] == 0 and n["log_softmax"] == 0, n
    with knobs(chase=1, chase_stage=0):
        _assert_same(_run(op, a, lab, Td, Sd, scale=scale), ref)
    op.check_lengths()


def test_chase_device_lengths_invalid_is_nan_and_reported(op, dev):
    """Device lengths that fail validation inside the chase launch: NaN costs and gradients, reported by
    check_lengths() -- the same contract as the two-kernel path."""
    _, _, T, S, a, lab = _problem("c2_row16_one_wave", dev)
    T2 = T.copy()
    T2[3] += 1  # sum_b T_b (S_b + 1) no longer matches acts.size(0)
    Td, Sd = torch.from_numpy(T2).to(dev), torch.from_numpy(S).to(dev)
    n = _launches(lambda: _run(op, a, lab, Td, Sd))
    assert n["chase"] == 1, n
    with pytest.raises(RuntimeError, match="failed validation"):
        op.check_lengths()
    c, g = _run(op, a, lab, Td, Sd)
    assert torch.isnan(c).all() and torch.isnan(g).all()
    with pytest.raises(RuntimeError, match="failed validation"):
        op.check_lengths()


def _helped(reset=True):
    import _mrnnt_lib as L
    return int(L.load_dev().mrnnt_chase_helped(1 if reset else 0))


@pytest.mark.parametrize("stage", [1, 0])
@pytest.mark.parametrize("name", ["c2_row16_one_wave", "ragged_row16_t1_s0", "halo_u2_full_idle_waves"])
def test_chase_self_help_every_column_bit_identical(op, dev, name, stage):
    """Wait budget 0: a recursion wave computes every column it does not find published itself, with the producers'
    own column body on its rows -- the result does not change (and the columns were helped)."""
    _, _, T, S, a, lab = _problem(name, dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St)
    with knobs(chase=1, chase_stage=stage, chase_wait_us=0, chase_delay_us=200, chase_pair=1):
        _helped()
        got = _run(op, a, lab, Tt, St)
        helped = _helped()
    _assert_same(got, ref)
    assert helped > 0, helped


def test_chase_producers_held_back_progress_and_replay(op, dev):
    """Producers that start late (2 ms): the recursion waves give up waiting after 20 us and help themselves; the
    producers still publish afterwards. Replaying the captured step on new logits must still follow them: late
    publications of one launch never satisfy the next (its tag differs)."""
    _, _, T, S, a0, lab = _problem("c2_row16_one_wave", dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=1, chase_wait_us=20, chase_delay_us=2000, chase_pair=1):
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
        _helped()
        gen = torch.Generator(device=dev).manual_seed(9)
        news = []
        for i in range(3):
            new = torch.randn(a0.shape, device=dev, generator=gen)
            news.append(new)
            with torch.no_grad():
                static.copy_(new)
            g.replay()
            torch.cuda.synchronize()
            news[-1] = (new, costs.detach().clone(), static.grad.clone())
        helped = _helped()
    assert helped > 0
    with knobs(chase=0):
        for new, c, gr in news:
            _assert_same((c, gr), _run(op, new, lab, Tt, St))


def test_chase_beside_a_kernel_holding_the_cus(op, dev):
    """A kernel on another stream occupies every workgroup slot of the chip for 30 ms while the chase launch starts:
    its recursion workgroups and producers get the CUs piecemeal -- the costs are right, never NaN."""
    import ctypes

    import _mrnnt_lib as L
    _, _, T, S, a, lab = _problem("c2_row16_one_wave", dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St)
    side = torch.cuda.Stream()
    for k in range(3):
        with torch.cuda.stream(side):
            assert L.devtools().mrnnt_occupy(30000, 2 + 3 * k, ctypes.c_void_p(side.cuda_stream)) == 0
        got = _run(op, a, lab, Tt, St)
        _assert_same(got, ref)
    torch.cuda.synchronize()


def test_chase_two_streams_near_the_recursion_limit(op, dev):
    """the spinning recursion workgroups of two concurrent chase launches, each at a batch near
    chase_pays' limit (2B = 240 of 256 CUs), can hold the slots their producers need. The waves help themselves
    after the wait budget, so both calls finish with the two-kernel path's bits."""
    rng = np.random.default_rng(77)
    B = 120
    acts, labels, T, S = random_problem(rng, B, (90, 100), 30, 128, force={b: (100, 30) for b in range(0, B, 7)})
    a, lab = torch.from_numpy(acts).to(dev), torch.from_numpy(labels).to(dev)
    b = torch.flip(a, [1]).contiguous()
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=0):
        ra, rb = _run(op, a, lab, Tt, St), _run(op, b, lab, Tt, St)
    n = _launches(lambda: _run(op, a, lab, Tt, St))
    assert n["chase"] == 1, n
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    outs = {}
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


@pytest.mark.parametrize("B", [64, 65])
def test_chase_device_lengths_batch_limit(op, dev, B):
    """Device lengths ride in one register per lane of every wave, so the chase launch takes them up to B = 64 and
    B = 65 plans with a setup kernel and runs the two-kernel forward -- both with the two-kernel path's bits."""
    rng = np.random.default_rng(600 + B)
    acts, labels, T, S = random_problem(rng, B, (20, 40), 12, 64, force={0: (1, 0), 5: (40, 12)})
    a, lab = torch.from_numpy(acts).to(dev), torch.from_numpy(labels[:, :max(1, int(S.max()))].copy()).to(dev)
    Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    with knobs(chase=0):
        ref = _run(op, a, lab, Tt, St)
    Td, Sd = Tt.to(dev), St.to(dev)
    n = _launches(lambda: _run(op, a, lab, Td, Sd))
    got = _run(op, a, lab, Td, Sd)
    _assert_same(got, ref)
    if B <= 64:
        assert n["chase"] == 1 and n["setup"] == 0, n
    else:
        assert n["chase"] == 0 and n["setup"] == 1, n
    op.check_lengths()


@pytest.mark.parametrize("lengths", ["host", "device"])
@pytest.mark.parametrize("name", list(CASES))
def test_product_chase_vs_oracle(op, dev, name, lengths):
    """The PRODUCT library (no knobs: the tuned defaults) on every chase shape, against the fp64 oracle directly.
    The bit-identity tests above anchor the chase to the development build's two-kernel path; this anchors the
    product build's own launch to the reference semantics, on host and device lengths."""
    acts, labels, T, S, a, lab = _problem(name, dev)
    if lengths == "host":
        Tt, St = torch.from_numpy(T), torch.from_numpy(S)
    else:
        Tt, St = torch.from_numpy(T).to(dev), torch.from_numpy(S).to(dev)
    got = {}
    n = _launches(lambda: got.setdefault("r", _run(op, a, lab, Tt, St)))
    if name == "c2_row16_one_wave":  # configs[1]: the shape the chase is tuned for takes it on both forms
        assert n["chase"] == 1 and n["log_softmax"] == 0, n
    c, g = got["r"]
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    assert_costs(c.cpu().numpy(), cr)
    assert_grads(g.cpu().numpy(), gr)
