"""GPU tests of the round-2 surface items: per-row state read-out against the reference's own golden state,
device-label safety, input validation, repeated backward, the HIP path against the library's CPU path, the
configs[4] full-length utterance against the oracle, RCCL initialisation and the N-rank bench launcher."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import oracle as O
from _parity import FIXTURES, assert_costs, assert_grads, assert_state, random_problem, used_rows

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def op():
    import monotonic_rnnt_op
    return monotonic_rnnt_op


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


def _t(x, dev, dt=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    return t.to(dev) if dt is None else t.to(dev, dt)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_golden_denominators_alpha_beta(op, dev, path):
    """mrnnt_read_state after a forward against the reference's own get_denom / get_alpha / get_beta at double
    precision (golden denom_f64 / alpha_f64 / beta_f64): the GPU's fp32 denominators and fp64 alpha / beta."""
    import _mrnnt_lib as L
    fx = dict(np.load(path))
    al = None if "alignment" not in fx else _t(fx["alignment"], dev)
    prep = op._Prepared(_t(fx["acts"], dev), _t(fx["labels"], dev), _t(fx["T"], dev), _t(fx["S"], dev), al,
                        int(fx.get("max_shift", 0)), int(fx["blank"]))
    _, ws = op._forward(prep, with_beta=True)
    n = fx["acts"].shape[0]
    den = torch.zeros(n, dtype=torch.float32, device=dev)
    alpha = torch.zeros(n, dtype=torch.float64, device=dev)
    beta = torch.zeros(n, dtype=torch.float64, device=dev)
    L.check(L.load().mrnnt_read_state(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                      ctypes.c_void_p(den.data_ptr()), ctypes.c_void_p(alpha.data_ptr()),
                                      ctypes.c_void_p(beta.data_ptr()), prep.stream()), "read_state")
    torch.cuda.synchronize()
    assert_state(den.cpu().numpy(), alpha.cpu().numpy(), beta.cpu().numpy(), fx, window=used_rows(fx), rel=1e-4)


@pytest.mark.parametrize("bad", [3, 7, -5, 1 << 30])
def test_device_label_out_of_range_gives_inf_cost_nan_grads(op, dev, bad):
    """A device label outside [0, V) is not read back (no sync) and never used as an index: its log-softmax pick is
    NaN, and the recursion's LSE turns a NaN transition into no probability (fmax drops the NaN; both directions
    stay -inf past that label position, which every path of the utterance crosses). So, pinned exactly, whatever
    the bad value: that utterance's cost is +inf and every element of its gradient NaN (exp(... - ll), ll = -inf,
    as the reference's cpu_rnnt.h forms it); the other utterances are exact (no access past a row)."""
    rng = np.random.default_rng(abs(bad) % 97)
    acts, labels, T, S = random_problem(rng, 3, (6, 14), 4, 3, force={0: (10, 3), 1: (9, 2), 2: (12, 4)})
    labels = np.where(labels >= 3, 1, labels).astype(np.int32)
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    r0, r1 = T[0] * (S[0] + 1), T[0] * (S[0] + 1) + T[1] * (S[1] + 1)
    for pos in range(S[1]):  # the bad label at every position of utterance 1
        lab_bad = labels.copy()
        lab_bad[1, pos] = bad
        a = _t(acts, dev).requires_grad_(True)
        costs = op.monotonic_rnnt_loss(a, _t(lab_bad, dev), _t(T, dev), _t(S, dev))
        costs.sum().backward()
        torch.cuda.synchronize()
        c, g = costs.detach().cpu().numpy().astype(np.float64), a.grad.cpu().numpy()
        assert np.isposinf(c[1]) and np.isfinite(c[[0, 2]]).all(), (pos, c)
        assert np.isnan(g[r0:r1]).all(), pos
        assert_costs(c[[0, 2]], cr[[0, 2]])
        assert_grads(np.concatenate([g[:r0], g[r1:]]), np.concatenate([gr[:r0], gr[r1:]]))


def test_host_labels_and_strides_validated(op, dev):
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "toy.npz")))
    acts, T, S = _t(fx["acts"], dev), torch.from_numpy(fx["T"]), torch.from_numpy(fx["S"])
    with pytest.raises(RuntimeError, match="outside"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1, 3]], dtype=torch.int32), T, S)  # host labels, V = 3
    with pytest.raises(RuntimeError, match="stride"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1]], dtype=torch.int32, device=dev), T, S)
    with pytest.raises(RuntimeError, match="stride"):
        op.monotonic_rnnt_loss(acts, torch.tensor([[1, 2]], dtype=torch.int32, device=dev), T, S,
                               torch.tensor([[0, 1, 0]], dtype=torch.int32, device=dev), 0)


def test_backward_twice_with_retain_graph(op, dev):
    rng = np.random.default_rng(3)
    acts, labels, T, S = random_problem(rng, 3, (5, 40), 8, 64)
    a = _t(acts, dev).requires_grad_(True)
    costs = op.monotonic_rnnt_loss(a, _t(labels, dev), torch.from_numpy(T), torch.from_numpy(S))
    (costs * 2).sum().backward(retain_graph=True)
    g1 = a.grad.clone()
    a.grad = None
    (costs * 2).sum().backward()
    assert torch.equal(a.grad, g1)
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    assert_grads(g1.cpu().numpy(), 2 * gr)


def test_broadcast_upstream_gradient(op, dev):
    """costs.sum() / costs.mean() hand backward a stride-0 [B] gradient, which the gradient kernel reads in place
    (grad_scale_broadcast, ABI v6: no copy kernel): bit-identical to the same scale as a materialised [B] vector."""
    rng = np.random.default_rng(6)
    acts, labels, T, S = random_problem(rng, 5, (5, 60), 20, 64)
    out = []
    for reduce in (lambda c: c.sum(), lambda c: c.mean(), lambda c: (c * torch.full_like(c, 1.0 / 5)).sum()):
        a = _t(acts, dev).requires_grad_(True)
        reduce(op.monotonic_rnnt_loss(a, _t(labels, dev), torch.from_numpy(T), torch.from_numpy(S))).backward()
        out.append(a.grad)
    assert torch.equal(out[1], out[2])
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    assert_grads(out[0].cpu().numpy(), gr)


def test_gpu_and_cpu_paths_agree(op, dev):
    """The same inputs through the HIP kernels (GPU tensors) and the library's host implementation (CPU
    tensors): both against the oracle, and against each other."""
    rng = np.random.default_rng(21)
    acts, labels, T, S = random_problem(rng, 6, (30, 160), 60, 300)
    out = []
    for d in (dev, torch.device("cpu")):
        a = _t(acts, d).requires_grad_(True)
        costs = op.monotonic_rnnt_loss(a, _t(labels, d), _t(T, d), _t(S, d))
        costs.sum().backward()
        out.append((costs.detach().cpu().numpy().astype(np.float64), a.grad.cpu().numpy()))
    cr, gr = O.oracle_rnnt(acts, labels, T, S, num_threads=8)
    for c, g in out:
        assert_costs(c, cr)
        assert_grads(g, gr)
    assert_costs(out[0][0], out[1][0].astype(np.float64))
    assert np.abs(out[0][1] - out[1][1]).max() <= 1e-4


def test_configs4_full_utterance_vs_oracle(op, dev):
    """configs[4] at full size for one utterance (T=1000, S=200, V=10000: 8 GB of logits) against the oracle on
    every element: the large-vocabulary log-softmax and gradient at the benchmarked length."""
    import _mrnnt_lib as L
    T, S, V = 1000, 200, 10000
    rows = T * (S + 1)
    acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
    L.synth_acts(acts.data_ptr(), 0, rows * V, 0, True, torch.cuda.current_stream().cuda_stream)
    labels = np.random.default_rng(1).integers(1, V, (1, S)).astype(np.int32)
    acts.requires_grad_(True)
    costs = op.monotonic_rnnt_loss(acts, _t(labels, dev), torch.tensor([T]), torch.tensor([S]))
    costs.sum().backward()
    torch.cuda.synchronize()
    c = costs.detach().cpu().numpy().astype(np.float64)
    g = acts.grad.cpu().numpy()
    del acts
    torch.cuda.empty_cache()
    host = O.synth_acts(0, rows * V, seed=0).reshape(rows, V)
    cr, gr = O.oracle_rnnt(host, labels, np.array([T]), np.array([S]), num_threads=16)
    assert_costs(c, cr)
    assert_grads(g, gr)


def test_rccl_world1_sharded_loss(op, dev):
    """torch.distributed over RCCL ("nccl" backend) at world size 1 on this GPU: shard_slice -> loss ->
    allreduce_loss (the one collective of the path), checked against the oracle's summed cost."""
    import torch.distributed as dist
    from distributed import allreduce_loss, shard_slice
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        rng = np.random.default_rng(9)
        acts, labels, T, S = random_problem(rng, 5, (20, 60), 10, 64)
        a, lab, Ts, Ss, (lo, hi) = shard_slice(_t(acts, dev), _t(labels, dev), T, S, 0, 1)
        assert (lo, hi) == (0, 5)
        a = a.detach().requires_grad_(True)
        costs = op.monotonic_rnnt_loss(a, lab, Ts, Ss)
        tot = allreduce_loss(costs)
        x = torch.ones(1, device=dev)
        dist.all_reduce(x)  # an RCCL kernel really ran on this device
        torch.cuda.synchronize()
        assert float(x.item()) == 1.0
        cr, _ = O.oracle_rnnt(acts, labels, T, S)
        assert abs(float(tot.item()) - cr.sum()) <= 1e-4 * abs(cr.sum())
    finally:
        dist.destroy_process_group()


def _bench(args, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_launches_two_ranks():
    """`bench.py --gpus 2` spawns two ranks itself (here both on this one GPU over gloo) and reports n_gpus 2 and
    the whole-job batch."""
    out = _bench(["--gpus", "2", "--dist-backend", "gloo", "--config", "c2", "--steps", "2", "--warmup", "1",
                  "--no-cpu"])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 32
    assert out["scaling"] == "weak" and out["value"] > 0


def test_bench_chunked_in_place_mode_matches_resident():
    """The in-place / chunked memory modes (configs[3] at N <= 2, configs[4]) compute the same loss as the
    resident autograd path on a small config forced into chunks by a tiny HBM budget."""
    res = _bench(["--config", "c2", "--steps", "1", "--warmup", "1", "--no-cpu"])
    chk = _bench(["--config", "c2", "--steps", "1", "--warmup", "1", "--no-cpu", "--hbm-budget-gb", "0.05"])
    assert res["config"]["memory_mode"] == "resident" and chk["config"]["memory_mode"] == "inplace"
    assert chk["config"]["chunks_per_step"] > 1
    assert abs(res["loss_check"] - chk["loss_check"]) <= 1e-5 * abs(res["loss_check"])
    assert res["roofline"]["live_rows"] == chk["roofline"]["live_rows"]


def test_fill_zero(dev):
    import _mrnnt_lib as L
    buf = torch.ones((1 << 20) + 64, dtype=torch.float32, device=dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.check(L.load().mrnnt_fill_zero(ctypes.c_void_p(buf.data_ptr() + 256), 4 << 20, sp), "fill_zero")
    torch.cuda.synchronize()
    assert torch.all(buf[64:64 + (1 << 20)] == 0) and torch.all(buf[:64] == 1) and torch.all(buf[64 + (1 << 20):] == 1)
    assert L.load().mrnnt_fill_zero(ctypes.c_void_p(buf.data_ptr() + 4), 64, sp) == L.RNNT_STATUS_INVALID_VALUE
    assert L.load().mrnnt_fill_zero(ctypes.c_void_p(buf.data_ptr()), 60, sp) == L.RNNT_STATUS_INVALID_VALUE


def test_grads_placement_arena_on_device(op, dev, monkeypatch):
    """The placement-aware gradient buffer (threshold lowered so a small call takes it, real fill probe): the
    kept buffer is reused once acts.grad is dropped, a held gradient is never overwritten, and the gradients
    equal the plain-allocation path bit for bit."""
    import _grads_placement as GP
    ar = GP.GradsArena(min_bytes=1 << 16)
    monkeypatch.setattr(GP, "ARENA", ar)
    rng = np.random.default_rng(17)
    acts, labels, T, S = random_problem(rng, 4, (40, 90), 20, 256)
    a = _t(acts, dev).requires_grad_(True)
    lab, Tt, St = _t(labels, dev), torch.from_numpy(T), torch.from_numpy(S)

    def step():
        op.monotonic_rnnt_loss(a, lab, Tt, St).sum().backward()
        torch.cuda.synchronize()
        return a.grad

    g1 = step()
    assert len(ar.log) == 1 and ar.log[0]["kept_gbps"] > 0
    p1, ref = g1.data_ptr(), g1.clone()
    a.grad = None
    del g1
    g2 = step()
    assert g2.data_ptr() == p1 and torch.equal(g2, ref)  # reused
    keep = a.grad
    a.grad = None
    g3 = step()  # `keep` still holds the kept buffer: a fresh one, `keep` untouched
    assert g3.data_ptr() != p1 and torch.equal(keep, ref) and torch.equal(g3, ref)
    monkeypatch.setenv("MRNNT_GRADS_PLACEMENT", "0")
    a.grad = None
    assert torch.equal(step(), ref)
    cr, gr = O.oracle_rnnt(acts, labels, T, S)
    assert_grads(ref.cpu().numpy(), gr)



def test_grads_placement_respects_record_stream(op, dev, monkeypatch):
    """ADVICE / VERDICT r2: a consumer that reads the previous gradient on a side stream and drops it after
    record_stream must not see it overwritten by the next backward. The kept block goes back through the caching
    allocator at reuse, which holds it until the side stream has passed its event: the next gradient lands
    elsewhere (a counted miss) and the consumer reads the values it was given."""
    import _grads_placement as GP
    ar = GP.GradsArena(min_bytes=1 << 16)
    monkeypatch.setattr(GP, "ARENA", ar)
    rng = np.random.default_rng(18)
    acts, labels, T, S = random_problem(rng, 4, (40, 90), 20, 256)
    a = _t(acts, dev).requires_grad_(True)
    lab, Tt, St = _t(labels, dev), _t(T, dev), _t(S, dev)
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)

    def step(scale):
        a.grad = None
        (op.monotonic_rnnt_loss(a, lab, Tt, St) * scale).sum().backward()
        return a.grad

    ref = step(1.0).clone()
    torch.cuda.synchronize()
    for rnd in range(3):
        g = step(1.0)
        p = g.data_ptr()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            torch.cuda._sleep(20_000_000)  # keep the side stream busy well past the next backward
            seen = g.clone()  # the consumer's read of the gradient, queued behind the sleep
        g.record_stream(side)
        a.grad = None
        del g
        g2 = step(-3.0)  # the next backward on the main stream, while the side stream has not read yet
        torch.cuda.synchronize()
        assert torch.equal(seen, ref), rnd  # the consumer saw the gradient it was handed
        assert g2.data_ptr() != p and torch.equal(g2, ref * -3.0)
        del g2
    assert ar.stats["reuse_misses"] >= 3 and ar.stats["handed_out"] >= 7
    torch.cuda.synchronize()
    hits = ar.stats["reuse_hits"]
    step(1.0)
    torch.cuda.synchronize()
    step(1.0)  # no side-stream use: the block comes straight back
    assert ar.stats["reuse_hits"] > hits

@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("device_lengths", [False, True], ids=["host_T_S", "device_T_S"])
def test_hip_graph_capture_replay(op, dev, aligned, device_lengths):
    """Forward + backward captured once in a HIP graph (torch.cuda.graph) and replayed on new logits written
    into the captured input: costs and gradients equal an eager call on the same logits and the oracle (the
    op makes no host synchronisation and allocates only through torch, so it is capture-safe). With device T / S
    (the reference's calling convention) nothing is planned from the lengths on the host at all."""
    rng = np.random.default_rng(40 + aligned)
    acts1, labels, T, S = random_problem(rng, 5, (30, 120), 25, 128)
    acts2 = rng.standard_normal(acts1.shape).astype(np.float32) * 2
    al = None
    if aligned:
        al_np = np.zeros((len(T), int(T.max())), np.int32)
        for b in range(len(T)):
            fr = ((np.arange(S[b]) + 0.5) * T[b] / max(S[b], 1)).astype(np.int64)
            al_np[b, fr] = labels[b, :S[b]]
        al = _t(al_np, dev)
    a = _t(acts1, dev).requires_grad_(True)
    lab, Tt, St = _t(labels, dev), torch.from_numpy(T), torch.from_numpy(S)
    if device_lengths:
        Tt, St = Tt.to(dev), St.to(dev)
    k = 3 if aligned else 0

    def fwd_bwd():
        costs = op.monotonic_rnnt_loss(a, lab, Tt, St, al, k)
        (costs * torch.arange(1, len(T) + 1, device=dev)).sum().backward()
        return costs

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            a.grad = None
            fwd_bwd()
    torch.cuda.current_stream(dev).wait_stream(side)
    a.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        c_static = fwd_bwd()
    with torch.no_grad():
        a.copy_(_t(acts2, dev))
    g.replay()
    torch.cuda.synchronize()
    c_graph, g_graph = c_static.detach().clone(), a.grad.detach().clone()
    g.replay()  # idempotent
    torch.cuda.synchronize()
    assert torch.equal(c_static, c_graph) and torch.equal(a.grad, g_graph)
    b = _t(acts2, dev).requires_grad_(True)
    ce = op.monotonic_rnnt_loss(b, lab, Tt, St, al, k)
    (ce * torch.arange(1, len(T) + 1, device=dev)).sum().backward()
    assert torch.equal(ce.detach(), c_graph) and torch.equal(b.grad, g_graph)
    if not aligned:
        cr, gr = O.oracle_rnnt(acts2, labels, T, S)
        assert_costs(c_graph.cpu().numpy().astype(np.float64), cr)
        w = np.repeat(np.arange(1, len(T) + 1), T * (S + 1))[:, None]
        assert_grads(g_graph.cpu().numpy(), gr * w)


def test_bench_graph_mode_matches_eager():
    """`bench.py --graph` (forward + backward replayed from a HIP graph) computes the loss of the eager step."""
    eager = _bench(["--config", "c2", "--steps", "5", "--warmup", "2", "--no-cpu"])
    graph = _bench(["--config", "c2", "--steps", "20", "--warmup", "3", "--no-cpu", "--graph"])
    assert graph["config"]["execution"] == "hip_graph_replay" and eager["config"]["execution"] == "eager"
    assert abs(graph["loss_check"] - eager["loss_check"]) <= 1e-6 * abs(eager["loss_check"])
    assert graph["kernels"]["grad"]["avg_ms"] > 0 and graph["ms_per_step"] > 0


def test_bench_eight_rank_rehearsal():
    """`bench.py --gpus 8` rehearsed with 8 gloo ranks sharing this GPU: configs[1]
    weak-scaled (8 x 16 utterances) and configs[3] strong-scaled in in-place chunks under a small HBM budget, whose
    all-reduced loss equals the one-rank run over the same 512 utterances. Every rank reports its device."""
    c2 = _bench(["--gpus", "8", "--dist-backend", "gloo", "--config", "c2", "--steps", "2", "--warmup", "1",
                 "--no-cpu"], 400)
    assert c2["n_gpus"] == 8 and c2["config"]["global_batch"] == 128 and c2["scaling"] == "weak"
    assert sorted(d["rank"] for d in c2["config"]["rank_devices"]) == list(range(8))
    assert {d["local_rank"] for d in c2["config"]["rank_devices"]} == set(range(8))
    # the keys the driver compares N > 1 with N = 1 by: every rank's step time, max / min, the
    # all-reduce's own latency; value is computed from the max over ranks
    rk = c2["ranks"]
    assert rk["n"] == 8 and len(rk["ms_per_step"]) == 8 and all(t > 0 for t in rk["ms_per_step"])
    assert rk["max_ms_per_step"] == max(rk["ms_per_step"]) == c2["ms_per_step"]
    assert rk["min_ms_per_step"] == min(rk["ms_per_step"]) and 0 < rk["balance_min_over_max"] <= 1
    assert rk["allreduce_4byte_us"] > 0 and rk["collective"] == "gloo (rehearsal)"
    assert rk["devices_distinct"] is False  # 8 gloo ranks share this one GPU; under RCCL bench.py requires distinct
    assert abs(c2["value"] - 128 * 2 / (c2["ms_per_step"] * 2e-3)) <= 1e-3 * c2["value"]
    one_c2 = _bench(["--config", "c2", "--steps", "2", "--warmup", "1", "--no-cpu"], 400)
    assert one_c2["ranks"]["n"] == 1 and one_c2["ranks"]["allreduce_4byte_us"] is None
    one = _bench(["--config", "ragged", "--steps", "1", "--warmup", "0", "--no-cpu", "--hbm-budget-gb", "30"], 400)
    eight = _bench(["--gpus", "8", "--dist-backend", "gloo", "--config", "ragged", "--steps", "1", "--warmup", "0",
                    "--no-cpu", "--hbm-budget-gb", "8"], 600)
    assert eight["n_gpus"] == 8 and eight["scaling"] == "strong"
    assert eight["config"]["global_batch"] == one["config"]["global_batch"] == 512
    assert eight["config"]["memory_mode"] == "inplace"
    assert abs(one["loss_check"] - eight["loss_check"]) <= 1e-6 * abs(one["loss_check"])


def test_bench_ragged_sharded_two_ranks_equals_one():
    """configs[3] strong-scaled over 2 ranks (gloo, both on this GPU, in-place chunks under a small HBM budget):
    the all-reduced loss of the sharded batch equals the one-rank run over the whole batch."""
    one = _bench(["--config", "ragged", "--steps", "1", "--warmup", "0", "--no-cpu", "--hbm-budget-gb", "30"], 400)
    two = _bench(["--gpus", "2", "--dist-backend", "gloo", "--config", "ragged", "--steps", "1", "--warmup", "0",
                  "--no-cpu", "--hbm-budget-gb", "30"], 400)
    assert one["config"]["memory_mode"] == "inplace" and two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert one["config"]["global_batch"] == two["config"]["global_batch"] == 512
    assert abs(one["loss_check"] - two["loss_check"]) <= 1e-6 * abs(one["loss_check"])
