"""Multi-rank tests of the batch-sharded path on the CPU with gloo: each rank takes its contiguous
slice of a ragged batch (pytorch_binding/distributed.py) and runs the PRODUCT path on it -- monotonic_rnnt_loss on
CPU tensors (the library's host implementation, mrnnt_cpu_*) with backward -- and one all-reduce gives the
full-batch loss. The rank gradients, concatenated, equal the full-batch gradients of the same path bit for bit, and
the all-reduced loss equals the fp64 oracle's sum (the oracle is only the checker here)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed import allreduce_loss, rows_per_utterance, shard_bounds, shard_slice


def test_shard_bounds_balanced_and_contiguous():
    rng = np.random.default_rng(0)
    T = rng.integers(200, 1601, 512)
    S = np.array([rng.integers(20, min(300, t) + 1) for t in T])
    cost = rows_per_utterance(T, S)
    for world in (1, 2, 4, 8):
        b = shard_bounds(cost, world)
        assert b[0][0] == 0 and b[-1][1] == 512
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        loads = [cost[lo:hi].sum() for lo, hi in b]
        assert max(loads) - cost.sum() / world <= cost.max()  # greedy prefix split: off by < one utterance


def _worker(rank, world, port, data, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import monotonic_rnnt_op as op
        acts, labels, T, S = data
        a, lab, t, s, (lo, hi) = shard_slice(torch.from_numpy(acts), torch.from_numpy(labels), T, S, rank, world)
        a = a.clone().requires_grad_(True)
        costs = op.monotonic_rnnt_loss(a, lab, t, s, blank_label=0)
        loss = costs.sum()
        loss.backward()
        total = allreduce_loss(costs)
        out[rank] = (lo, hi, float(total), costs.detach().numpy().copy(), a.grad.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_product_path_equals_full_batch(world):
    import monotonic_rnnt_op as op
    import oracle as O
    rng = np.random.default_rng(3 + world)
    B, V = 7, 12
    T = rng.integers(3, 30, B).astype(np.int32)
    S = np.array([rng.integers(0, min(t, 6) + 1) for t in T], np.int32)
    rows = int(np.sum(T * (S + 1)))
    acts = rng.standard_normal((rows, V)).astype(np.float32)
    labels = rng.integers(1, V, (B, int(S.max()))).astype(np.int32)
    a = torch.from_numpy(acts).clone().requires_grad_(True)
    full_costs = op.monotonic_rnnt_loss(a, torch.from_numpy(labels), torch.from_numpy(T), torch.from_numpy(S))
    full_costs.sum().backward()
    full_grads = a.grad.numpy()
    oracle_costs, oracle_grads = O.oracle_rnnt(acts, labels, T, S)
    port = 29500 + (os.getpid() % 1000) + 7 * world
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, (acts, labels, T, S), out), nprocs=world, join=True)
        res = [out[r] for r in range(world)]
    spans = [(lo, hi) for lo, hi, *_ in res]
    assert spans[0][0] == 0 and spans[-1][1] == B and all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    # the rank gradients, concatenated in rank order, are the full-batch gradients (bit for bit: utterances are
    # independent in every pass), and so are the costs
    np.testing.assert_array_equal(np.concatenate([r[4] for r in res]), full_grads)
    np.testing.assert_array_equal(np.concatenate([r[3] for r in res]), full_costs.detach().numpy())
    # every rank holds the same all-reduced loss: the oracle's full-batch sum
    for r in res:
        assert abs(r[2] - oracle_costs.sum()) <= 1e-5 * abs(oracle_costs.sum())
    assert np.abs(full_grads - oracle_grads).max() <= 1e-4
