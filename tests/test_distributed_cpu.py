"""world_size-2 gloo test of the batch-sharded path: each rank takes its contiguous slice
of a ragged batch (pytorch_binding/distributed.py), computes its utterances' costs (here the oracle stands
in for the GPU kernels, which the -m gpu tests cover), and one all-reduce gives the full-batch loss."""
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
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        acts, labels, T, S = data
        a, lab, t, s, (lo, hi) = shard_slice(torch.from_numpy(acts), torch.from_numpy(labels), T, S, rank, world)
        costs, _ = O.oracle_rnnt(a.numpy(), lab.numpy(), t.numpy(), s.numpy(), grads=False)
        total = allreduce_loss(torch.from_numpy(costs))
        out[rank] = (lo, hi, float(total))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_loss_equals_full_batch(world):
    rng = np.random.default_rng(3)
    B, V = 7, 12
    T = rng.integers(3, 30, B).astype(np.int32)
    S = np.array([rng.integers(0, min(t, 6) + 1) for t in T], np.int32)
    rows = int(np.sum(T * (S + 1)))
    acts = rng.standard_normal((rows, V)).astype(np.float32)
    labels = rng.integers(1, V, (B, int(S.max()))).astype(np.int32)
    import oracle as O
    full, _ = O.oracle_rnnt(acts, labels, T, S, grads=False)
    port = 29500 + (os.getpid() % 1000)
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, (acts, labels, T, S), out), nprocs=world, join=True)
        res = dict(out)
    spans = sorted((lo, hi) for lo, hi, _ in res.values())
    assert spans[0][0] == 0 and spans[-1][1] == B and spans[0][1] == spans[1][0]
    for _, _, tot in res.values():
        assert abs(tot - full.sum()) <= 1e-5 * abs(full.sum())
