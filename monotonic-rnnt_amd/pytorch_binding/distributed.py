"""Batch sharding of the monotonic RNN-T loss over the GPUs of a node.

Utterances are independent and acts rows are packed utterance-major, so each rank owns a contiguous
slice of utterances = a contiguous byte range of acts. No data-path collective: each rank runs the full
single-GPU path on its slice, gradients stay rank-local, and the only exchange is one all-reduce of the
summed loss (4 bytes; backend "nccl" = RCCL over xGMI on MI355X, "gloo" in the CPU tests).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def rows_per_utterance(T: Sequence[int], S: Sequence[int]) -> np.ndarray:
    T = np.asarray(T, np.int64)
    S = np.asarray(S, np.int64)
    return T * (S + 1)


def shard_bounds(cost: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous utterance ranges [lo, hi) per rank with balanced sum of `cost` (rows, or rows*V):
    rank r ends at the first prefix sum >= total*(r+1)/world (greedy prefix split)."""
    cost = np.asarray(cost, np.int64)
    cum = np.concatenate([[0], np.cumsum(cost)])
    total = cum[-1]
    bounds, lo = [], 0
    for r in range(world):
        hi = len(cost) if r == world - 1 else int(np.searchsorted(cum, total * (r + 1) / world))
        hi = min(max(hi, lo), len(cost))
        bounds.append((lo, hi))
        lo = hi
    return bounds


def shard_slice(acts: torch.Tensor, labels: torch.Tensor, T, S, rank: int, world: int):
    """This rank's (acts rows, labels rows, T, S, utterance range) of a packed batch."""
    T_np = np.asarray(T.cpu() if torch.is_tensor(T) else T, np.int64).reshape(-1)
    S_np = np.asarray(S.cpu() if torch.is_tensor(S) else S, np.int64).reshape(-1)
    rows = rows_per_utterance(T_np, S_np)
    lo, hi = shard_bounds(rows, world)[rank]
    r0 = int(rows[:lo].sum())
    r1 = r0 + int(rows[lo:hi].sum())
    return (acts[r0:r1], labels[lo:hi], torch.as_tensor(T_np[lo:hi], dtype=torch.int32),
            torch.as_tensor(S_np[lo:hi], dtype=torch.int32), (lo, hi))


def allreduce_loss(local_costs: torch.Tensor) -> torch.Tensor:
    """Sum of all ranks' costs (one all-reduce of a single element). Returns a new detached tensor."""
    tot = local_costs.detach().sum().reshape(1).clone()
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    return tot[0]
