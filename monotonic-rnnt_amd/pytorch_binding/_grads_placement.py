"""Placement-aware gradient buffers for large calls.

On MI355X the streaming write rate of a large allocation depends on its physical backing: about one in three
52.7 GB grads buffers of the headline writes ~20 % slower than the others (5.2-5.5 against 6.5-7.2 TB/s for a
nontemporal fill of the whole buffer; gradient pass 15.3-16.0 against 12.4-13.1 ms). The counters put it on the
memory side -- 2.5x the DRAM write-credit stalls, same address-translation traffic
(profiles/r02/slow_buffer/rootcause_pmc.json) -- and the rate is constant over the buffer's life, so the caching
allocator, which hands the same block to every later step, keeps a slow draw for the whole run.

For gradient outputs of at least MIN_BYTES this module keeps one buffer per (device, dtype), chosen once: a
candidate from the caching allocator is timed with one nontemporal zero fill over its whole length
(mrnnt_fill_zero, the gradient pass's store stream: ~8 ms for 52.7 GB); below FAST_GBPS a further candidate is
allocated while the earlier ones are still held (so it is a different block), up to MAX_CANDIDATES or until HBM
runs short, and the fastest is kept (the others go back to the caching allocator). Later calls get a view of the
kept buffer whenever nothing else holds it (storage use count 1: e.g. the previous step's acts.grad was
dropped), and a plain allocation otherwise, so a caller that keeps gradients across calls never sees them
overwritten. Under HIP-graph capture the graph's memory pool serves gradients as usual. MRNNT_GRADS_PLACEMENT=0
turns this off (plain torch.empty_like); release() drops the kept buffers.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Callable, Dict, List, Optional, Tuple

import torch

MIN_BYTES = 4 << 30        # below this a slow draw costs under a millisecond: plain allocations
FAST_GBPS = 6300.0         # whole-buffer nontemporal fill rate of the fast classes (6.5-7.2 TB/s measured)
MAX_CANDIDATES = 5         # HBM is the usual limit: 4 candidates of 52.7 GB beside the headline's acts
HBM_RESERVE = 4 << 30      # free device memory left untouched when trying a further candidate


# storage use count (private torch API, present in 2.x): without it a kept buffer could not be proven unshared,
# so the module falls back to plain allocations
_use_count = getattr(torch._C, "_storage_Use_Count", None)


def enabled() -> bool:
    return _use_count is not None and os.environ.get("MRNNT_GRADS_PLACEMENT", "1") != "0"


class _Kept:
    __slots__ = ("storage", "nbytes", "gbps")

    def __init__(self, storage, nbytes: int, gbps: float):
        self.storage, self.nbytes, self.gbps = storage, nbytes, gbps


def _fill_gbps(buf: torch.Tensor) -> float:
    """Time one whole-buffer nontemporal zero fill (after one untimed fill) on the current stream."""
    try:
        from . import _mrnnt_lib as L
    except ImportError:
        import _mrnnt_lib as L
    n = buf.numel() - buf.numel() % 16
    stream = torch.cuda.current_stream(buf.device)
    sp = ctypes.c_void_p(stream.cuda_stream)
    fill = L.load().mrnnt_fill_zero
    L.check(fill(ctypes.c_void_p(buf.data_ptr()), n, sp), "fill_zero")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    L.check(fill(ctypes.c_void_p(buf.data_ptr()), n, sp), "fill_zero")
    e1.record(stream)
    e1.synchronize()
    return n / (e0.elapsed_time(e1) * 1e-3) / 1e9


def _free_bytes(dev: torch.device) -> int:
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free)


class GradsArena:
    """One kept gradient buffer per (device, dtype). The device hooks are injectable for host-side tests."""

    def __init__(self, probe: Callable[[torch.Tensor], float] = _fill_gbps,
                 free_bytes: Callable[[torch.device], int] = _free_bytes,
                 alloc: Optional[Callable[[int, torch.device], torch.Tensor]] = None,
                 fast_gbps: float = FAST_GBPS, max_candidates: int = MAX_CANDIDATES, min_bytes: int = MIN_BYTES,
                 require_cuda: bool = True):
        self._probe, self._free = probe, free_bytes
        self._alloc = alloc or (lambda n, dev: torch.empty(n, dtype=torch.uint8, device=dev))
        self.fast_gbps, self.max_candidates, self.min_bytes = fast_gbps, max_candidates, min_bytes
        self.require_cuda = require_cuda
        self._kept: Dict[Tuple[torch.device, torch.dtype], _Kept] = {}
        self._lock = threading.Lock()
        self.log: List[dict] = []  # one record per placement decision (bench.py reports it)

    def like(self, acts: torch.Tensor) -> torch.Tensor:
        """A contiguous uninitialised tensor of acts' shape, dtype and device."""
        nbytes = acts.numel() * acts.element_size()
        if nbytes < self.min_bytes or (self.require_cuda and not acts.is_cuda) or _capturing(acts):
            return torch.empty_like(acts, memory_format=torch.contiguous_format)
        key = (acts.device, acts.dtype)
        with self._lock:
            kept = self._kept.get(key)
            if kept is not None and _use_count(kept.storage._cdata) > 1:
                return torch.empty_like(acts, memory_format=torch.contiguous_format)  # still held by the caller
            if kept is None or kept.nbytes < nbytes:
                if kept is not None:
                    del self._kept[key]
                    kept = None  # the old block goes back to the caching allocator before the new one is chosen
                kept = self._kept[key] = self._choose(nbytes, acts.device)
        out = torch.empty(0, dtype=acts.dtype, device=acts.device)
        return out.set_(kept.storage, 0, acts.shape, _contiguous_strides(acts.shape))

    def _choose(self, nbytes: int, dev: torch.device) -> _Kept:
        cands: List[Tuple[float, torch.Tensor]] = []
        while True:
            buf = self._alloc(nbytes, dev)
            cands.append((self._probe(buf), buf))
            best = max(c[0] for c in cands)
            if best >= self.fast_gbps or len(cands) >= self.max_candidates:
                break
            if self._free(dev) < nbytes + HBM_RESERVE:
                break
        rate, buf = max(cands, key=lambda c: c[0])
        self.log.append({"bytes": nbytes, "candidates_gbps": [round(c[0], 1) for c in cands],
                         "kept_gbps": round(rate, 1)})
        return _Kept(buf.untyped_storage(), nbytes, rate)

    def release(self) -> None:
        with self._lock:
            self._kept.clear()


def _capturing(acts: torch.Tensor) -> bool:
    """Inside HIP-graph capture the probe cannot synchronise: the graph's own pool serves the gradient."""
    return acts.is_cuda and torch.cuda.is_current_stream_capturing()


def _contiguous_strides(shape) -> Tuple[int, ...]:
    st, acc = [], 1
    for d in reversed(tuple(shape)):
        st.append(acc)
        acc *= max(int(d), 1)
    return tuple(reversed(st))


ARENA = GradsArena()


def grads_like(acts: torch.Tensor) -> torch.Tensor:
    return ARENA.like(acts) if enabled() else torch.empty_like(acts, memory_format=torch.contiguous_format)


def release() -> None:
    """Drop the kept gradient buffers (they return to the caching allocator)."""
    ARENA.release()
