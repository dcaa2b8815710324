"""Placement-aware gradient buffers for large calls.

On MI355X the streaming write rate of a large allocation depends on its physical backing: about one in three
52.7 GB grads buffers of the headline writes ~20 % slower than the others (5.2-5.5 against 6.5-7.2 TB/s for a
nontemporal fill of the whole buffer; gradient pass 15.3-16.0 against 12.4-13.1 ms). The counters put it on the
memory side -- 2.5x the DRAM write-credit stalls, same address-translation traffic
(profiles/r02/slow_buffer/rootcause_pmc.json) -- and the rate is constant over the buffer's life, so the caching
allocator, which hands the same block to every later step, keeps a slow draw for the whole run.

For gradient outputs of at least MIN_BYTES this module keeps one buffer per (device, dtype), chosen once: a
candidate from the caching allocator is timed with one nontemporal zero fill over its whole length
(mrnnt_fill_zero, the gradient pass's store stream: ~8 ms for 52.7 GB); below FAST_GBPS ONE further candidate is
allocated while the first is still held (so it is a different block) when free memory allows (>= 3x the need),
and the faster is kept; the other candidate is released to the driver (torch.cuda.empty_cache), so the caching
allocator holds no second block of that size.

Reuse is safe by construction: the kept buffer is only ever caching-allocator memory, and it goes back through the
allocator at every reuse. Each call hands out a view of the kept storage; on the next call, if nothing else holds
it (storage use count 1: the caller dropped the previous gradient), the module drops its own reference -- the
allocator then honours every stream the caller recorded on it (Tensor.record_stream: the block is not reusable
until those streams pass their events) -- and immediately asks the allocator for the same size on the current
stream. When the block is ready the allocator's best fit returns that very block (a "hit": the fast placement is
kept); when a side stream still uses it, or the stream differs, it returns another block (a "miss", counted): that
block is handed out as a plain allocation -- not kept, so the caching allocator gets it back when the caller drops
the gradient, and the module never holds a second block of that size -- and the next call tries to take the fast
block back again (after two misses in a row it gives up on it and chooses afresh). A gradient the caller still
holds is never reused (plain allocation). Under HIP-graph
capture the graph's memory pool serves gradients as usual. MRNNT_GRADS_PLACEMENT=0 turns this off (plain
torch.empty_like), and so does a torch without the storage use count; release() drops the kept buffers.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Callable, Dict, List, Optional, Tuple

import torch

MIN_BYTES = 4 << 30        # below this a slow draw costs under a millisecond: plain allocations
FAST_GBPS = 6300.0         # whole-buffer nontemporal fill rate of the fast classes (6.5-7.2 TB/s measured)
MAX_CANDIDATES = 2         # the first draw and at most one more
FREE_FACTOR = 3            # a further candidate only while free memory is >= FREE_FACTOR x its size


# storage use count (private torch API, present in 2.x): without it a kept buffer could not be proven unshared,
# so the module falls back to plain allocations
_use_count = getattr(torch._C, "_storage_Use_Count", None)


def enabled() -> bool:
    return _use_count is not None and os.environ.get("MRNNT_GRADS_PLACEMENT", "1") != "0"


class _Kept:
    """The kept block (storage held), or -- after a missed take-back -- only its record (storage None): the block sits
    in the caching allocator until the streams recorded on it pass, and the next call asks for it again."""
    __slots__ = ("storage", "ptr", "nbytes", "gbps", "misses")

    def __init__(self, storage, nbytes: int, gbps: Optional[float], ptr: Optional[int] = None, misses: int = 0):
        self.storage, self.nbytes, self.gbps, self.misses = storage, nbytes, gbps, misses
        self.ptr = storage.data_ptr() if storage is not None else ptr


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
                 release_unused: Optional[Callable[[], None]] = None,
                 fast_gbps: float = FAST_GBPS, max_candidates: int = MAX_CANDIDATES, min_bytes: int = MIN_BYTES,
                 require_cuda: bool = True, allocator_refs: int = 0,
                 on_release: Optional[Callable[[int], None]] = None):
        self._probe, self._free = probe, free_bytes
        self._alloc = alloc or (lambda n, dev: torch.empty(n, dtype=torch.uint8, device=dev))
        self._release_unused = release_unused or (lambda: torch.cuda.empty_cache())
        self.fast_gbps, self.max_candidates, self.min_bytes = fast_gbps, max_candidates, min_bytes
        self.require_cuda = require_cuda
        self._on_release = on_release  # test hook: told the address of every block this arena lets go of
        self._held = 1 + allocator_refs  # storage references when only this arena holds the block (a test
        #                                 allocator may keep one of its own)
        self._kept: Dict[Tuple[torch.device, torch.dtype], _Kept] = {}
        self._lock = threading.Lock()
        self.log: List[dict] = []  # one record per placement decision (bench.py reports it)
        self.stats = {"handed_out": 0, "reuse_hits": 0, "reuse_misses": 0, "held_by_caller": 0}

    def like(self, acts: torch.Tensor) -> torch.Tensor:
        """A contiguous uninitialised tensor of acts' shape, dtype and device."""
        nbytes = acts.numel() * acts.element_size()
        if nbytes < self.min_bytes or (self.require_cuda and not acts.is_cuda) or _capturing(acts):
            return torch.empty_like(acts, memory_format=torch.contiguous_format)
        key = (acts.device, acts.dtype)
        with self._lock:
            kept = self._kept.get(key)
            if kept is not None and kept.storage is not None and _use_count(kept.storage._cdata) > self._held:
                self.stats["held_by_caller"] += 1
                return torch.empty_like(acts, memory_format=torch.contiguous_format)  # still held by the caller
            storage = None
            if kept is not None and kept.nbytes >= nbytes:
                ptr, kb, gbps, misses = kept.ptr, kept.nbytes, kept.gbps, kept.misses
                if kept.storage is not None:
                    # the last reference: the caching allocator owns the block, with the caller's streams
                    self._kept[key] = _Kept(None, kb, gbps, ptr, misses)
                    kept = None
                    if self._on_release:
                        self._on_release(ptr)
                buf = self._alloc(kb, acts.device)
                if buf.data_ptr() == ptr:
                    self.stats["reuse_hits"] += 1
                    storage = buf.untyped_storage()
                    self._kept[key] = _Kept(storage, kb, gbps)
                else:
                    # still in use on another stream (or another stream's pool): hand the other block out plainly
                    self.stats["reuse_misses"] += 1
                    storage = buf.untyped_storage()
                    if misses + 1 >= 2:
                        del self._kept[key]  # the fast block is gone for good: choose afresh next time
                    else:
                        self._kept[key] = _Kept(None, kb, gbps, ptr, misses + 1)
                    self.stats["handed_out"] += 1
                    out = torch.empty(0, dtype=acts.dtype, device=acts.device)
                    return out.set_(storage, 0, acts.shape, _contiguous_strides(acts.shape))
            else:
                if kept is not None:
                    del self._kept[key]
                    kept = None  # the old block goes back to the caching allocator before the new one is chosen
                kept = self._kept[key] = self._choose(nbytes, acts.device)
                storage = kept.storage
            self.stats["handed_out"] += 1
            out = torch.empty(0, dtype=acts.dtype, device=acts.device)
            return out.set_(storage, 0, acts.shape, _contiguous_strides(acts.shape))

    def _choose(self, nbytes: int, dev: torch.device) -> _Kept:
        cands: List[Tuple[float, torch.Tensor]] = []
        while True:
            buf = self._alloc(nbytes, dev)
            cands.append((self._probe(buf), buf))
            best = max(c[0] for c in cands)
            if best >= self.fast_gbps or len(cands) >= self.max_candidates:
                break
            if self._free(dev) < FREE_FACTOR * nbytes:
                break
        rate, buf = max(cands, key=lambda c: c[0])
        self.log.append({"bytes": nbytes, "candidates_gbps": [round(c[0], 1) for c in cands],
                         "kept_gbps": round(rate, 1)})
        kept = _Kept(buf.untyped_storage(), nbytes, rate)
        if len(cands) > 1:
            slower = [c[1].data_ptr() for c in cands if c[1] is not buf]
            del buf
            cands.clear()  # the slower candidate is unused now: back to the driver, not left cached beside ours
            for q in slower:
                if self._on_release:
                    self._on_release(q)
            self._release_unused()
        return kept

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
