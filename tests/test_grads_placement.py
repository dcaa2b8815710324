"""Host-side tests of the placement-aware gradient buffers (pytorch_binding/_grads_placement.py): the choice
between candidate blocks, reuse only when nothing else holds the kept buffer, and the limits. The device probe,
the allocator and the free-memory query are replaced by fakes, so this runs on CPU tensors."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "monotonic-rnnt_amd",
                                "pytorch_binding"))
import _grads_placement as GP  # noqa: E402


class Fake:
    """A caching-allocator stand-in: it keeps every block it made (one tensor each, so a block the arena keeps has
    storage use count 2 when nothing else uses it: allocator_refs=1); a block the arena lets go of (on_release) is
    free again unless `busy` (another stream still uses it: the device allocator holds such a block back until
    that stream passes its event), and alloc() hands a free block of the size back, as the device allocator's best
    fit does (of two free blocks of the size, the one released first: a deterministic order -- CPU addresses are not,
    so ordering by address made the take-back test depend on where the host allocator put the two blocks)."""

    def __init__(self, rates, free=1 << 60):
        self.rates = list(rates)
        self.free = free
        self.blocks = {}    # data_ptr -> tensor
        self.freed = {}     # data_ptr -> None, in release order
        self.allocs = []    # data_ptr of every block handed out, in order
        self.busy = set()
        self.released = 0

    def probe(self, buf):
        return self.rates.pop(0)

    def alloc(self, n, dev):
        for q in list(self.freed):
            if self.blocks[q].numel() == n and q not in self.busy:
                del self.freed[q]
                blk = self.blocks[q]
                break
        else:
            blk = torch.empty(n, dtype=torch.uint8)
            self.blocks[blk.data_ptr()] = blk
        self.allocs.append(blk.data_ptr())
        return torch.empty(0, dtype=torch.uint8).set_(blk.untyped_storage())

    def on_release(self, ptr):
        self.freed[ptr] = None

    def release_unused(self):
        self.released += 1
        for q in [q for q in self.freed if q not in self.busy]:
            del self.freed[q]
            del self.blocks[q]

    def arena(self, **kw):
        return GP.GradsArena(probe=self.probe, free_bytes=lambda d: self.free, alloc=self.alloc,
                             release_unused=self.release_unused, min_bytes=64, require_cuda=False, allocator_refs=1,
                             on_release=self.on_release, **kw)


def acts(rows=8, V=16, dtype=torch.float32):
    return torch.randn(rows, V).to(dtype)


def test_keeps_faster_of_two_candidates_and_stops_when_fast():
    f = Fake([5000.0, 5400.0, 1.0])
    ar = f.arena()
    g = ar.like(acts())
    assert ar.log[-1]["candidates_gbps"] == [5000.0, 5400.0] and ar.log[-1]["kept_gbps"] == 5400.0
    assert g.data_ptr() == f.allocs[1] and g.shape == (8, 16) and g.dtype == torch.float32 and g.is_contiguous()
    assert f.released == 1 and list(f.blocks) == [f.allocs[1]]  # the slower candidate went back to the driver
    f2 = Fake([6500.0])
    ar2 = f2.arena()
    ar2.like(acts())
    assert ar2.log[-1]["candidates_gbps"] == [6500.0] and f2.released == 0  # fast first draw: no second candidate


def test_candidate_limits():
    f = Fake([1.0, 3.0, 9.0])
    ar = f.arena(max_candidates=2)
    g = ar.like(acts())
    assert ar.log[-1]["candidates_gbps"] == [1.0, 3.0] and g.data_ptr() == f.allocs[1]
    f = Fake([1.0, 9.0], free=3 * 512 - 1)  # a second candidate needs free memory >= 3x its size
    ar = f.arena()
    ar.like(acts())
    assert ar.log[-1]["candidates_gbps"] == [1.0]
    f = Fake([1.0, 9.0], free=3 * 512)
    ar = f.arena()
    ar.like(acts())
    assert ar.log[-1]["candidates_gbps"] == [1.0, 9.0]


def test_reused_only_when_not_held():
    f = Fake([7000.0])
    ar = f.arena()
    a = acts()
    g1 = ar.like(a)
    p = g1.data_ptr()
    g2 = ar.like(a)  # g1 still alive (e.g. gradients kept across steps): a different buffer
    assert g2.data_ptr() != p
    g1.fill_(1.0)
    g2.fill_(2.0)
    assert float(g1.sum()) == g1.numel()
    del g1
    g3 = ar.like(a)
    assert g3.data_ptr() == p and len(ar.log) == 1
    view = g3[2:4]  # a view keeps the storage held
    del g3
    assert ar.like(a).data_ptr() != p
    del view
    assert ar.like(a).data_ptr() == p


def test_smaller_reuses_larger_rechooses_and_dtype_keys():
    f = Fake([7000.0, 7100.0, 7200.0])
    ar = f.arena()
    g = ar.like(acts(rows=8))
    p = g.data_ptr()
    del g
    g = ar.like(acts(rows=4))  # fits in the kept buffer
    assert g.data_ptr() == p and g.shape == (4, 16)
    del g
    g = ar.like(acts(rows=32))  # larger: chosen again
    assert len(ar.log) == 2 and g.shape == (32, 16)
    del g
    h = ar.like(acts(rows=8, dtype=torch.bfloat16))  # another dtype: its own buffer
    assert len(ar.log) == 3 and h.dtype == torch.bfloat16


def test_small_and_disabled_are_plain(monkeypatch):
    f = Fake([])
    ar = GP.GradsArena(probe=f.probe, alloc=f.alloc, min_bytes=1 << 40, require_cuda=False)
    ar.like(acts())
    assert not ar.log and not f.allocs
    monkeypatch.setenv("MRNNT_GRADS_PLACEMENT", "0")
    assert not GP.enabled()
    g = GP.grads_like(acts())
    assert g.shape == (8, 16)


@pytest.mark.parametrize("shape", [(3, 5, 7, 11), (13, 4)])
def test_views_have_contiguous_strides(shape):
    f = Fake([7000.0])
    ar = f.arena()
    a = torch.zeros(shape)
    g = ar.like(a)
    assert g.shape == a.shape and g.stride() == a.stride()


def test_reuse_goes_back_through_the_allocator():
    """A reused gradient is the kept block handed back by the allocator (a hit); a block another stream still uses
    (Tensor.record_stream: the device allocator holds it until that stream passes its event) is not handed back:
    the block the allocator gives instead is handed out plainly, NOT kept (the module never holds a
    second block of that size), and the next call takes the fast block back once it is free."""
    f = Fake([7000.0])
    ar = f.arena()
    a = acts()
    g1 = ar.like(a)
    p = g1.data_ptr()
    del g1
    g2 = ar.like(a)
    assert g2.data_ptr() == p and ar.stats["reuse_hits"] == 1
    f.busy.add(p)  # a side stream still reads the previous gradient
    del g2
    g3 = ar.like(a)
    q = g3.data_ptr()
    assert q != p and ar.stats["reuse_misses"] == 1
    assert all(k.storage is None for k in ar._kept.values())  # the arena holds neither block now
    f.on_release(q)  # the caller drops the plain gradient: back to the allocator
    del g3
    f.busy.clear()
    assert ar.like(a).data_ptr() == p and ar.stats["reuse_hits"] == 2  # the fast block again
    assert len(ar.log) == 1  # no new probe: placement decisions only at the first choice


def test_two_misses_in_a_row_rechoose():
    f = Fake([7000.0, 6900.0])
    ar = f.arena()
    a = acts()
    g = ar.like(a)
    p = g.data_ptr()
    f.busy.add(p)
    del g
    for _ in range(2):  # the fast block stays busy: two plain hand-outs
        h = ar.like(a)
        assert h.data_ptr() != p
        f.on_release(h.data_ptr())
        del h
    assert not ar._kept  # given up on
    ar.like(a)
    assert len(ar.log) == 2  # chosen afresh


def test_no_use_count_means_plain(monkeypatch):
    monkeypatch.setattr(GP, "_use_count", None)
    assert not GP.enabled()
