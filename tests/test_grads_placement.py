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
    def __init__(self, rates, free=1 << 60):
        self.rates = list(rates)
        self.free = free
        self.allocs = []

    def probe(self, buf):
        return self.rates.pop(0)

    def alloc(self, n, dev):
        t = torch.empty(n, dtype=torch.uint8)
        self.allocs.append(t.data_ptr())
        return t

    def arena(self, **kw):
        return GP.GradsArena(probe=self.probe, free_bytes=lambda d: self.free, alloc=self.alloc, min_bytes=64,
                             require_cuda=False, **kw)


def acts(rows=8, V=16, dtype=torch.float32):
    return torch.randn(rows, V).to(dtype)


def test_keeps_fastest_of_candidates_and_stops_when_fast():
    f = Fake([5000.0, 5400.0, 6900.0, 1.0])
    ar = f.arena()
    g = ar.like(acts())
    assert ar.log[-1]["candidates_gbps"] == [5000.0, 5400.0, 6900.0] and ar.log[-1]["kept_gbps"] == 6900.0
    assert g.data_ptr() == f.allocs[2] and g.shape == (8, 16) and g.dtype == torch.float32 and g.is_contiguous()
    f2 = Fake([6500.0])
    ar2 = f2.arena()
    ar2.like(acts())
    assert ar2.log[-1]["candidates_gbps"] == [6500.0]  # fast first draw: no second candidate


def test_max_candidates_and_free_memory_limit():
    f = Fake([1.0, 3.0, 2.0, 9.0])
    ar = f.arena(max_candidates=3)
    g = ar.like(acts())
    assert ar.log[-1]["candidates_gbps"] == [1.0, 3.0, 2.0] and g.data_ptr() == f.allocs[1]
    f = Fake([1.0, 9.0], free=0)  # no room for a second candidate
    ar = f.arena()
    ar.like(acts())
    assert ar.log[-1]["candidates_gbps"] == [1.0]


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
