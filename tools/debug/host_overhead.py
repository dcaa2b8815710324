"""Host-side cost of one loss step at a small config (configs[1]: B=16, T=200, S=40, V=256), piece by piece.

    python tools/debug/host_overhead.py [--iters 300]

Prints per-step microseconds: the whole step issued back to back (GPU time included when the GPU is the bound),
then each host piece alone (the GPU is far from saturated at this size, so these are host times).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
import monotonic_rnnt_op as op  # noqa: E402
import _mrnnt_lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=300)
args = ap.parse_args()
dev = torch.device("cuda:0")
B, T, S, V = 16, 200, 40, 256
Tn = np.full(B, T, np.int32)
Sn = np.full(B, S, np.int32)
acts = torch.randn(B * T * (S + 1), V, device=dev).requires_grad_(True)
labels = torch.randint(1, V, (B, S), dtype=torch.int32, device=dev)
T_t, S_t = torch.from_numpy(Tn), torch.from_numpy(Sn)
res = {}


def timeit(name, fn, n=args.iters):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res[name] = {"issue_us": round((t1 - t0) / n * 1e6, 1), "with_drain_us": round((t2 - t0) / n * 1e6, 1)}


def step():
    acts.grad = None
    op.monotonic_rnnt_loss(acts, labels, T_t, S_t).sum().backward()


timeit("full step (autograd)", step)
L.profile_enable(True)
timeit("full step, per-kernel events on", step)
L.profile_enable(False)
timeit("forward only (autograd, no grad)", lambda: op.monotonic_rnnt_loss(acts.detach(), labels, T_t, S_t))
timeit("_Prepared", lambda: op._Prepared(acts, labels, T_t, S_t, None, 0, 0))
prep = op._Prepared(acts, labels, T_t, S_t, None, 0, 0)
timeit("prep.workspace()", prep.workspace)
timeit("_forward(with_beta)", lambda: op._forward(prep, True))
_, ws = op._forward(prep, True)
timeit("_backward", lambda: op._backward(prep, ws, None))
lib = L.load()
costs = torch.empty(B, device=dev)
wsp, wsn = ctypes.c_void_p(ws.data_ptr()), ws.numel()
cp = ctypes.c_void_p(costs.data_ptr())
st = prep.stream()
timeit("mrnnt_forward (ctypes call only)", lambda: lib.mrnnt_forward(ctypes.byref(prep.problem), wsp, wsn, cp, 1, st))
grads = torch.empty_like(acts)
gp = ctypes.c_void_p(grads.data_ptr())
timeit("mrnnt_backward (ctypes call only)", lambda: lib.mrnnt_backward(ctypes.byref(prep.problem), wsp, None, gp, st))
timeit("torch.empty_like(acts)", lambda: torch.empty_like(acts))
timeit("lengths cache lookup", lambda: op._lengths(T_t, S_t).on(dev))


def ctx():
    with torch.cuda.device(dev):
        pass


timeit("torch.cuda.device ctx", ctx)
print(json.dumps(res, indent=1))
