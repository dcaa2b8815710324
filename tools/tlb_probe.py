"""Why is the gradient pass slow on some grads buffers? Time and count it per buffer, in one process.

    python tools/tlb_probe.py [--buffers 3] [--reps 5]
    rocprofv3 --pmc <counters> -d DIR -o run --output-format csv -- python3 tools/tlb_probe.py

For each of several 52.7 GB grads buffers (torch allocations, as bench.py's autograd path makes them) this times,
in this order, with HIP events:
  grad      the gradient kernel writing that buffer (headline workload, mrnnt_backward through the C ABI)
  copy_full the nontemporal copy probe acts -> buffer over the WHOLE 52.7 GB
  copy_8g   the same probe over the first 8 GiB only
Each is one warm-up launch + `reps` timed launches, so under rocprofv3 the dispatches map onto (buffer, probe)
in order. Round 2 (profiles/r02/placement_probe_b.jsonl): about one buffer in three makes the gradient kernel
15.3-16.0 ms instead of 12.5-13.4, in every launch shape, while an 8 GiB copy into the same buffer is as fast
as into any other. The question this answers: does the whole-buffer copy see it too (a property of the
buffer's full extent, e.g. its page-table footprint), and which counters move with it.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
import monotonic_rnnt_op as op  # noqa: E402
import _mrnnt_lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--buffers", type=int, default=3)
ap.add_argument("--scan-gib", type=int, default=0, help="also copy into every SCAN-GiB sub-range of each buffer")
a = ap.parse_args()
dev = torch.device("cuda:0")
B, T, S, V = 64, 1000, 200, 1024
rows = B * T * (S + 1)
stream = torch.cuda.current_stream(dev)
sh = stream.cuda_stream
acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
L.synth_acts(acts.data_ptr(), 0, rows * V, 0, True, sh)
labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, S)).astype(np.int32)).to(dev)
Tt, St = torch.full((B,), T, dtype=torch.int32), torch.full((B,), S, dtype=torch.int32)
prep = op._Prepared(acts, labels, Tt, St, None, 0, 0)
_, ws = op._forward(prep, with_beta=True)
lib = L.load()
tools = L.devtools()
nbytes = rows * V * 4


def time_ms(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(a.reps):
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def copy(ptr, n):
    n -= n % 16
    return lambda: tools.mrnnt_copy_probe(ctypes.c_void_p(ptr), ctypes.c_void_p(acts.data_ptr()), n, ctypes.c_void_p(sh))


out = {"acts_ptr": hex(acts.data_ptr()), "buffers": []}
keep = []
for i in range(a.buffers):
    g = torch.empty_like(acts)
    keep.append(g)
    p = g.data_ptr()
    gm = time_ms(lambda: L.check(lib.mrnnt_backward(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()), None,
                                                    ctypes.c_void_p(p), ctypes.c_void_p(sh)), "backward"))
    cf = time_ms(copy(p, nbytes))
    c8 = time_ms(copy(p, 8 << 30))
    rec = {"k": i, "ptr": hex(p), "grad_ms": round(gm, 3),
           "copy_full_gbps": round(2 * (nbytes - nbytes % 16) / (cf * 1e-3) / 1e9, 1),
           "copy_8g_gbps": round(2 * (8 << 30) / (c8 * 1e-3) / 1e9, 1)}
    if a.scan_gib:
        sub = a.scan_gib << 30
        rec["scan_gbps"] = [round(2 * sub / (time_ms(copy(p + o, sub)) * 1e-3) / 1e9)
                            for o in range(0, nbytes - sub + 1, sub)]
    out["buffers"].append(rec)
print(json.dumps(out), flush=True)
