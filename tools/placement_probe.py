"""Does a fresh process draw a slow gradient buffer, and which launch shape / allocation avoids it?

    python tools/placement_probe.py [--reps 5] [--buffers 4]

One process = the headline workload as bench.py builds it (acts 52.7 GB synthetic, grads from the caching
allocator). For each of several grads buffers (torch allocations, a hipMalloc and a hipExtMallocWithFlags
contiguous buffer) it times the gradient kernel (mrnnt_backward through the C ABI of the development build) under
a few launch variants (column visiting order, workgroups per CU) and the nontemporal copy probe into it. Prints
one JSON line. Run it in several fresh processes: round 1 saw about one process in four with a gradient kernel
15.4-15.9 ms instead of 12.4-13.4 ms (profiles/r01/grad_placement_study.json).
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
ap.add_argument("--buffers", type=int, default=3, help="torch grads buffers per process")
ap.add_argument("--variants", default="scatter:col_scatter=2;inorder:col_scatter=0;inorder8:col_scatter=0,grad_grid_per_cu=8;scatter8:col_scatter=2,grad_grid_per_cu=8")
a = ap.parse_args()
VARIANTS = [(v.split(":")[0], dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(":")[1].split(",")))
            for v in a.variants.split(";")]
dev = torch.device("cuda:0")
B, T, S, V = 64, 1000, 200, 1024
rows = B * T * (S + 1)
stream = torch.cuda.current_stream(dev)
sh = stream.cuda_stream
acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
L.synth_acts(acts.data_ptr(), 0, rows * V, 0, True, sh)
labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, S)).astype(np.int32)).to(dev)
Tt, St = torch.full((B,), T, dtype=torch.int32), torch.full((B,), S, dtype=torch.int32)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
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
    return round(float(np.median(ts)), 3)


with L.use(L.load_dev()):
    lib = L.load()
    prep = op._Prepared(acts, labels, Tt, St, None, 0, 0)
    _, ws = op._forward(prep, with_beta=True)

    def probe(ptr):
        res = {"ptr": hex(ptr)}
        for name, kn in VARIANTS:
            saved = {k: L.tune(k, v) for k, v in kn.items()}
            res[name] = time_ms(lambda: L.check(lib.mrnnt_backward(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                                                   None, ctypes.c_void_p(ptr), ctypes.c_void_p(sh)),
                                                "backward"))
            for k, v in saved.items():
                L.tune(k, v)
        n = 8 << 30
        c = time_ms(lambda: L.devtools().mrnnt_copy_probe(ctypes.c_void_p(ptr), ctypes.c_void_p(acts.data_ptr()), n,
                                                          ctypes.c_void_p(sh)))
        res["copy_gbps"] = round(2 * n / (c * 1e-3) / 1e9, 1)
        return res

    out = {"acts_ptr": hex(acts.data_ptr()), "buffers": []}
    keep = []
    for i in range(a.buffers):
        g = torch.empty_like(acts)
        keep.append(g)
        out["buffers"].append({"kind": f"torch{i}", **probe(g.data_ptr())})
    del keep
    torch.cuda.empty_cache()
    for name, alloc in (("hipMalloc", lambda p: hip.hipMalloc(ctypes.byref(p), nbytes)),
                        ("contiguous", lambda p: hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, 4))):
        p = ctypes.c_void_p()
        rc = alloc(p)
        if rc != 0 or not p.value:
            out["buffers"].append({"kind": name, "error": rc})
            continue
        out["buffers"].append({"kind": name, **probe(p.value)})
        torch.cuda.synchronize()
        hip.hipFree(p)
print(json.dumps(out), flush=True)
