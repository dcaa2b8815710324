"""Where inside a slow-write grads buffer is it slow?  (the placement effect)

    python tools/chunk_probe.py [--buffers 3] [--chunk-gib 1] [--reps 3]

One process = the headline acts (52.7 GB synthetic) and several grads buffers of the same size from the caching
allocator, all held at once. For each buffer: the gradient kernel's time over the whole buffer (the class it
falls in), a nontemporal write over the whole buffer, then per chunk of --chunk-gib GiB a nontemporal write
and a nontemporal copy from the acts chunk at the same offset (the gradient pass's pairing) and from a shifted
acts chunk (a different physical pairing). Prints one JSON line: per buffer, the per-chunk write / copy rates in
GB/s, so a buffer that is slow only in some chunks (physical pages of one kind) is told apart from a buffer that
is slow everywhere (a property of the pairing or of the whole allocation).
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
ap.add_argument("--buffers", type=int, default=3)
ap.add_argument("--chunk-gib", type=int, default=1)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--windows", default="1,2,4,8,16", help="GiB: whole-buffer write as back-to-back launches of this size")
ap.add_argument("--no-chunks", action="store_true")
a = ap.parse_args()

dev = torch.device("cuda:0")
B, T, S, V = 64, 1000, 200, 1024
rows = B * T * (S + 1)
stream = torch.cuda.current_stream(dev)
sh = ctypes.c_void_p(stream.cuda_stream)
acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
L.synth_acts(acts.data_ptr(), 0, rows * V, 0, True, stream.cuda_stream)
labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, S)).astype(np.int32)).to(dev)
Tt, St = torch.full((B,), T, dtype=torch.int32), torch.full((B,), S, dtype=torch.int32)
tools = L.devtools()
lib = L.load()
nbytes = rows * V * 4
chunk = a.chunk_gib << 30
nchunks = nbytes // chunk


def time_ms(fn, reps=None):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps or a.reps):
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def ok(rc, what):
    if rc:
        raise RuntimeError(f"{what} failed ({rc})")


prep = op._Prepared(acts, labels, Tt, St, None, 0, 0)
_, ws = op._forward(prep, with_beta=True)
out = {"acts_ptr": hex(acts.data_ptr()), "chunk_gib": a.chunk_gib, "nchunks": int(nchunks), "buffers": []}
keep = []
for i in range(a.buffers):
    g = torch.empty_like(acts)
    keep.append(g)
    gp, ap_ = g.data_ptr(), acts.data_ptr()
    rec = {"k": i, "ptr": hex(gp)}
    rec["grad_ms"] = round(time_ms(lambda: ok(lib.mrnnt_backward(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                                                 None, ctypes.c_void_p(gp), sh), "backward")), 3)
    full = nbytes - nbytes % 16
    rec["write_full_gbps"] = round(full / (time_ms(lambda: ok(tools.mrnnt_write_probe(ctypes.c_void_p(gp), full, sh), "write")) * 1e-3) / 1e9, 1)
    wins = {}
    for wg in [int(x) for x in a.windows.split(",") if x]:
        step = wg << 30

        def windowed():
            for off in range(0, full, step):
                ok(tools.mrnnt_write_probe(ctypes.c_void_p(gp + off), min(step, full - off), sh), "write")
        wins[wg] = round(full / (time_ms(windowed) * 1e-3) / 1e9, 1)
    rec["write_windowed_gbps"] = wins
    w, c, cs = [], [], []
    for k in range(0 if a.no_chunks else nchunks):
        off = k * chunk
        sft = ((k + nchunks // 2) % nchunks) * chunk
        w.append(round(chunk / (time_ms(lambda: ok(tools.mrnnt_write_probe(ctypes.c_void_p(gp + off), chunk, sh), "write")) * 1e-3) / 1e9))
        c.append(round(2 * chunk / (time_ms(lambda: ok(tools.mrnnt_copy_probe(ctypes.c_void_p(gp + off), ctypes.c_void_p(ap_ + off), chunk, sh), "copy")) * 1e-3) / 1e9))
        cs.append(round(2 * chunk / (time_ms(lambda: ok(tools.mrnnt_copy_probe(ctypes.c_void_p(gp + off), ctypes.c_void_p(ap_ + sft), chunk, sh), "copy")) * 1e-3) / 1e9))
    rec["write_chunks"], rec["copy_chunks"], rec["copy_shifted_chunks"] = w, c, cs
    rec["summary"] = {n: [int(np.min(v)), int(np.median(v)), int(np.max(v))] for n, v in
                      (("write", w), ("copy", c), ("copy_shifted", cs)) if v}
    rec["summary"]["windowed"] = wins
    out["buffers"].append(rec)
    print(json.dumps({"k": i, "grad_ms": rec["grad_ms"], "write_full_gbps": rec["write_full_gbps"], **rec["summary"]}),
          file=sys.stderr, flush=True)
print(json.dumps(out), flush=True)
