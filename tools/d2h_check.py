#!/usr/bin/env python3
"""Eager training steps of the configs[1] shape with the lengths on the GPU or on the host, for a rocprofv3
memory-copy trace (an eager step with device lengths makes no device-to-host copy).

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- python3 tools/d2h_check.py --lengths device
  python3 tools/d2h_check.py --summarise DIR     # copies by direction inside the steps (first to last kernel)

The steps read nothing back; after them one .item() (outside the step window) checks the loss is finite.
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lengths: str, steps: int):
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
    import monotonic_rnnt_op as op
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    B, T, S, V = 16, 200, 40, 256
    acts = torch.randn(B * T * (S + 1), V, device=dev, requires_grad=True)
    labels = torch.from_numpy(rng.integers(1, V, (B, S)).astype(np.int32)).to(dev)
    Tl = torch.full((B,), T, dtype=torch.int32)
    Sl = torch.full((B,), S, dtype=torch.int32)
    if lengths == "device":
        Tl, Sl = Tl.to(dev), Sl.to(dev)
    for _ in range(3):  # warm-up (allocations, the status word, the host-lengths upload)
        acts.grad = None
        op.monotonic_rnnt_loss(acts, labels, Tl, Sl).sum().backward()
    torch.cuda.synchronize()
    loss = None
    for _ in range(steps):
        acts.grad = None
        loss = op.monotonic_rnnt_loss(acts, labels, Tl, Sl).sum()
        loss.backward()
    torch.cuda.synchronize()
    assert np.isfinite(loss.item())


def summarise(d: str):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ks = []
    with open(kt) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    sm = [k for k in ks if "softmax" in k[2]]
    gr = [k for k in ks if "grad_" in k[2]]
    # the timed steps: from the first log-softmax after the 3 warm-up steps to the last gradient kernel
    lo, hi = sm[3][0], gr[-1][1]
    copies = {}
    total = {}
    if mc:
        with open(mc[0]) as f:
            for r in csv.DictReader(f):
                direction = r.get("Direction") or r.get("Kind") or "?"
                s = int(r["Start_Timestamp"])
                total[direction] = total.get(direction, 0) + 1
                if lo <= s <= hi:
                    copies[direction] = copies.get(direction, 0) + 1
    # ROCm runs small pageable copies as blit kernels (__amd_rocclr_copyBuffer), which the memory-copy trace does not
    # list: count every kernel launched inside the window by name
    inside = {}
    for b, e, n in ks:
        if lo <= b <= hi:
            key = n.split("(")[0].replace("void ", "")[:60]
            inside[key] = inside.get(key, 0) + 1
    blits = sum(v for k, v in inside.items() if "rocclr" in k)
    print(json.dumps({"kernel_trace": kt, "steps_window_ns": [lo, hi], "log_softmax_launches_in_window":
                      sum(1 for k in sm if lo <= k[0] <= hi), "memory_copies_in_steps": copies,
                      "memory_copies_whole_run": total, "blit_copy_kernels_in_steps": blits,
                      "kernels_in_steps": inside}, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--lengths", default="device", choices=["device", "host"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--summarise", default=None)
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a.lengths, a.steps)
