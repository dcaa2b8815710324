"""Per-step kernel times of the headline step over a long run (is the gradient kernel's rate stable in time?).

  python tools/step_trace.py [--steps N] [--config headline] [--acts-dtype f32]

Prints one JSON object: per step the forward (log-softmax + recursion) and backward (gradient kernel) times
from torch.cuda events on the current stream (the stream the op launches on), and the wall time.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--config", default="headline")
    ap.add_argument("--acts-dtype", default="f32")
    a = ap.parse_args()
    import monotonic_rnnt_op as op
    import _mrnnt_lib as L
    from bench import lengths_for
    lib = L.load()
    dev = torch.device("cuda:0")
    T, S, V, workload = lengths_for(a.config, 0, 1)[:4]
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
    L.synth_acts(acts.data_ptr(), 0, rows * V, 0, True, stream.value)
    if a.acts_dtype != "f32":
        acts = acts.to(torch.bfloat16 if a.acts_dtype == "bf16" else torch.float16)
        torch.cuda.empty_cache()
    labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (len(T), int(S.max()))).astype(np.int32)).to(dev)
    T_t, S_t = torch.from_numpy(T), torch.from_numpy(S)
    acts.requires_grad_(True)
    out = []
    t_start = time.perf_counter()
    for i in range(a.steps):
        acts.grad = None
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        costs = op.monotonic_rnnt_loss(acts, labels, T_t, S_t, blank_label=0)
        loss = costs.sum()
        e[1].record()
        loss.backward()
        e[2].record()
        torch.cuda.synchronize()
        out.append({"step": i, "t": round(time.perf_counter() - t_start, 3), "fwd_ms": round(e[0].elapsed_time(e[1]), 3),
                    "bwd_ms": round(e[1].elapsed_time(e[2]), 3)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
