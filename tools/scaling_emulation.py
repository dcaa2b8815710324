"""Per-rank work of the batch-sharded configs[3] (B=512 ragged, V=1024) measured on ONE MI355X.

  python tools/scaling_emulation.py [--worlds 2,4,8] [--steps 3] [--warmup 1]

The sharded path has no data-path collective: rank r of N runs the single-GPU path on its
contiguous utterance slice (bench.shard_bounds, balanced by rows) and the only exchange is one 4-byte loss
all-reduce. So the N-GPU step time is max over ranks of the slice time (+ the all-reduce latency, ~10-30 us),
and the slices can be timed one after another on one GPU. For every N this tool runs every rank's slice
(synthetic acts regenerated per slice, untimed), times `steps` loss+grad steps with HIP events, and reports
per-rank ms, the emulated N-GPU step (max) and utt/s. The 1-GPU number for the whole batch (292 GB of acts
does not fit 288 GB of HBM) is the sum of the N=2 slices, i.e. the batch run as two chunks.

Grads are written in place over acts when acts + grads would not fit (the reference extension's output-buffer
form, monotonic_rnnt_cpp.gpu_monotonic_rnnt(..., grads=acts)); the gradient kernel reads every element of a
row before it writes it, and the log-softmax pass is complete by then, so in-place is exact.
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
sys.path.insert(0, ROOT)

HBM_BUDGET = 250e9  # bytes of acts (+ grads) this tool lets one slice use


def run_slice(op, L, lib, T, S, V, row0, steps, warmup, dev):
    B = len(T)
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
    inplace = 2 * acts.numel() * 4 > HBM_BUDGET
    grads = acts if inplace else torch.empty_like(acts)
    labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, int(S.max()))).astype(np.int32)).to(dev)
    T_t, S_t = torch.from_numpy(T), torch.from_numpy(S)
    costs = torch.zeros(B, device=dev)
    times = []
    for i in range(warmup + steps):
        # regenerate the inputs every step (an in-place step overwrote them); not timed
        L.check(lib.mrnnt_synth_acts(ctypes.c_void_p(acts.data_ptr()), row0 * V, rows * V, 0, 1, stream), "synth")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(acts, labels, T_t, S_t, costs, grads, 0)
        e1.record()
        torch.cuda.synchronize()
        if i >= warmup:
            times.append(e0.elapsed_time(e1))
    finite = bool(torch.isfinite(costs).all().item())
    del acts, grads
    torch.cuda.empty_cache()
    return {"utterances": B, "rows": rows, "acts_gb": round(rows * V * 4 / 1e9, 2), "inplace_grads": inplace,
            "ms": round(float(np.median(times)), 3), "finite": finite}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import monotonic_rnnt_op as op
    import _mrnnt_lib as L
    from bench import lengths_for

    lib = L.load()
    dev = torch.device("cuda:0")
    out = {"workload": "configs[3]: B=512, T~U[200,1600], S~U[20,min(300,T)] (seed 0), V=1024, fp32",
           "method": "every rank's slice timed in turn on one GPU (no data-path collective; N-GPU step = max "
                     "over ranks + one 4-byte all-reduce, not included)", "worlds": {}}
    for N in [int(x) for x in args.worlds.split(",")]:
        ranks, row0 = [], 0
        for r in range(N):
            T, S, V, _ = lengths_for("ragged", r, N)
            res = run_slice(op, L, lib, T, S, V, row0, args.steps, args.warmup, dev)
            row0 += res["rows"]
            ranks.append(res)
            print(json.dumps({"N": N, "rank": r, **res}), file=sys.stderr, flush=True)
        step = max(x["ms"] for x in ranks)
        out["worlds"][N] = {"ranks": ranks, "step_ms": step, "utt_per_s": round(512 / (step * 1e-3), 1),
                            "sum_ms": round(sum(x["ms"] for x in ranks), 3),
                            "balance": round(min(x["ms"] for x in ranks) / step, 4)}
    if 2 in out["worlds"]:
        s = out["worlds"][2]["sum_ms"]
        out["one_gpu_two_chunks"] = {"step_ms": s, "utt_per_s": round(512 / (s * 1e-3), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
