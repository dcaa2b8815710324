"""Fused joint network + loss vs the unfused pipeline it replaces, on one MI355X.

  python tools/joint_bench.py [--B 64 --T 1000 --S 200 --V 1024 --H 512] [--steps 5] [--warmup 2] [--no-unfused]

fused   : monotonic_rnnt_joint_loss(enc, pred, W, b, ...).sum().backward()
unfused : h = tanh(enc[:, :, None] + pred[:, None]); z = h @ W.T + b  (bf16 [B, T, S+1, V], torch / hipBLASLt);
          monotonic_rnnt_loss(z, ...) on the padded bf16 layout (read in place); .sum().backward() through autograd
Both compute the same loss and gradients for enc, pred, W, b. Synthetic N(0, 1) enc/pred, W ~ N(0, 4/H), bias
N(0, 0.01). Prints one JSON object: ms per step, utt/s, per-kernel ms and TFLOP/s of the fused kernels against
the dense bf16 MFMA peak (2.5 PFLOP/s, MI355X_MICROARCH.md), live-row fraction, max |cost difference|.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))

PEAK_TFLOPS = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--S", type=int, default=200)
    ap.add_argument("--V", type=int, default=1024)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-unfused", action="store_true")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--align-k", type=int, default=None,
                    help="alignment-restricted loss (max_distance_from_alignment = K) on bench.py's synthetic alignment")
    ap.add_argument("--ab", default=None, metavar="JSON",
                    help="list of knob dicts: after the main line, interleaved rounds of one fused step per variant "
                         "(per-kernel library timings, median over --ab-rounds)")
    ap.add_argument("--ab-rounds", type=int, default=7)
    a = ap.parse_args()
    import _mrnnt_lib as L
    import monotonic_rnnt_joint as J
    import monotonic_rnnt_op as op

    if a.tune or a.ab:
        L.select_dev()  # launch knobs live in the development build
    for kv in a.tune:
        k, v = kv.split("=")
        assert L.tune(k, int(v)) >= 0, k
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    B, T, S, V, H = a.B, a.T, a.S, a.V, a.H
    enc = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    pred = torch.randn(B, S + 1, H, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
    W = (torch.randn(V, H, device=dev, generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16).requires_grad_(True)
    bias = (0.1 * torch.randn(V, device=dev, generator=g)).requires_grad_(True)
    labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, S)).astype(np.int32)).to(dev)
    Tl = torch.full((B,), T, dtype=torch.int32)
    Sl = torch.full((B,), S, dtype=torch.int32)
    n_band = B * ((S + 1) * (T - S + 1) - 1)
    al, k = None, 0
    if a.align_k is not None:
        sys.path.insert(0, ROOT)
        from bench import synthetic_alignment
        al_np, n_band = synthetic_alignment(labels.cpu().numpy(), Tl.numpy(), Sl.numpy(), a.align_k)
        al, k = torch.from_numpy(al_np).to(dev), a.align_k  # n_band: the rows the forward computes

    def fused():
        for x in (enc, pred, W, bias):
            x.grad = None
        c = J.monotonic_rnnt_joint_loss(enc, pred, W, bias, labels, Tl, Sl, alignment=al, max_distance_from_alignment=k)
        c.sum().backward()
        return c

    def unfused():
        for x in (enc, pred, W, bias):
            x.grad = None
        h = torch.tanh(enc[:, :, None, :] + pred[:, None, :, :])
        z = torch.nn.functional.linear(h, W, bias.to(torch.bfloat16))  # [B, T, S+1, V] bf16
        c = op.monotonic_rnnt_loss(z, labels, Tl, Sl, al, k)
        c.sum().backward()
        return c

    def timeit(fn, prof=False):
        for _ in range(a.warmup):
            fn()
        torch.cuda.synchronize()
        if prof:
            L.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            c = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        pr = L.profile_read() if prof else None
        if prof:
            L.profile_enable(False)
        return dt, c.detach(), pr

    out = {"config": {"B": B, "T": T, "S": S, "V": V, "H": H, "dtype": "bf16 operands, fp32 accumulate",
                      "align_k": a.align_k},
           "tune": a.tune or None}
    dt, c_f, pr = timeit(fused, prof=True)
    # live rows of the backward pass (the gradient kernel's row count)
    prep = J._JointPrepared(enc.detach(), pred.detach(), W.detach(), bias.detach(), labels, Tl, Sl, 0, al, k)
    _, ws = prep.forward(with_beta=True)
    G, _ = prep.backward_rows(ws, None)
    n_live = G.shape[0]
    del G, ws
    ms = lambda k: pr[k][0] / max(1, pr[k][1])  # noqa: E731
    f_fwd = 2.0 * n_band * V * H
    f_bwd = 2.0 * n_live * V * H
    out["fused"] = {
        "ms_per_step": round(dt * 1e3, 3), "utt_per_s": round(B / dt, 1),
        "forward_rows": n_band, "live_rows": n_live, "live_frac": round(n_live / n_band, 4),
        "kernels_ms": {"joint_fwd": round(ms("joint_fwd"), 3), "alpha_beta": round(ms("alpha_beta"), 3),
                       "joint_bwd": round(ms("joint_bwd"), 3), "joint_reduce": round(ms("joint_reduce"), 3),
                       "joint_dpre": round(ms("joint_dpre"), 3)},
        "joint_dpre_tflops": round(f_bwd * H / H / (ms("joint_dpre") * 1e-3) / 1e12, 1) if pr["joint_dpre"][1] else None,
        "joint_fwd_tflops": round(f_fwd / (ms("joint_fwd") * 1e-3) / 1e12, 1),
        "joint_bwd_tflops": round(f_bwd / (ms("joint_bwd") * 1e-3) / 1e12, 1),
        "peak_tflops": PEAK_TFLOPS,
    }
    out["fused"]["joint_fwd_frac"] = round(out["fused"]["joint_fwd_tflops"] / PEAK_TFLOPS, 4)
    out["fused"]["joint_bwd_frac"] = round(out["fused"]["joint_bwd_tflops"] / PEAK_TFLOPS, 4)
    if not a.no_unfused:
        torch.cuda.empty_cache()
        dt_u, c_u, _ = timeit(unfused)
        out["unfused"] = {"ms_per_step": round(dt_u * 1e3, 3), "utt_per_s": round(B / dt_u, 1),
                          "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1)}
        out["speedup"] = round(dt_u / dt, 3)
        out["max_rel_cost_diff"] = float(((c_f.double() - c_u.double()).abs() / c_u.double().abs().clamp(min=1))
                                         .max().item())
    if a.ab:
        variants = json.loads(a.ab)
        saved = [{k: L.tune(k) for k in v} for v in variants]
        runs = [dict() for _ in variants]
        steps = [[] for _ in variants]
        for r in range(a.ab_rounds):
            for vi, v in enumerate(variants):
                for k, x in v.items():
                    assert L.tune(k, int(x)) >= 0, k
                fused()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fused()
                e1.record()
                torch.cuda.synchronize()
                steps[vi].append(e0.elapsed_time(e1))
                L.profile_enable(True)
                fused()
                torch.cuda.synchronize()
                pr = L.profile_read()
                L.profile_enable(False)
                for k in ("joint_fwd", "joint_bwd", "joint_reduce", "joint_dpre"):
                    if pr[k][1]:
                        runs[vi].setdefault(k, []).append(pr[k][0] / pr[k][1])
                for k, x in saved[vi].items():
                    L.tune(k, x)
        out["ab"] = [{"knobs": v, "step_ms_median": round(float(np.median(steps[vi])), 3),
                      "step_ms_min": round(float(np.min(steps[vi])), 3),
                      "median_ms": {k: round(float(np.median(x)), 4) for k, x in runs[vi].items()},
                      "min_ms": {k: round(float(np.min(x)), 4) for k, x in runs[vi].items()}}
                     for vi, v in enumerate(variants)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
