"""A/B of the joint backward's dH GEMM on one MI355X: mrnnt_joint_dpre (hand-written MFMA, dpre = (G W)(1 - Hact^2))
in its launch variants (development build knob joint_dpre_nw) against hipBLASLt's dH = G W (torch), on synthetic
operands of the headline joint size (n live rows, V, H as tools/joint_bench.py measures them: n = 3,893,785 at
B = 64, T = 1000, S = 200, V = 1024, H = 512).

  python tools/dpre_bench.py [--n 3893785] [--V 1024] [--H 512] [--reps 10] [--variants '[{"joint_dpre_nw": 8}, ...]']

Prints one JSON object: per variant the median / min ms (HIP events, rocprof-comparable), TFLOP/s and fraction of the
2.5 PF dense bf16 peak, and the bytes moved / achieved GB/s; every variant's output is checked bit-identical to the
first one's and within bf16 tolerance of torch's fp32 product.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))

PEAK = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3893785)
    ap.add_argument("--V", type=int, default=1024)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default='[{"joint_dpre_nw": 0}, {"joint_dpre_nw": 2}, {"joint_dpre_nw": 1}]')
    a = ap.parse_args()
    import _mrnnt_lib as L
    L.select_dev()
    import monotonic_rnnt_joint as J

    dev = torch.device("cuda:0")
    n, V, H = a.n, a.V, a.H
    # a joint problem with at least n in-band rows (mrnnt_joint_dpre checks n against it)
    B, T, S = 64, 1000, 200
    g = torch.Generator(device=dev).manual_seed(0)
    enc = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16)
    pred = torch.randn(B, S + 1, H, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(V, H, device=dev, generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16)
    labels = torch.randint(1, V, (B, S), device=dev, dtype=torch.int32)
    prep = J._JointPrepared(enc, pred, W, None, labels, torch.full((B,), T, dtype=torch.int32),
                            torch.full((B,), S, dtype=torch.int32), 0)
    G = (torch.randn(n, V, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    Hact = torch.tanh(torch.randn(n, H, device=dev, generator=g)).to(torch.bfloat16)
    prep.problem.hact_ld = H
    flop = 2.0 * n * V * H
    bytes_dpre = (n * V + 2 * n * H) * 2  # G read, Hact read, dpre written
    bytes_blas = (n * V + n * H) * 2      # G read, dH written

    def time_it(fn, reps):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        fn()
        torch.cuda.synchronize()
        for s, e in ev:
            s.record()
            fn()
            e.record()
        torch.cuda.synchronize()
        return [s.elapsed_time(e) for s, e in ev]

    out = {"n": n, "V": V, "H": H, "tflop": round(flop / 1e12, 3), "variants": []}
    ref = None
    for v in json.loads(a.variants):
        saved = {k: L.tune(k) for k in v}
        for k, x in v.items():
            assert L.tune(k, int(x)) >= 0, k
        res = {}
        t = time_it(lambda: res.__setitem__("d", prep.dpre(G, Hact)), a.reps)
        d = res["d"]
        if ref is None:
            ref = d.clone()
        # the forms sum the same products in different k orders within an MFMA: compare within bf16 rounding
        same = bool(torch.equal(d, ref))
        diff = float((d.float() - ref.float()).abs().max().item())
        med = float(np.median(t))
        out["variants"].append({"knobs": v, "median_ms": round(med, 4), "min_ms": round(min(t), 4),
                                "tflops": round(flop / (med * 1e-3) / 1e12, 1),
                                "frac_of_peak": round(flop / (med * 1e-3) / 1e12 / PEAK, 4),
                                "gbps": round(bytes_dpre / (med * 1e-3) / 1e9, 1), "bit_identical_to_first": same,
                                "max_abs_diff_to_first": diff})
        for k, x in saved.items():
            L.tune(k, x)
    # hipBLASLt dH (what the library path replaced), same operands
    Wt = W.t().contiguous()
    t = time_it(lambda: G @ Wt.t(), a.reps)
    med = float(np.median(t))
    out["hipblaslt_dH"] = {"median_ms": round(med, 4), "min_ms": round(min(t), 4),
                           "tflops": round(flop / (med * 1e-3) / 1e12, 1), "gbps": round(bytes_blas / (med * 1e-3) / 1e9, 1)}
    # accuracy of the first variant on a sample of rows against torch's fp32 product
    idx = torch.arange(0, n, max(1, n // 4096), device=dev)
    r = (G[idx].float() @ W.float()) * (1.0 - Hact[idx].float() ** 2)
    err = (ref[idx].float() - r).abs()
    out["max_abs_err_vs_fp32"] = float(err.max().item())
    out["max_ref"] = float(r.abs().max().item())
    out["within_tol"] = bool((err <= 2.0 ** -7 * r.abs() + 1e-3 * r.abs().max()).all().item())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
