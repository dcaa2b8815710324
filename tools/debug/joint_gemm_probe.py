"""Backward GEMMs of the fused joint at H = 512 (n = 3.9 M live rows, V = 1024): the forms torch / hipBLASLt offers.

  dH = G W      ([n, V] x [V, H] -> [n, H] bf16)
  dW = G^T Hact ([V, n] x [n, H] -> [V, H] fp32, split-K)
Prints one JSON object of median ms per form.
"""
import json
import time

import torch

dev = torch.device("cuda:0")
n, V, H = 3_893_785, 1024, 512
g = torch.Generator(device=dev).manual_seed(0)
G = (torch.randn(n, V, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
Hact = torch.randn(n, H, device=dev, generator=g).tanh().to(torch.bfloat16)
W = (torch.randn(V, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return round(ts[len(ts) // 2], 3)


out = {}
Wt = W.t().contiguous()
out["dH = G @ W"] = timeit(lambda: G @ W)
out["dH = G @ Wt.t() (W^T stored)"] = timeit(lambda: G @ Wt.t())
out["dH^T = W^T @ G^T"] = timeit(lambda: (W.t() @ G.t()))
out["dH fp32 out"] = timeit(lambda: torch.mm(G, W, out_dtype=torch.float32))
for c in (2, 4, 8):
    m = n // c

    def chunked(c=c, m=m):
        o = torch.empty(n, H, device=dev, dtype=torch.bfloat16)
        for i in range(c):
            hi = n if i == c - 1 else (i + 1) * m
            torch.mm(G[i * m:hi], W, out=o[i * m:hi])
        return o
    out[f"dH chunked {c}"] = timeit(chunked)


def splitk(chunks):
    mm = n // chunks
    head = chunks * mm
    part = torch.bmm(G[:head].view(chunks, mm, -1).transpose(1, 2), Hact[:head].view(chunks, mm, -1),
                     out_dtype=torch.float32).sum(0)
    if head < n:
        part += torch.mm(G[head:].t(), Hact[head:], out_dtype=torch.float32)
    return part


for c in (8, 16, 32, 64, 128):
    out[f"dW split-K bmm {c}"] = timeit(lambda c=c: splitk(c))
out["dW single mm fp32"] = timeit(lambda: torch.mm(G.t(), Hact, out_dtype=torch.float32))
out["dW single mm bf16"] = timeit(lambda: torch.mm(G.t(), Hact))
out["read G once (sum)"] = timeit(lambda: G.sum(dtype=torch.float32))
print(json.dumps(out, indent=1), flush=True)
