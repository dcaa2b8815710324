"""hipBLASLt timings for the joint backward's GEMM shapes (n live rows = 3.89 M at the headline, V = 1024, H = 512):
dH = G @ W (bf16 out) and dW = G^T Hact (fp32, split-K batched vs single)."""
import json
import torch

dev = torch.device("cuda:0")
n, V, H = 3893785, 1024, 512
G = torch.randn(n, V, device=dev).to(torch.bfloat16)
Hact = torch.randn(n, H, device=dev).to(torch.bfloat16)
W = torch.randn(V, H, device=dev).to(torch.bfloat16)


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def splitk(chunks, out_dtype=torch.float32):
    m = n // chunks
    head = chunks * m
    def f():
        p = torch.bmm(G[:head].view(chunks, m, -1).transpose(1, 2), Hact[:head].view(chunks, m, -1),
                      out_dtype=out_dtype).sum(0, dtype=torch.float32)
        if head < n:
            p += torch.mm(G[head:].t(), Hact[head:], out_dtype=torch.float32)
        return p
    return f


res = {}
flop = 2.0 * n * V * H
res["dH = G @ W"] = t(lambda: G @ W)
res["dH = (W^T G^T)^T"] = t(lambda: (W.t() @ G.t()).t())
res["dH mm out fp32"] = t(lambda: torch.mm(G, W, out_dtype=torch.float32))
for ch in (8, 16, 32, 64, 128):
    res[f"dW splitK {ch} fp32"] = t(splitk(ch))
res["dW single mm fp32"] = t(lambda: torch.mm(G.t(), Hact, out_dtype=torch.float32))
res["dW single mm bf16"] = t(lambda: G.t() @ Hact)
res["db G.sum(0)"] = t(lambda: G.sum(0, dtype=torch.float32))
print(json.dumps({k: {"ms": round(v, 3), "tflops": round(flop / (v * 1e-3) / 1e12, 1)} for k, v in res.items()}, indent=1))
