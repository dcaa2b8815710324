"""dW = G^T Hact with a wider Hact (ones column for dbias): split-K GEMM time per Hact row stride, against
G.sum(0) -- picks the stride at which folding dbias into the GEMM pays (n live rows of the H = 512 / 256
headline joint runs, V = 1024)."""
import json
import sys

import torch

dev = torch.device("cuda:0")


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 3)


def splitk(G, Hact, chunks=32):
    n = G.shape[0]
    m = n // chunks
    head = chunks * m

    def f():
        p = torch.bmm(G[:head].view(chunks, m, -1).transpose(1, 2), Hact[:head].view(chunks, m, -1),
                      out_dtype=torch.float32).sum(0)
        if head < n:
            p += torch.mm(G[head:].t(), Hact[head:], out_dtype=torch.float32)
        return p
    return f


res = {}
V = 1024
CASES = {512: (512, 520, 528, 544, 576, 640, 768), 256: (256, 264, 272, 288, 320, 384), 128: (128, 136, 144, 160, 192, 256),
         384: (384, 392, 400, 416, 448, 512), 640: (640, 648, 656, 672, 704, 768)}
for H in [int(h) for h in sys.argv[1:]] or (512, 256):
    n, lds = 3893785, CASES[H]
    G = torch.randn(n, V, device=dev).to(torch.bfloat16)
    r = {"G.sum(0)": t(lambda: G.sum(0, dtype=torch.float32))}
    for ld in lds:
        Hact = torch.randn(n, ld, device=dev).to(torch.bfloat16)
        r[f"splitK ld={ld}"] = t(splitk(G, Hact))
        del Hact
    res[f"H={H}"] = r
    del G
    torch.cuda.empty_cache()
    print(json.dumps({f"H={H}": r}), flush=True)
json.dump(res, sys.stdout, indent=1)
