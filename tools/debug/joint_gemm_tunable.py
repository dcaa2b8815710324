"""How far hipBLASLt's other solutions go for the fused joint's two backward GEMMs at H = 512 (n = 3.9 M live
rows, V = 1024), against the heuristic's first choice: torch TunableOp times every candidate solution for the shape
(PYTORCH_TUNABLEOP_* set below, before torch initialises the GPU) and keeps the fastest.

Prints one JSON object: median ms per form with the heuristic choice (tunable off) and with the tuned choice.
"""
import json
import os
import sys

mode = sys.argv[1] if len(sys.argv) > 1 else "off"
if mode == "tuned":
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
    os.environ["PYTORCH_TUNABLEOP_VERBOSE"] = "0"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.environ.get("TUNABLE_FILE", "gpurun_out/tunableop_results.csv")
    os.environ["PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS"] = "2000"
import torch  # noqa: E402

dev = torch.device("cuda:0")
n, V, H = 3_893_785, 1024, 512
g = torch.Generator(device=dev).manual_seed(0)
G = (torch.randn(n, V, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
Hact = torch.randn(n, H, device=dev, generator=g).tanh().to(torch.bfloat16)
W = (torch.randn(V, H, device=dev, generator=g) * 0.05).to(torch.bfloat16)
Wt = W.t().contiguous()


def timeit(fn, reps=7):
    for _ in range(2):
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


def splitk(chunks=32):
    mm = n // chunks
    head = chunks * mm
    part = torch.bmm(G[:head].view(chunks, mm, -1).transpose(1, 2), Hact[:head].view(chunks, mm, -1),
                     out_dtype=torch.float32).sum(0)
    if head < n:
        part += torch.mm(G[head:].t(), Hact[head:], out_dtype=torch.float32)
    return part


out = {"mode": mode}
out["dH = G @ W"] = timeit(lambda: G @ W)
out["dH = G @ Wt.t()"] = timeit(lambda: G @ Wt.t())
out["dW split-K 32 (bmm fp32 out)"] = timeit(lambda: splitk(32))
out["dW split-K 32 bf16 bmm + float sum"] = timeit(
    lambda: torch.bmm(G[:32 * (n // 32)].view(32, n // 32, -1).transpose(1, 2),
                      Hact[:32 * (n // 32)].view(32, n // 32, -1)).float().sum(0))
out["dW single mm"] = timeit(lambda: torch.mm(G.t(), Hact))
print(json.dumps(out), flush=True)
