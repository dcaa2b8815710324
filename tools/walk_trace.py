"""Walk progress inside one chase launch (development build, chase_probe bit 8: s_memrealtime stamps, 10 ns ticks):
configs[1], device lengths. Per recursion workgroup, when the walk wave finished walk positions [0, 8 (i + 1)) and when
its loader wave published `loaded` >= 8 i; with the launch timeline of tools/chase_trace.py (producers done). Prints
medians over the alpha and beta workgroups (us from the launch's first stamp).

  python tools/walk_trace.py OUT.json [knob=value ...]   (chase_probe bits are or-ed with 8)"""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "monotonic-rnnt_amd/pytorch_binding")
import _mrnnt_lib as L  # noqa: E402
import monotonic_rnnt_op as op  # noqa: E402
from _parity import knobs  # noqa: E402

dev = torch.device("cuda:0")
B, T, S, V = 16, 200, 40, 256
g = torch.Generator(device=dev).manual_seed(0)
acts = torch.randn(B * T * (S + 1), V, device=dev, generator=g)
labels = torch.randint(1, V, (B, S), device=dev, dtype=torch.int32, generator=g)
Tt = torch.full((B,), T, dtype=torch.int32, device=dev)
St = torch.full((B,), S, dtype=torch.int32, device=dev)
kn = {k: int(v) for k, v in (a.split("=") for a in sys.argv[2:])}
kn["chase_probe"] = kn.get("chase_probe", 0) | 8
out = {"workload": "configs[1] B=16 T=200 S=40 V=256, device lengths", "knobs": kn, "runs": []}
nb = T // 8
with knobs(chase=1, chase_stage=1, **kn):
    lib = L.load_dev()
    for it in range(8):
        a = acts.detach().clone().requires_grad_(True)
        c = op.monotonic_rnnt_loss(a, labels, Tt, St)
        c.sum().backward()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4096 * 4))()
        n = lib.mrnnt_chase_trace(buf, 4096 * 4)
        tr = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(-1, 4).astype(np.int64)
        wbuf = (ctypes.c_ulonglong * (128 * 64))()
        m = lib.mrnnt_chase_walk_trace(wbuf, 128 * 64)
        wt = np.frombuffer(wbuf, dtype=np.uint64)[:m].reshape(-1, 64).astype(np.int64)
        if it < 3:
            continue
        nrec = 2 * B
        t0 = tr[:, 0][tr[:, 0] > 0].min()
        live = tr[:, 0] >= t0
        rel = (tr - t0) / 100.0
        prod = rel[nrec:][live[nrec:]]
        w = (wt[:nrec] - t0) / 100.0
        run = {"prod_done_us": [float(np.median(prod[:, 3])), float(prod[:, 3].max())],
               "rec_first_frame_us": float(np.median(rel[:nrec, 2])),
               "rec_done_us": [float(np.median(rel[:nrec, 3])), float(rel[:nrec, 3].max())]}
        for name, sel in (("alpha", slice(0, nrec, 2)), ("beta", slice(1, nrec, 2))):
            run[name + "_walk_us"] = [round(float(x), 2) for x in np.median(w[sel, :nb], axis=0)]
            run[name + "_loaded_us"] = [round(float(x), 2) for x in np.median(w[sel, 32:32 + nb + 1], axis=0)]
        out["runs"].append(run)
        print(json.dumps({k: v for k, v in run.items() if not k.endswith("_us") or len(str(v)) < 40}), flush=True)
r = out["runs"][-1]
print("alpha walk (every 8 frames):", r["alpha_walk_us"])
print("alpha loaded >= 8i:", r["alpha_loaded_us"])
print("beta walk:", r["beta_walk_us"])
print("beta loaded:", r["beta_loaded_us"])
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/walk_trace.json", "w"), indent=1)
