"""Timeline of the fused joint's d_enc / d_pred reduce (joint_reduce_kernel; development build, joint_probe bit 4:
g_reduce_trace, s_memrealtime stamps of thread 0, 10 ns ticks) at the joint bench's H = 512 shape (B 64, T 1000,
S 200, V 1024, joint_bench.py's synthetic inputs). Splits each traced workgroup's life into setup (label range + the
accumulator clear), per-frame row sums (loads of dH / Hact rows and the LDS accumulation), per-frame barriers (the
two barriers around the d_enc sum of the frame) and the flush of its d_pred partials; prints medians over the
workgroups and the launch's span.

  python tools/reduce_trace.py OUT.json"""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "monotonic-rnnt_amd/pytorch_binding")
import _mrnnt_lib as L  # noqa: E402
import monotonic_rnnt_joint as J  # noqa: E402
from _parity import knobs  # noqa: E402

B, T, S, V, H = 64, 1000, 200, 1024, 512
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
enc = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
pred = torch.randn(B, S + 1, H, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
W = (torch.randn(V, H, device=dev, generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16).requires_grad_(True)
bias = (0.1 * torch.randn(V, device=dev, generator=g)).requires_grad_(True)
labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, S)).astype(np.int32)).to(dev)
Tl = torch.full((B,), T, dtype=torch.int32)
Sl = torch.full((B,), S, dtype=torch.int32)
NW = 8192
out = {"workload": f"joint H={H}: B={B} T={T} S={S} V={V}", "runs": []}
with knobs(joint_probe=16):
    lib = L.load_dev()
    for it in range(4):
        for x in (enc, pred, W, bias):
            x.grad = None
        L.profile_enable(True)
        J.monotonic_rnnt_joint_loss(enc, pred, W, bias, labels, Tl, Sl).sum().backward()
        torch.cuda.synchronize()
        prof = L.profile_read()
        L.profile_enable(False)
        buf = (ctypes.c_ulonglong * (NW * 16))()
        n = lib.mrnnt_joint_reduce_trace(buf, NW * 16)
        tr = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(-1, 16).astype(np.int64)
        if it < 1:
            continue
        live = (tr[:, 0] > 0) & (tr[:, 15] >= tr[:, 0])
        t0 = tr[live, 0].min()
        w = (tr[live] - t0) / 100.0  # us
        setup = w[:, 1] - w[:, 0]
        rows = np.stack([w[:, 2 + 2 * f] - (w[:, 1] if f == 0 else w[:, 1 + 2 * f]) for f in range(6)], 1)
        sync = np.stack([w[:, 3 + 2 * f] - w[:, 2 + 2 * f] for f in range(6)], 1)
        loop = w[:, 14] - w[:, 1]
        flush = w[:, 15] - w[:, 14]
        life = w[:, 15] - w[:, 0]
        run = {
            "reduce_ms_hip_events": prof["joint_reduce"][0],
            "traced_workgroups": int(live.sum()),
            "span_us": float(w[:, 15].max()),
            "median_us": {"life": float(np.median(life)), "setup": float(np.median(setup)),
                          "frame_loop": float(np.median(loop)), "flush": float(np.median(flush)),
                          "rows_per_frame_f0_5": [float(x) for x in np.median(rows, 0)],
                          "barriers_per_frame_f0_5": [float(x) for x in np.median(sync, 0)]},
            "share_of_life": {"setup": float(np.median(setup / life)), "frame_rows": float(np.median(rows.sum(1) / life)),
                              "frame_barriers": float(np.median(sync.sum(1) / life)),
                              "frames_6_on": float(np.median((w[:, 14] - w[:, 13]) / life)),
                              "flush": float(np.median(flush / life))},
        }
        out["runs"].append(run)
        print(json.dumps(run), flush=True)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/reduce_trace.json", "w"), indent=1)
