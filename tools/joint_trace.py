"""Timeline of the fused joint forward (development build, g_joint_trace): waves 0 and 4 of the first 4096
workgroups at H = 512 (tools/joint_bench.py's problem). Only the forward kernel stamps (the chunk-0 marks included:
the backward kernels share the chunk loop but not its TRACE flag), so a read after a training step still shows the
last forward alone. Run twice: as the product computes, and with the development probe joint_probe = 1 (every row's
pred load on row 0 -- results wrong, timing only), to show what the activation build's pred loads cost."""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "monotonic-rnnt_amd/pytorch_binding")
import _mrnnt_lib as L  # noqa: E402

L.select_dev()
import monotonic_rnnt_joint as J  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
B, T, S, V, H = 64, 1000, 200, 1024, 512
enc = torch.randn(B, T, H, device=dev, generator=g).to(torch.bfloat16)
pred = torch.randn(B, S + 1, H, device=dev, generator=g).to(torch.bfloat16)
W = (torch.randn(V, H, device=dev, generator=g) * (2.0 / H ** 0.5)).to(torch.bfloat16)
bias = (0.1 * torch.randn(V, device=dev, generator=g))
labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, S)).astype(np.int32)).to(dev)
Tl = torch.full((B,), T, dtype=torch.int32)
Sl = torch.full((B,), S, dtype=torch.int32)
lib = L.load_dev()
L.tune("joint_trace", 1)  # the forward instantiation with the stamps (the default one has none)
out = {}
for probe in (0, 1):
    L.tune("joint_probe", probe)
    out[f"joint_probe={probe}"] = []
    for it in range(3):
        with torch.no_grad():
            J.monotonic_rnnt_joint_loss(enc, pred, W, bias, labels, Tl, Sl)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4096 * 64))()
        n = lib.mrnnt_joint_trace(buf, 4096 * 64)
        tr = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(-1, 8, 8).astype(np.int64)
        t0 = tr[:, :, 0].min(axis=1, keepdims=True)
        rel = (tr - t0[:, :, None]) / 100.0  # us since the workgroup's first wave started
        build_end = rel[:, :, 2]
        res = {
            "tile_us_median": float(np.median(rel[:, :, 4].max(axis=1))),
            "build_us_median": float(np.median(rel[:, :, 2] - rel[:, :, 1])),
            "build_end_first_us": float(np.median(build_end.min(axis=1))),
            "build_end_last_us": float(np.median(build_end.max(axis=1))),
            "build_skew_us": float(np.median(build_end.max(axis=1) - build_end.min(axis=1))),
            "first_chunk_done_after_last_build_us": float(np.median(rel[:, :, 3].min(axis=1) - build_end.max(axis=1))),
            "rest_chunks_us": float(np.median(rel[:, :, 4] - rel[:, :, 3])),
            "wave_start_spread_us": float(np.median(rel[:, :, 0].max(axis=1))),
            "chunk0_wait_us": float(np.median(rel[:, :, 5] - rel[:, :, 2])),
            "chunk0_barrier_us": float(np.median(rel[:, :, 6] - rel[:, :, 5])),
            "chunk0_mma_us": float(np.median(rel[:, :, 7] - rel[:, :, 6])),
            "chunk0_epilogue_us": float(np.median(rel[:, :, 3] - rel[:, :, 7])),
        }
        out[f"joint_probe={probe}"].append(res)
        print(probe, json.dumps(res), flush=True)
L.tune("joint_probe", 0)
L.tune("joint_trace", 0)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/joint_trace.json", "w"), indent=1)
