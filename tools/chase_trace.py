"""Timeline of one chase launch (development build, g_chase_trace: s_memrealtime stamps per workgroup, 10 ns ticks):
configs[1] with device and host lengths -- recursion start / lengths resolved / first frame / walk done, producers
start / first slot / first flag / done, medians and maxima over the launch (us from the first stamp).

  python tools/chase_trace.py OUT.json"""
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
Th = torch.full((B,), T, dtype=torch.int32)
Sh = torch.full((B,), S, dtype=torch.int32)
out = {}
# (lengths form, chase_stage, chase_probe): the product's staged walk, the walk without ring reads after its first
# frames (probe 4: it no longer waits for frames) and with a max in place of the log-sum-exp (probe 2) -- the probes'
# results are wrong, timing only. (A 32-frame ring, measured in round 5: profiles/r05/chase/.)
for form, stage, probe in [("device", 1, 0), ("host", 1, 0), ("device", 1, 4), ("device", 1, 2)]:
    Tt, St = (Th, Sh) if form == "host" else (Th.to(dev), Sh.to(dev))
    with knobs(chase=1, chase_stage=stage, chase_probe=probe):
        lib = L.load_dev()
        res = []
        for it in range(6):
            a = acts.detach().clone().requires_grad_(True)
            c = op.monotonic_rnnt_loss(a, labels, Tt, St)
            c.sum().backward()
            torch.cuda.synchronize()
            buf = (ctypes.c_ulonglong * (4096 * 4))()
            n = lib.mrnnt_chase_trace(buf, 4096 * 4)
            tr = np.frombuffer(buf, dtype=np.uint64)[:n].reshape(-1, 4).astype(np.int64)
            if it < 2:
                continue
            nrec = 2 * B
            t0 = tr[:, 0][tr[:, 0] > 0].min()
            live = tr[:, 0] >= t0  # workgroups written this launch
            rel = (tr - t0) / 100.0  # us
            rec = rel[:nrec]
            prod = rel[nrec:][live[nrec:]]
            res.append({
                "rec_start_us": [float(np.median(rec[:, 0])), float(rec[:, 0].max())],
                "rec_resolved_us": [float(np.median(rec[:, 1])), float(rec[:, 1].max())],
                "rec_first_frame_us": [float(np.median(rec[:, 2])), float(rec[:, 2].max())] if stage else None,
                "rec_done_us": [float(np.median(rec[:, 3])), float(rec[:, 3].max())] if stage else None,
                "prod_n": int(len(prod)),
                "prod_start_us": [float(np.percentile(prod[:, 0], 50)), float(prod[:, 0].max())],
                "prod_first_slot_us": [float(np.percentile(prod[:, 1], 50)), float(prod[:, 1].max())],
                "prod_first_flag_us": [float(np.percentile(prod[:, 2], 50)), float(prod[:, 2].max())],
                "prod_done_us": [float(np.percentile(prod[:, 3], 50)), float(prod[:, 3].max())],
                "wg0_prod": [float(x) for x in rel[nrec]],
                "alpha0": [float(x) for x in rel[0]],
                "beta0": [float(x) for x in rel[1]],
            })
        out[f"{form}_stage{stage}_probe{probe}"] = res
        print(form, stage, probe, json.dumps(res[-1]), flush=True)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/chase_trace.json", "w"), indent=1)
