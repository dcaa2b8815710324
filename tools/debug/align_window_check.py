"""Debug: alignment-restricted GPU gradients vs the oracle, rows with nonzero gradient outside the window."""
import sys, os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O
import monotonic_rnnt_op as op
import _mrnnt_lib as L

L.select_dev()  # the dp_halo knob lives in the development build
dev = torch.device("cuda:0")
for (B, T, S, V, k) in [(2, 50, 10, 16, 2), (2, 200, 40, 64, 2), (2, 1000, 200, 64, 2), (1, 1000, 200, 1024, 2)]:
    rng = np.random.default_rng(0)
    rows_per = T * (S + 1)
    acts = rng.standard_normal((B * rows_per, V)).astype(np.float32)
    labels = rng.integers(1, V, (B, S)).astype(np.int32)
    al = np.zeros((B, T), np.int32)
    frames = ((np.arange(S) + 0.5) * T / S).astype(np.int64)
    al[:, frames] = labels
    for dv in (2, 0):
        L.tune("dp_halo", dv)
        a = torch.from_numpy(acts).to(dev).requires_grad_(True)
        c = op.monotonic_rnnt_loss(a, torch.from_numpy(labels).to(dev), torch.full((B,), T, dtype=torch.int32),
                                   torch.full((B,), S, dtype=torch.int32), torch.from_numpy(al).to(dev), k, 0)
        c.sum().backward()
        g = a.grad.cpu().numpy()
        cr, gr = O.oracle_rnnt(acts, labels, [T] * B, [S] * B, alignment=al, max_shift=k, num_threads=4)
        m = np.concatenate([[0], np.cumsum(al[0] != 0)])
        t = np.arange(T)
        mn, mx = m[np.clip(t + 1 - k, 0, T)], m[np.clip(t + 1 + k, 0, T)]
        wlo = np.minimum(mn - 1, np.concatenate([[0], mn[:-1]]))
        whi = np.maximum(mx, np.concatenate([[0], mx[:-1]]))
        s = np.arange(S + 1)
        outside = ((s[None, :] < wlo[:, None]) | (s[None, :] > whi[:, None])).reshape(-1)
        gm = np.abs(g).max(1).reshape(B, rows_per)
        bad = np.argwhere(gm[:, outside] > 0)
        err = np.abs(g - gr).max()
        print(f"B={B} T={T} S={S} V={V} dp_halo={dv}: costs {c.detach().cpu().numpy()} ref {cr} grad err {err:.3e} "
              f"outside-nonzero {len(bad)}", flush=True)
        if len(bad):
            idx = np.nonzero(outside)[0][bad[:5, 1]]
            for b_, r in zip(bad[:5, 0], idx):
                tt, ss = divmod(int(r), S + 1)
                print("   b", b_, "t", tt, "s", ss, "band t", mn[tt], mx[tt], "band t-1", mn[tt - 1], mx[tt - 1],
                      "win", wlo[tt], whi[tt], "g", gm[b_, r], "ref", np.abs(gr[b_ * rows_per + r]).max())
L.tune("dp_halo", 2)
