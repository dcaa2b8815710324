"""Where do the chase launch's alpha / beta differ from the two-kernel path's? (development build; configs[1] shape)
Prints, per array, the number of differing cells and the first few (utterance, t, s, values)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _mrnnt_lib as L  # noqa: E402

L.select_dev()
import monotonic_rnnt_op as op  # noqa: E402
from _parity import random_problem  # noqa: E402

dev = torch.device("cuda:0")
rng = np.random.default_rng(1)
B, T_, S_ = 16, 200, 40
acts, labels, T, S = random_problem(rng, B, (T_, T_), S_, 256, force={b: (T_, S_) for b in range(B)})
a = torch.from_numpy(acts).to(dev)
lab = torch.from_numpy(labels).to(dev)


def state(chase, stage):
    L.tune("chase", chase)
    L.tune("chase_stage", stage)
    prep = op._Prepared(a, lab, torch.from_numpy(T), torch.from_numpy(S), None, 0, 0)
    _, ws = op._forward(prep, with_beta=True)
    n = acts.shape[0]
    den = torch.zeros(n, dtype=torch.float32, device=dev)
    al = torch.zeros(n, dtype=torch.float64, device=dev)
    be = torch.zeros(n, dtype=torch.float64, device=dev)
    L.check(L.load().mrnnt_read_state(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                      ctypes.c_void_p(den.data_ptr()), ctypes.c_void_p(al.data_ptr()),
                                      ctypes.c_void_p(be.data_ptr()), prep.stream()), "read_state")
    torch.cuda.synchronize()
    return den.cpu().numpy(), al.cpu().numpy(), be.cpu().numpy()


ref = state(0, 1)
for stage in (1, 0):
    got = state(1, stage)
    print(f"chase stage={stage}")
    for name, x, y in zip(("den", "alpha", "beta"), got, ref):
        bad = np.flatnonzero(~((x == y) | (np.isnan(x) & np.isnan(y))))
        print(f"  {name}: {bad.size} differing cells")
        for i in bad[:8]:
            b, r = divmod(int(i), T_ * (S_ + 1))
            t, s = divmod(r, S_ + 1)
            print(f"    b={b} t={t} s={s}: chase {x[i]!r} two-kernel {y[i]!r}")
