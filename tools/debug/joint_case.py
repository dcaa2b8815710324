"""Describe tests/test_gpu_joint.py random cases on the host (no GPU): python tools/debug/joint_case.py SEED...

Prints the case parameters and, from the fp64 host reference, the size of d_bias against the column sums of
|dz| it cancels from (the bf16 storage of the logit gradient G bounds d_bias's error by ~2^-9 of the latter).
"""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
spec = importlib.util.spec_from_file_location("tj", os.path.join(ROOT, "tests", "test_gpu_joint.py"))
tj = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tj)
import oracle as O  # noqa: E402
import torch  # noqa: E402

for sd in map(int, sys.argv[1:]):
    enc, pred, w, bias, labels, T, S, blank, scale, al, k = tj.random_joint_case(sd)
    V, H = w.shape
    print(sd, "H", H, "V", V, "T", T.tolist(), "S", S.tolist(), "blank", blank, "scale", scale, "align", al is not None,
          "k", k, "bias", bias is not None)
    if bias is None:
        continue
    B = len(T)
    W64 = w.double()
    rows = []
    for b in range(B):
        h = torch.tanh(enc[b, : T[b]].float()[:, None, :] + pred[b, : S[b] + 1].float()[None]).to(torch.bfloat16)
        rows.append((h.double() @ W64.T + bias.double()).reshape(-1, V))
    acts = torch.cat(rows).float().numpy()
    _, dz = O.oracle_rnnt(acts, labels, T, S, blank=blank, alignment=al, max_shift=k, num_threads=4)
    dz = dz * np.repeat(np.asarray(scale, np.float64), T * (S + 1))[:, None]
    db = dz.sum(0)
    print("   max|db| %.3e   max_v sum_rows|dz| %.3e   ratio %.3e" % (np.abs(db).max(), np.abs(dz).sum(0).max(),
                                                                     np.abs(db).max() / np.abs(dz).sum(0).max()))
