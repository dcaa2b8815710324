import sys, os
sys.path[:0] = ["tests", "oracle", "monotonic-rnnt_amd/pytorch_binding"]
import numpy as np, torch
import test_gpu_joint as TJ
import monotonic_rnnt_joint as jop
dev = torch.device("cuda:0")
for H, V in [(128, 64), (256, 1000), (512, 256), (640, 130)]:
    enc, pred, w, bias, labels, T, S = TJ.make_case(H + V, 3, (1, 24), 8, H, V)
    c, de, dp, dw, db = TJ.run_joint(jop, dev, enc, pred, w, bias, labels, T, S)
    cr, de_r, dp_r, dw_r, db_r = TJ.host_reference(enc, pred, w, bias, labels, T, S)
    rel = lambda x, r: ((x.double().cpu() - r).abs().max() / r.abs().max()).item()
    print(H, V, "cost rel", np.max(np.abs(c - cr) / np.maximum(1, np.abs(cr))), "enc", rel(de, de_r), "pred", rel(dp, dp_r), "w", rel(dw, dw_r), "b", rel(db, db_r))
