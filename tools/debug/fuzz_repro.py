"""Re-run tests/test_gpu_fuzz.py cases in a given order and print per-utterance costs vs the oracle (debugging aid).

    python tools/debug/fuzz_repro.py 133            # one case in a fresh process
    python tools/debug/fuzz_repro.py 132,133        # a sequence (state carried between calls?)
    python tools/debug/fuzz_repro.py 133 dp_halo=0  # with launch knobs
"""
import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
spec = importlib.util.spec_from_file_location("fz", os.path.join(ROOT, "tests", "test_gpu_fuzz.py"))
fz = importlib.util.module_from_spec(spec)
spec.loader.exec_module(fz)

import oracle as O  # noqa: E402
import monotonic_rnnt_op as op  # noqa: E402
import _mrnnt_lib as L  # noqa: E402

seeds = [int(s) for s in sys.argv[1].split(",")]
if sys.argv[2:]:
    L.select_dev()  # launch knobs live in the development build
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    assert L.tune(k, int(v)) >= 0, k
dev = torch.device("cuda:0")
for sd in seeds:
    c = fz.make_case(sd)
    T, S = c["T"], c["S"]
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[c["dtype"]]
    a = torch.from_numpy(c["acts"]).to(tdt)
    host = a.float().numpy()
    if c["padded"]:
        a = torch.from_numpy(fz.pad(host, T, S, int(T.max()) + 2, int(S.max()) + 3)).to(tdt)
    a = a.to(dev)
    lab = torch.from_numpy(c["labels"]).to(dev)
    al = None if c["align"] is None else torch.from_numpy(c["align"]).to(dev)
    for rep in range(2):
        costs = op.monotonic_rnnt_loss(a, lab, torch.from_numpy(T), torch.from_numpy(S), al, c["k"], c["blank"])
        torch.cuda.synchronize()
        print("seed", sd, "rep", rep, "gpu", costs.float().cpu().numpy().tolist(), flush=True)
    cr, _ = O.oracle_rnnt(host, c["labels"], T, S, blank=c["blank"], alignment=c["align"], max_shift=c["k"],
                          num_threads=8)
    print("seed", sd, "oracle", cr.tolist(), flush=True)
