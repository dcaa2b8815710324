"""Print the parameters of tests/test_gpu_fuzz.py cases (debugging aid): python tools/debug/fuzz_case.py SEED..."""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
spec = importlib.util.spec_from_file_location("fz", os.path.join(ROOT, "tests", "test_gpu_fuzz.py"))
fz = importlib.util.module_from_spec(spec)
spec.loader.exec_module(fz)

for sd in map(int, sys.argv[1:]):
    c = fz.make_case(sd)
    print(sd, "V", c["V"], "T", c["T"].tolist(), "S", c["S"].tolist(), c["dtype"], "padded", c["padded"],
          "align", c["align"] is not None, "k", c["k"], "blank", c["blank"], "scale", c["scale"].tolist())
    for b in range(len(c["T"])):
        lab = c["labels"][b, : c["S"][b]]
        print("   utt", b, "labels==blank at", np.nonzero(lab == c["blank"])[0].tolist())
