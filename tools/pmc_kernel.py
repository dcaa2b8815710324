"""Average rocprofv3 --pmc counter values per kernel (name substring filter) from run_counter_collection.csv files.

  python tools/pmc_kernel.py DIR [DIR ...] --match joint_fwd
"""
import argparse
import csv
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--match", action="append", default=[])
a = ap.parse_args()
vals = defaultdict(lambda: defaultdict(list))
for d in a.dirs:
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for row in csv.DictReader(open(os.path.join(root, f))):
                    name = row["Kernel_Name"]
                    if a.match and not any(m in name for m in a.match):
                        continue
                    key = name.split("(")[0].replace("void ", "")[:70]
                    vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v) / len(v):18.4g}   (n={len(v)})")
