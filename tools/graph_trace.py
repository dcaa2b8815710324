#!/usr/bin/env python3
"""Kernel timeline of a profiled bench run (rocprofv3 --kernel-trace --output-format csv): per kernel the average
in-trace duration, and per step of the hot path (a log-softmax launch up to the next one) the span, the busy time
and the idle gaps between its kernels -- how a HIP-graph replay's step divides between kernels and launch gaps.

  python tools/graph_trace.py <dir with *kernel_trace.csv> [--last N]
"""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    n = name.split("(")[0]
    for k in ("chase", "softmax", "recursion", "grad", "setup", "reduce_kernel", "Fill", "fill", "elementwise"):
        if k in n:
            return k + ("" if k not in ("softmax", "grad", "recursion") else ":" + n.split("<")[0].split("::")[-1])
    return n[-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=200, help="steps at the end of the trace to summarise")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    steps, cur = [], []
    for r in rows:
        first = r[2].startswith("softmax") or r[2].startswith("chase")  # the forward's first kernel of the path
        if first and cur:
            steps.append(cur)
            cur = []
        if first or cur:
            cur.append(r)
    if cur:
        steps.append(cur)
    steps = [s for s in steps if any(k[2].startswith("grad") for k in s)][-a.last:]
    dur = collections.defaultdict(list)
    spans, busy, gaps = [], [], collections.defaultdict(list)
    for s in steps:
        spans.append((s[-1][1] - s[0][0]) / 1e3)
        busy.append(sum(e - b for b, e, _ in s) / 1e3)
        for (b0, e0, n0), (b1, e1, n1) in zip(s, s[1:]):
            gaps[f"{n0} -> {n1}"].append((b1 - e0) / 1e3)
        for b, e, n in s:
            dur[n].append((e - b) / 1e3)
    period = [(b[0][0] - a[0][0]) / 1e3 for a, b in zip(steps, steps[1:])]  # start to start: the whole step
    out = {"trace": path, "steps": len(steps),
           "step_period_us": round(sum(period) / len(period), 2) if period else None,
           "step_span_us": round(sum(spans) / len(spans), 2), "step_busy_us": round(sum(busy) / len(busy), 2),
           "kernel_us": {k: round(sum(v) / len(v), 2) for k, v in dur.items()},
           "gap_us": {k: round(sum(v) / len(v), 2) for k, v in gaps.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
