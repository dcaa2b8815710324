"""Summarise one profiling round (tools/gpu_profile.sh) into committed files under profiles/.

  python tools/pmc_summary.py --stats DIR --fetch DIR --write DIR --bench JSON --tag rNN [--config headline]

Inputs (rocprofv3 CSV output directories, `-o run --output-format csv`):
  --stats : `--kernel-trace --stats` run of the bench command  -> run_kernel_stats.csv
  --fetch : `--pmc FETCH_SIZE` run                             -> run_counter_collection.csv
  --write : `--pmc WRITE_SIZE` run                             -> run_counter_collection.csv
  --bench : the bench JSON line of the --stats run (its HIP-event kernel averages are cross-checked)

Outputs:
  profiles/<tag>/kernel_stats_headline.csv  : the rocprofv3 stats summary as produced
  profiles/<tag>/pmc_per_launch.json        : FETCH_SIZE / WRITE_SIZE (KiB) per launch for every kernel
  profiles/pmc_grad_traffic.json            : HBM bytes per launch of the gradient kernel, corrected per
                                              MI355X_MICROARCH.md (gfx950 FETCH_SIZE counts 1/2 of a 16-B/lane
                                              streaming read: x2; WRITE_SIZE exact), read by bench.py
"""
import argparse
import csv
import json
import os
import sys
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """'void mrnnt::grad_kernel<mrnnt::IoF32, 4, 1, true, true>(mrnnt::DevProblem, ...)' -> 'grad_kernel<...>'"""
    n = name.split("(")[0].replace("void ", "").replace("mrnnt::", "")
    return n


def family(name):
    n = short(name)
    for fam in ("grad_staged_kernel", "grad_rows_kernel", "grad_kernel", "grad_scalar_kernel", "softmax_lean_kernel",
                "softmax_kernel", "softmax_scalar_kernel", "recursion_kernel", "setup_kernel",
                "synth_kernel", "pad_zero_kernel", "align_"):
        if n.startswith(fam):
            return fam
    return None


def counters(d, counter):
    per = defaultdict(list)
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def source_sha256():
    sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
    import _mrnnt_lib
    return _mrnnt_lib.source_sha256()


def lib_sha256():
    import hashlib
    h = hashlib.sha256()
    with open(os.path.join(ROOT, "monotonic-rnnt_amd", "libmonotonic_rnnt_amd.so"), "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--bench", required=True)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--config", default="headline")
    ap.add_argument("--dtype", default="f32", help="acts dtype of the profiled bench (f32 / bf16 / f16)")
    a = ap.parse_args()
    # the headline f32 run feeds bench.py's `traffic` (profiles/pmc_grad_traffic.json); other runs keep their own files
    main_run = a.config == "headline" and a.dtype == "f32"
    sfx = "" if main_run else f"_{a.config}_{a.dtype}"
    elem = {"f32": 4, "bf16": 2, "f16": 2}[a.dtype]
    out_dir = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(out_dir, exist_ok=True)
    shutil.copy(os.path.join(a.stats, "run_kernel_stats.csv"), os.path.join(out_dir, f"kernel_stats_{a.config}{'' if a.dtype == 'f32' else '_' + a.dtype}.csv"))
    bench = json.loads(open(a.bench).read().strip().splitlines()[-1])

    stats = {}
    with open(os.path.join(a.stats, "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) / 1e6}
    fetch = counters(a.fetch, "FETCH_SIZE")
    write = counters(a.write, "WRITE_SIZE")
    per = {}
    for name in sorted(set(fetch) | set(write)):
        if family(name) is None:
            continue
        fk = sum(fetch.get(name, [0])) / max(1, len(fetch.get(name, [0])))
        wk = sum(write.get(name, [0])) / max(1, len(write.get(name, [0])))
        per[short(name)] = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk, "launches": len(fetch.get(name, [])),
                            "hbm_bytes_corrected": fk * 1024 * 2 + wk * 1024,
                            "rocprof_avg_ms": next((v["avg_ms"] for k, v in stats.items() if short(k) == short(name)),
                                                   None)}
    json.dump({"units": "KiB per launch as reported by rocprofv3 (separate --pmc passes); "
                        "hbm_bytes_corrected = FETCH_SIZE*2 + WRITE_SIZE (gfx950 correction)",
               "kernels": per}, open(os.path.join(out_dir, f"pmc_per_launch{sfx}.json"), "w"), indent=1)

    grad = [k for k in per if family(k) in ("grad_staged_kernel", "grad_kernel", "grad_rows_kernel")]
    soft = [k for k in per if family(k) in ("softmax_lean_kernel", "softmax_kernel")]
    assert grad and soft, per.keys()
    g, s = per[grad[0]], per[soft[0]]
    alg = bench["roofline"]["algorithmic_bytes_per_launch"]
    res = {
        "config": a.config,
        "dtype": a.dtype,
        "kernel": grad[0],
        "hbm_bytes_per_launch": int(round(g["hbm_bytes_corrected"])),
        "read_bytes_corrected": int(round(g["FETCH_SIZE_KiB"] * 2048)),
        "write_bytes": int(round(g["WRITE_SIZE_KiB"] * 1024)),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round(g["hbm_bytes_corrected"] / alg, 4),
        "softmax_kernel": soft[0],
        "softmax_read_bytes_corrected": int(round(s["FETCH_SIZE_KiB"] * 2048)),
        "softmax_algorithmic_bytes": bench["config"]["inband_rows_per_gpu"] * bench["config"]["V"] * elem,
        "rocprof_avg_ms": {"grad": g["rocprof_avg_ms"], "log_softmax": s["rocprof_avg_ms"]},
        "bench_hip_event_avg_ms": {"grad": bench["kernels"]["grad"]["avg_ms"],
                                   "log_softmax": bench["kernels"]["log_softmax"]["avg_ms"]},
        "correction": "FETCH_SIZE(KiB)*1024*2 (gfx950 half-count of 16-B/lane streaming reads) + WRITE_SIZE(KiB)*1024",
        # what the counters were measured on: bench.py uses this record for a library built from these very sources
        # (source_sha256, path-independent build) or for this very binary (lib_sha256)
        "lib_sha256": lib_sha256(),
        "source_sha256": source_sha256(),
        "source": f"profiles/{a.tag}/pmc_per_launch{sfx}.json (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, "
                  f"python3 bench.py --config {a.config} --acts-dtype {a.dtype} --steps 3 --warmup 1 --no-cpu)",
    }
    out = os.path.join(ROOT, "profiles", "pmc_grad_traffic.json") if main_run else \
        os.path.join(out_dir, f"pmc_grad_traffic{sfx}.json")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
