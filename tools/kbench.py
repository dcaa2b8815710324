"""In-process A/B of kernel launch variants (interleaved rounds, per-kernel HIP-event times).

  python tools/kbench.py [--config headline|c2|ragged] [--rounds R] [--variants JSON]

Each variant is a dict of mrnnt_tune knobs; every round runs forward(with beta) + backward once per
variant, in round-robin order, and records the per-kernel duration from HIP events around each launch.
Prints one JSON object with the median / min per kernel per variant and the achieved GB/s.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))
sys.path.insert(0, ROOT)

DEFAULT_VARIANTS = [
    {"softmax_grid_per_cu": 0, "grad_grid_per_cu": 32},
    {"softmax_grid_per_cu": 0, "grad_grid_per_cu": 24},
    {"softmax_grid_per_cu": 0, "grad_grid_per_cu": 48},
    {"softmax_grid_per_cu": 0, "grad_grid_per_cu": 64},
    {"softmax_grid_per_cu": 64, "grad_grid_per_cu": 32},
    {"softmax_grid_per_cu": 0, "grad_grid_per_cu": 32, "grad_variant": 1},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="headline")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default=None)
    ap.add_argument("--probe", action="store_true",
                    help="variants are timing probes that change the results (chase_probe, joint_probe): no cost check")
    ap.add_argument("--rank", default="0/1", help="r/N: time rank r's slice of an N-way sharded config")
    ap.add_argument("--fragment-gb", type=float, default=0.0,
                    help="before allocating, map this many GB as --fragment-mib pieces and free every other one, "
                         "so the big buffers are built from scattered physical memory (TLB / fragment-size study)")
    ap.add_argument("--fragment-mib", type=int, default=2)
    ap.add_argument("--buffers", type=int, default=1,
                    help="allocate this many acts and grads buffers (variant knobs acts_buf / grads_buf pick one): "
                         "does the gradient kernel's speed depend on where a buffer sits?")
    ap.add_argument("--acts-buffers", type=int, default=0,
                    help="allocate this many acts buffers but one grads buffer (variant knob acts_buf picks one): the "
                         "log-softmax read side over several physical placements in one process")
    ap.add_argument("--acts-dtype", default="f32", choices=["f32", "bf16", "f16"],
                    help="element type of acts / grads (the kernels' IoBF16 / IoF16 paths)")
    ap.add_argument("--ws-first", action="store_true",
                    help="allocate the workspace before grads (the order the autograd surface produces)")
    args = ap.parse_args()
    variants = json.loads(args.variants) if args.variants else DEFAULT_VARIANTS

    import _mrnnt_lib as L
    from bench import lengths_for

    lib = L.select_dev()  # launch knobs live in the development build
    # every knob any variant sets is restored to its default before each variant (a knob left set by the previous
    # variant would otherwise carry over into the next one, round after round)
    SPECIAL = ("grads_buf", "acts_buf", "grads_offset_kb")
    keys = {"softmax_variant", "grad_variant", "softmax_grid_per_cu", "grad_grid_per_cu", "nt_store", "nt_load",
            "occ_skip", "col_scatter", "col_xcd", "dp_halo"} | {k for v in variants for k in v if k not in SPECIAL}
    DEFAULTS = {k: L.tune(k) for k in sorted(keys)}
    bad = [k for k, v in DEFAULTS.items() if v < 0]
    if bad:  # a knob the development build does not know (e.g. a removed one) fails loudly, never silently skipped
        raise SystemExit(f"kbench: unknown knobs {bad}")
    dev = torch.device("cuda:0")
    keep = []
    if args.fragment_gb > 0:
        piece = args.fragment_mib << 20
        pieces = [torch.empty(piece, dtype=torch.uint8, device=dev) for _ in range(int(args.fragment_gb * 1e9 // piece))]
        keep = pieces[::2]
        del pieces
        torch.cuda.empty_cache()
    rk, wd = (int(x) for x in args.rank.split("/"))
    T, S, V, workload = lengths_for(args.config, rk, wd)[:4]
    B = len(T)
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    n_band = int(np.sum((S.astype(np.int64) + 1) * (T - S + 1) - 1))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
    L.synth_acts(acts.data_ptr(), 0, rows * V, 0, True, stream.value)
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[args.acts_dtype]
    elem = torch.empty(0, dtype=tdt).element_size()
    if tdt != torch.float32:
        acts = acts.to(tdt)
        torch.cuda.empty_cache()
    MAX_OFF_KB = 1 << 20  # grads may be shifted by up to 1 GiB (variant knob "grads_offset_kb")
    if not args.ws_first:
        grads_store = torch.empty(rows * V + MAX_OFF_KB * 256, dtype=tdt, device=dev)
    labels = torch.from_numpy(np.random.default_rng(1).integers(1, V, (B, int(S.max()))).astype(np.int32)).to(dev)
    T_dev = torch.from_numpy(T).to(dev)
    S_dev = torch.from_numpy(S).to(dev)
    costs = torch.empty(B, dtype=torch.float32, device=dev)
    p = L.MrnntProblem()
    p.B, p.V, p.blank, p.max_shift = B, V, 0, 0
    p.T_host, p.S_host = T.ctypes.data, S.ctypes.data
    p.T_dev, p.S_dev = T_dev.data_ptr(), S_dev.data_ptr()
    p.acts, p.labels, p.label_stride = acts.data_ptr(), labels.data_ptr(), labels.size(1)
    p.alignment, p.align_stride, p.align_blank, p.num_rows = None, 0, 0, rows
    p.acts_dtype = {"f32": L.MRNNT_F32, "bf16": L.MRNNT_BF16, "f16": L.MRNNT_F16}[args.acts_dtype]
    n = ctypes.c_size_t(0)
    L.check(lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)), "ws")
    ws = torch.empty(n.value, dtype=torch.uint8, device=dev)
    if args.ws_first:
        grads_store = torch.empty(rows * V + MAX_OFF_KB * 256, dtype=tdt, device=dev)
    grads_holder = {"t": grads_store[: rows * V].view(rows, V)}
    acts_list, grads_list = [acts], [grads_store]
    for _ in range(args.buffers - 1):
        acts_list.append(acts.clone())
        grads_list.append(torch.empty(rows * V, dtype=tdt, device=dev))
    for _ in range(max(0, args.acts_buffers - len(acts_list))):
        acts_list.append(acts.clone())
    out_alloc = {"acts": acts.data_ptr(), "grads": grads_store.data_ptr(), "ws": ws.data_ptr()}

    def run_once():
        L.check(lib.mrnnt_forward(ctypes.byref(p), ctypes.c_void_p(ws.data_ptr()), n.value,
                                  ctypes.c_void_p(costs.data_ptr()), 1, stream), "fwd")
        L.check(lib.mrnnt_backward(ctypes.byref(p), ctypes.c_void_p(ws.data_ptr()), None,
                                   ctypes.c_void_p(grads_holder["t"].data_ptr()), stream), "bwd")

    ref_costs = None
    times = [dict(log_softmax=[], alpha_beta=[], chase=[], grad=[]) for _ in variants]
    for r in range(args.rounds + 1):
        for i, v in enumerate(variants):
            for k, val in DEFAULTS.items():
                L.tune(k, val)
            gb_i, ab_i = int(v.get("grads_buf", 0)), int(v.get("acts_buf", 0))
            p.acts = acts_list[ab_i].data_ptr()
            for k, val in v.items():
                if k in ("grads_buf", "acts_buf"):
                    continue
                if k == "grads_offset_kb":
                    o = int(val) * 256
                    grads_holder["t"] = grads_store[o: o + rows * V].view(rows, V)
                    continue
                if L.tune(k, val) < 0:
                    raise SystemExit(f"kbench: unknown knob {k}")
            if "grads_offset_kb" not in v:
                grads_holder["t"] = grads_list[gb_i][: rows * V].view(rows, V)
            L.profile_enable(True)
            run_once()
            prof = L.profile_read()
            L.profile_enable(False)
            c = costs.cpu().numpy()
            if ref_costs is None:
                ref_costs = c
            if not args.probe and not np.allclose(c, ref_costs, rtol=1e-6):
                raise SystemExit(f"kbench: variant {v} changed the costs")
            if r == 0:
                continue  # warm-up round
            for k in times[i]:
                times[i][k].append(prof[k][0])
    out_alloc["acts_bufs"] = [t.data_ptr() for t in acts_list]
    out_alloc["grads_bufs"] = [t.data_ptr() for t in grads_list]
    out = {"alloc": out_alloc, "fragment": {"gb": args.fragment_gb, "mib": args.fragment_mib, "held": len(keep)}, "workload": workload, "acts_dtype": args.acts_dtype, "rows": rows, "inband_rows": n_band, "V": V, "variants": []}
    gb = (n_band + rows) * V * elem / 1e9
    sb = n_band * V * elem / 1e9
    for v, t in zip(variants, times):
        med = {k: float(np.median(x)) for k, x in t.items()}
        out["variants"].append({"knobs": v, "median_ms": med, "min_ms": {k: float(np.min(x)) for k, x in t.items()},
                                "grad_gbps": round(gb / (med["grad"] * 1e-3), 1),
                                "softmax_gbps": round(sb / (med["log_softmax"] * 1e-3), 1) if med["log_softmax"] else None,
                                "step_ms": round(sum(med.values()), 3)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
