"""bench.py -- MI355X monotonic RNN-T loss+grad throughput (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config headline|c2|ragged]

One step = forward (log-softmax row reduce + alpha/beta DP) + backward (logit gradient, dL/dcost fused)
over one batch through the autograd surface (monotonic_rnnt_loss(...).sum().backward()), plus, for N > 1,
the single RCCL all-reduce of the summed loss. Inputs are synthetic and resident in HBM before timing.
Scaling is weak: every rank owns its own B utterances (batch sharding, no data-path collective).

Rank 0 prints ONE JSON line with the contract fields plus:
  roofline     : the gradient kernel (dominant), algorithmic bytes (N_live + N) * V * 4 per launch (N_live = in-band
                 rows whose fp32 gradient is not exactly zero, the rows it reads) divided by its average duration
                 from HIP events recorded around each launch on its stream in the timed region; the SURVEY §8d
                 formula (N_v + N) * V * 4 is reported beside it as formula_bytes_per_launch / formula_gbps
  cpu_baseline : the reference's own CpuRNNTComputer<float> (oracle/_ref) -- or the oracle port when the reference
                 build is absent -- timed on a bounded sample of the same workload on the host cores
  kernels      : per-kernel average ms and achieved GB/s
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))

METRIC = "utterances/sec + achieved HBM GB/s, (B,T,S,V)=(64,1000,200,1024)"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def lengths_for(config, rank, world):
    """Per-rank utterance lengths (weak scaling: each rank owns its own B utterances)."""
    if config == "headline":  # BASELINE.json configs[2]
        B, T, S, V = 64, 1000, 200, 1024
        return np.full(B, T, np.int32), np.full(B, S, np.int32), V, "B=64,T=1000,S=200,V=1024 (configs[2], headline)"
    if config == "c2":  # configs[1]
        B, T, S, V = 16, 200, 40, 256
        return np.full(B, T, np.int32), np.full(B, S, np.int32), V, "B=16,T=200,S=40,V=256 (configs[1])"
    if config == "c5":  # configs[4]: V = 10000; 64 utterances = 514.6 GB of acts > 288 GB, so the batch runs as
        # four 16-utterance chunks (128.6 GB acts + 128.6 GB grads each); one chunk is the measured unit
        B, T, S, V = 16, 1000, 200, 10000
        return (np.full(B, T, np.int32), np.full(B, S, np.int32), V,
                "B=16 chunk of B=64,T=1000,S=200,V=10000 (configs[4], large vocab; batch = 4 chunks)")
    if config == "ragged64":  # the first 64 utterances of configs[3] (fits one GPU with separate grads)
        rng = np.random.default_rng(0)
        Tg = rng.integers(200, 1601, 512).astype(np.int32)
        Sg = np.array([rng.integers(20, min(300, t) + 1) for t in Tg], np.int32)
        return Tg[:64], Sg[:64], 1024, "first 64 utterances of configs[3] (ragged T, S), V=1024"
    if config == "ragged":  # configs[3]: B=512 global, T~U[200,1600], S~U[20,min(300,T)], sharded over ranks
        rng = np.random.default_rng(0)
        Tg = rng.integers(200, 1601, 512).astype(np.int32)
        Sg = np.array([rng.integers(20, min(300, t) + 1) for t in Tg], np.int32)
        from distributed import shard_bounds
        lo, hi = shard_bounds(Tg.astype(np.int64) * (Sg + 1), world)[rank]
        return Tg[lo:hi], Sg[lo:hi], 1024, f"B=512 ragged (T~U[200,1600], S~U[20,min(300,T)]), V=1024, rank slice [{lo},{hi})"
    raise SystemExit(f"unknown config {config}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="headline", choices=["headline", "c2", "ragged", "ragged64", "c5"])
    ap.add_argument("--cpu-sample", type=int, default=20, help="utterances in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="OpenMP threads of the CPU baseline (the GPU box's CPU share per GPU is 16)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--acts-dtype", default="f32", choices=["f32", "bf16", "f16"],
                    help="element type of acts/grads (extension; the headline metric is f32, the reference's type)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="launch knob for experiments (mrnnt_tune); the defaults are the tuned values")
    ap.add_argument("--align-k", type=int, default=None,
                    help="alignment-restricted loss (restrict_to_alignment, max_distance_from_alignment = K) on a "
                         "synthetic alignment with the labels evenly spaced over the frames")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, the real path) or gloo (rehearsal: several ranks may share one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def coll_tensor(x):  # gloo collectives run on host tensors
        return x.cpu() if gloo else x

    import monotonic_rnnt_op as op
    import _mrnnt_lib as L

    lib = L.load()
    for kv in args.tune:
        k, v = kv.split("=")
        if L.tune(k, int(v)) < 0:
            raise SystemExit(f"unknown knob {k}")
    T, S, V, workload = lengths_for(args.config, rank, world)
    B = len(T)
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    n_band = int(np.sum((S.astype(np.int64) + 1) * (T - S + 1) - 1))  # in-band rows N_v
    # global row offset of this rank's first utterance, so every rank streams different synthetic data
    all_rows = [rows]
    if world > 1:
        t = coll_tensor(torch.tensor([rows], dtype=torch.int64, device=dev))
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        all_rows = [int(x.item()) for x in g]
    row0 = sum(all_rows[:rank])

    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    acts = torch.empty((rows, V), dtype=torch.float32, device=dev)
    L.check(lib.mrnnt_synth_acts(ctypes.c_void_p(acts.data_ptr()), row0 * V, rows * V, 0, 1, stream), "synth")
    elem = {"f32": 4, "bf16": 2, "f16": 2}[args.acts_dtype]
    if args.acts_dtype != "f32":
        acts = acts.to(torch.bfloat16 if args.acts_dtype == "bf16" else torch.float16)
        torch.cuda.empty_cache()
    rng = np.random.default_rng(1 + rank)
    labels = torch.from_numpy(rng.integers(1, V, (B, max(1, int(S.max())))).astype(np.int32)).to(dev)
    T_t = torch.from_numpy(T)
    S_t = torch.from_numpy(S)
    align, n_window = None, None
    if args.align_k is not None:
        al_np, n_window = synthetic_alignment(labels.cpu().numpy(), T, S, args.align_k)
        align = torch.from_numpy(al_np).to(dev)
        workload += f", alignment-restricted (k={args.align_k}, labels evenly spaced)"
    acts.requires_grad_(True)
    torch.cuda.synchronize()

    def step():
        acts.grad = None
        costs = op.monotonic_rnnt_loss(acts, labels, T_t, S_t, align, args.align_k or 0, blank_label=0)
        loss = costs.sum()
        loss.backward()
        if world > 1:
            tot = coll_tensor(loss.detach().clone())
            dist.all_reduce(tot)  # the one RCCL exchange of the path: 4 bytes over xGMI
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    L.profile_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = L.profile_read()
    L.profile_enable(False)
    el = coll_tensor(torch.tensor([elapsed], dtype=torch.float64, device=dev))
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    total_utts = coll_tensor(torch.tensor([B], dtype=torch.int64, device=dev))
    if world > 1:
        dist.all_reduce(total_utts)
    total_utts = int(total_utts.item())

    # live rows: in-band rows whose gradient is not exactly zero in fp32 -- the only acts rows the gradient
    # kernel reads (occupancy skip); counted once after the timed region
    live = live_rows(op, L, acts, labels, T_t, S_t, dev, align, args.align_k or 0)
    grad_bytes = (live + rows) * V * elem  # algorithmic: read live acts rows once, write every grads row once
    formula_grad_bytes = (n_band + rows) * V * elem  # SURVEY.md §8d formula: every in-band row read
    n_read = n_band if n_window is None else n_window  # rows the log-softmax pass reads
    softmax_bytes = n_read * V * elem
    step_bytes = (n_read + live + rows) * V * elem

    def avg_ms(name):
        ms, n = prof[name]
        return ms / n if n else None

    g_ms = avg_ms("grad")
    s_ms = avg_ms("log_softmax")
    d_ms = avg_ms("alpha_beta")
    achieved = grad_bytes / (g_ms * 1e-3) / 1e9 if g_ms else None

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_grad_traffic.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            # only a measurement of this config and of the kernel this run launches counts
            gv = L.tune("grad_variant")
            fam = {3: "grad_rows_kernel", 5: "grad_staged_kernel", 6: "grad_staged_kernel"}.get(gv, "grad_kernel")
            elem = {"f32": "IoF32", "bf16": "IoBF16", "f16": "IoF16"}[args.acts_dtype]
            if pm.get("config") == args.config and pm.get("kernel", "").startswith(f"{fam}<{elem}"):
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    copy_gbps = same_buffers_copy_gbps(lib, L, dev, acts.detach(), acts.grad)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0 and args.acts_dtype == "f32":
        cpu = cpu_baseline(lib, L, acts, labels, T, S, V, args.cpu_sample, stream, args.cpu_threads)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(total_utts * args.steps / elapsed, 3),
            "unit": "utt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.acts_dtype,
            "data": "synthetic: counter-hash N(0,1)-like acts (seed 0), labels U[1,V-1] (seed 1+rank); inputs resident in HBM",
            "config": {"workload": workload, "utterances_per_gpu": B, "global_batch": total_utts,
                       "rows_per_gpu": rows, "inband_rows_per_gpu": n_band, "V": V,
                       **({"window_rows_per_gpu": n_window} if n_window is not None else {}),
                       "parallelism": f"dp{world} (batch-sharded, one 4-byte "
                                      f"{'gloo (rehearsal)' if gloo else 'RCCL'} loss all-reduce)"},
            "achieved_hbm_gbps_step": round(step_bytes * total_utts / B * args.steps / elapsed / 1e9, 1),
            "roofline": {"kernel": "logit gradient (grad_variant %d)" % L.tune("grad_variant"), "bound": "hbm",
                         "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
                         "traffic": traffic, "algorithmic_bytes_per_launch": grad_bytes,
                         "avg_launch_ms": round(g_ms, 4) if g_ms else None,
                         "live_rows": live, "inband_rows": n_band,
                         "formula_bytes_per_launch": formula_grad_bytes,
                         "formula_gbps": round(formula_grad_bytes / (g_ms * 1e-3) / 1e9, 1) if g_ms else None,
                         "copy_gbps_same_buffers": copy_gbps,
                         "frac_of_copy_same_buffers": round(achieved / copy_gbps, 4) if achieved and copy_gbps else None},
            "kernels": {
                "log_softmax": {"avg_ms": round(s_ms, 4) if s_ms else None,
                                "gbps": round(softmax_bytes / (s_ms * 1e-3) / 1e9, 1) if s_ms else None},
                "alpha_beta": {"avg_ms": round(d_ms, 4) if d_ms else None},
                "grad": {"avg_ms": round(g_ms, 4) if g_ms else None, "gbps": round(achieved, 1) if achieved else None},
            },
            "cpu_baseline": cpu,
            "tune": args.tune or None,
            "alloc": {"acts": acts.data_ptr(), "grads": acts.grad.data_ptr()},
            "loss_check": float(loss.item()),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def same_buffers_copy_gbps(lib, L, dev, src_t, dst_t, gib=8, reps=5):
    """Device-copy rate on THIS run's own buffers (mrnnt_copy_probe: the gradient pass's access pattern,
    nontemporal, read + write bytes / time, HIP events on the stream it runs on), acts -> grads, after the timed
    region. HBM streaming rates depend on where a buffer sits physically: two 52 GB buffers of one process can
    differ by ~20 % for writes and ~10 % for reads (profiles/r01/grad_placement_study.json), so the gradient
    kernel is compared with a plain copy between the same two buffers. None if the buffers are too small."""
    n = min(gib << 30, src_t.numel() * src_t.element_size(), dst_t.numel() * dst_t.element_size())
    n -= n % 16
    if n < (1 << 30):
        return None
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    run = lambda: L.check(lib.mrnnt_copy_probe(ctypes.c_void_p(dst_t.data_ptr()), ctypes.c_void_p(src_t.data_ptr()),  # noqa: E731
                                               n, sp), "copy_probe")
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return round(2 * n / (ms * 1e-3) / 1e9, 1)


def synthetic_alignment(labels, T, S, k):
    """[B, T_max] alignment with label i of utterance b at frame floor((i + 0.5) T_b / S_b) (blank = 0 elsewhere),
    and the number of lattice rows the log-softmax pass reads under it (the alignment window of each column:
    mrnnt_softmax.hip align_window, from the band of gpu_workspace_manager.h:191-219)."""
    B = len(T)
    al = np.zeros((B, int(T.max())), np.int32)
    n_window = 0
    for b in range(B):
        Tb, Sb = int(T[b]), int(S[b])
        fr = ((np.arange(Sb) + 0.5) * Tb / max(Sb, 1)).astype(np.int64)
        al[b, fr] = labels[b, :Sb]
        m = np.concatenate([[0], np.cumsum(al[b, :Tb] != 0)])
        t = np.arange(Tb)
        mn = m[np.clip(t + 1 - k, 0, Tb)]
        mx = m[np.clip(t + 1 + k, 0, Tb)]
        wlo = np.minimum(mn - 1, np.concatenate([[0], mn[:-1]]))
        whi = np.maximum(mx, np.concatenate([[0], mx[:-1]]))
        lo = np.maximum(np.maximum(0, t - (Tb - Sb)), wlo)
        hi = np.minimum(np.minimum(t, Sb), whi)
        n_window += int(np.maximum(hi - lo + 1, 0).sum())
    return al, n_window


def live_rows(op, L, acts, labels, T, S, dev, align=None, k=0):
    """In-band rows the gradient kernel reads on this workload (mrnnt_grad_live_rows after one forward)."""
    prep = op._Prepared(acts.detach(), labels, T, S, align, k, 0)
    _, ws = op._forward(prep, with_beta=True)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    L.check(L.load().mrnnt_grad_live_rows(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                          ctypes.c_void_p(cnt.data_ptr()), prep.stream()), "grad_live_rows")
    return int(cnt.item())


def cpu_baseline(lib, L, acts, labels, T, S, V, n_sample, stream, max_threads=16):
    """Time the reference CPU path on the first n_sample utterances of the same synthetic workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": f"oracle unavailable: {e}"}
    n = min(n_sample, len(T))
    kind = "reference" if O.ref_available() else "port"
    fn = O.ref_rnnt if kind == "reference" else O.oracle_rnnt
    # the reference indexes acts with 32-bit offsets (cpu_workspace_manager.h:48): one call takes at most
    # 2^31 / (rows per utterance * V) utterances (10 at the headline); the sample is that call (<= max_threads
    # utterances, OpenMP over utterances) repeated until n_sample utterances have been processed
    rows_u = T[:n].astype(np.int64) * (S[:n] + 1)
    g = 1
    while g < min(n, max_threads) and int(rows_u[:g + 1].sum()) * V < 2 ** 31:
        g += 1
    reps = (n + g - 1) // g
    rows = int(rows_u[:g].sum())
    host = acts.detach()[:rows].float().cpu().numpy()
    lab = labels[:g].cpu().numpy()
    threads = max(1, min(g, os.cpu_count() or 1))
    finite = True
    t0 = time.perf_counter()
    for _ in range(reps):
        costs, _ = fn(host, lab, T[:g], S[:g], precision="f32", num_threads=threads)
        finite = finite and bool(np.all(np.isfinite(costs)))
    dt = time.perf_counter() - t0
    n = g * reps
    return {"value": round(n / dt, 4), "unit": "utt/s", "cores": threads, "kind": kind,
            "sample": f"{n} utterances of the same workload (T={int(T[0])}, S={int(S[0])}, V={V}): "
                      f"{reps} call(s) of {g}, cost_and_grad at fp32, OpenMP over utterances "
                      f"({threads} threads), {dt:.2f} s",
            "finite": finite}


if __name__ == "__main__":
    main()
