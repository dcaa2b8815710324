"""bench.py -- MI355X monotonic RNN-T loss+grad throughput (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config headline|c2|ragged|ragged64|c5]

One step = forward (log-softmax row reduce + alpha/beta DP) + backward (logit gradient, dL/dcost fused)
over one batch through the autograd surface (monotonic_rnnt_loss(...).sum().backward()), plus, for N > 1,
the single RCCL all-reduce of the summed loss. Inputs are synthetic and resident in HBM before timing.

--gpus N > 1 without a torch.distributed environment launches N ranks itself (torch.distributed.run, one
process per GPU, 127.0.0.1 rendezvous) before this process touches the GPU, and exits with their status;
rank 0 prints the JSON line. Under torchrun (WORLD_SIZE set) WORLD_SIZE must equal --gpus.

Scaling: headline / c2 / c5 are weak (every rank owns its own B utterances); ragged (configs[3], B = 512
global) is strong: the batch is sharded over the ranks by rows (contiguous prefix split).
A rank whose shard does not fit acts + grads in HBM writes the gradient in place over the logits (the
reference extension's output-buffer form, gpu_monotonic_rnnt(..., grads=acts)); a shard whose logits alone do
not fit (configs[3] at N = 1: 292 GB) runs as chunks of utterances. In those two modes the logits are
regenerated before each chunk outside the timed intervals, and the step time is the sum of the timed chunk
intervals (each bracketed by barrier + synchronize).

Rank 0 prints ONE JSON line with the contract fields plus:
  roofline     : the gradient kernel (dominant): algorithmic bytes (N_live + N) * V * elem of its launches (N_live =
                 in-band rows whose fp32 gradient is not exactly zero, the rows it reads) divided by their duration
                 from HIP events recorded around each launch on its stream in the timed region; the SURVEY §8d
                 formula (N_v + N) * V * 4 is reported beside it as formula_bytes_per_launch / formula_gbps
  cpu_baseline : the reference's own CpuRNNTComputer<float> (oracle/_ref) -- or the oracle port when the reference
                 build is absent -- timed on a bounded sample of the same workload on the host's CPU share, as
                 concurrent calls of at most the reference's 32-bit-offset utterance count each; the library's
                 own host implementation (RNNT_CPU) on the same sample is reported beside it
  kernels      : per-kernel average ms and achieved GB/s
"""
import argparse
import ctypes
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "monotonic-rnnt_amd", "pytorch_binding"))

METRIC = "utterances/sec + achieved HBM GB/s, (B,T,S,V)=(64,1000,200,1024)"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def ragged_lengths():
    """configs[3]: B=512, T~U[200,1600], S~U[20,min(300,T)], seed 0."""
    rng = np.random.default_rng(0)
    Tg = rng.integers(200, 1601, 512).astype(np.int32)
    Sg = np.array([rng.integers(20, min(300, t) + 1) for t in Tg], np.int32)
    return Tg, Sg


def lengths_for(config, rank, world):
    """This rank's utterance lengths, V, workload name and scaling mode."""
    if config == "headline":  # BASELINE.json configs[2]
        B, T, S, V = 64, 1000, 200, 1024
        return np.full(B, T, np.int32), np.full(B, S, np.int32), V, "B=64,T=1000,S=200,V=1024 (configs[2], headline)", "weak"
    if config == "c2":  # configs[1]
        B, T, S, V = 16, 200, 40, 256
        return np.full(B, T, np.int32), np.full(B, S, np.int32), V, "B=16,T=200,S=40,V=256 (configs[1])", "weak"
    if config == "halo":  # (experiments) a chase-launch shape with the 4-wave halo recursion: S + 1 = 101 > 64
        B, T, S, V = 16, 400, 100, 256
        return np.full(B, T, np.int32), np.full(B, S, np.int32), V, "B=16,T=400,S=100,V=256 (4-wave chase)", "weak"
    if config == "c5":  # configs[4]: V = 10000, 64 utterances = 514.6 GB of acts: run as chunks
        B, T, S, V = 64, 1000, 200, 10000
        return (np.full(B, T, np.int32), np.full(B, S, np.int32), V,
                "B=64,T=1000,S=200,V=10000 (configs[4], large vocab; chunked, in-place grads)", "weak")
    if config == "ragged64":  # the first 64 utterances of configs[3]
        Tg, Sg = ragged_lengths()
        return Tg[:64], Sg[:64], 1024, "first 64 utterances of configs[3] (ragged T, S), V=1024", "weak"
    if config == "ragged":  # configs[3], sharded over ranks
        Tg, Sg = ragged_lengths()
        lo, hi = ragged_slice(rank, world)
        return (Tg[lo:hi], Sg[lo:hi], 1024,
                f"B=512 ragged (T~U[200,1600], S~U[20,min(300,T)]), V=1024, sharded over {world}", "strong")
    raise SystemExit(f"unknown config {config}")


def ragged_slice(rank, world):
    """Utterances [lo, hi) of configs[3] owned by `rank` (contiguous prefix split balanced by rows, §8e)."""
    from distributed import shard_bounds
    Tg, Sg = ragged_lengths()
    return shard_bounds(Tg.astype(np.int64) * (Sg + 1), world)[rank]


def labels_for(config, scaling, rank, world, B, S_max, V):
    """Synthetic labels U[1, V-1]: weak-scaled configs draw each rank's own batch (seed 1 + rank); the strong-scaled
    configs[3] draws the global batch (seed 1) and each rank takes its slice, so every world size computes the
    same 512 utterances."""
    if scaling != "strong":
        return np.random.default_rng(1 + rank).integers(1, V, (B, S_max)).astype(np.int32)
    Tg, Sg = ragged_lengths()
    lo, hi = ragged_slice(rank, world)
    glob = np.random.default_rng(1).integers(1, V, (len(Tg), max(1, int(Sg.max())))).astype(np.int32)
    return np.ascontiguousarray(glob[lo:hi, :S_max])


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="headline", choices=["headline", "c2", "ragged", "ragged64", "c5", "halo"])
    ap.add_argument("--cpu-sample", type=int, default=16, help="utterances in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the CPU baseline (0 = this process's CPU share: affinity / cgroup quota)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--acts-dist", default="normal", choices=["normal", "uniform"],
                    help="synthetic logit distribution: counter-hash N(0,1)-like (default) or U[0,1), the reference's "
                         "own generator's distribution (tests/random.cpp:4-20); the gradient kernel's bytes depend on "
                         "it through the live-row fraction")
    ap.add_argument("--acts-dtype", default="f32", choices=["f32", "bf16", "f16"],
                    help="element type of acts/grads (extension; the headline metric is f32, the reference's type)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="launch knob (runs the development build libmonotonic_rnnt_amd_dev.so; experiments only)")
    ap.add_argument("--align-k", type=int, default=None,
                    help="alignment-restricted loss (restrict_to_alignment, max_distance_from_alignment = K) on a "
                         "synthetic alignment with the labels evenly spaced over the frames")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, the real path) or gloo (rehearsal: several ranks may share one GPU)")
    ap.add_argument("--hbm-budget-gb", type=float, default=0.0,
                    help="cap the bytes a rank may allocate for acts (+ grads) (0 = free HBM minus a reserve)")
    ap.add_argument("--graph", action="store_true",
                    help="capture forward + backward once in a HIP graph and time its replays (host-launch-bound "
                         "sizes such as configs[1]); per-kernel times then come from eager steps after the timing")
    ap.add_argument("--host-lengths", action="store_true",
                    help="time the steps with input / label lengths as host tensors (planned exactly on the host); "
                         "the default passes them as GPU tensors, the reference's calling convention "
                         "(monotonic_rnnt.cu:85-88: planned without reading them back, lattice built on the device). "
                         "The other form is timed after the measured steps in the same process (lengths_ab)")
    ap.add_argument("--device-lengths", action="store_true", help=argparse.SUPPRESS)  # (the default; kept for old scripts)
    ap.add_argument("--no-lengths-ab", action="store_true", help="skip timing the other lengths form")
    ap.add_argument("--shard", default=None, metavar="R/N",
                    help="time only shard R of the N-way sharded config in this one process (strong-scaling "
                         "emulation on one GPU: the sharded path has no data-path collective; tools/shard_scaling.py)")
    ap.add_argument("--cpu-worker", default=None, help=argparse.SUPPRESS)
    return ap.parse_args()


# ---------------------------------------------------------------------------------------------------------
# N-rank launch (before any GPU call in this process)

def launch_ranks(args) -> int:
    import torch
    n = args.gpus
    if args.dist_backend == "nccl" and torch.cuda.device_count() < n:  # device_count does not initialise HIP
        print(f"bench.py: --gpus {n} needs {n} GPUs, {torch.cuda.device_count()} visible "
              "(use --dist-backend gloo to rehearse several ranks on one GPU)", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


# ---------------------------------------------------------------------------------------------------------

def main():
    args = parse()
    if args.cpu_worker:
        return cpu_worker(json.loads(args.cpu_worker))
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or 1)
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.shard:  # checked before anything touches the GPU
        try:
            r, n = (int(x) for x in args.shard.split("/"))
        except ValueError:
            raise SystemExit(f"bench.py: --shard wants R/N, got {args.shard!r}")
        if world != 1 or not 0 <= r < n:
            raise SystemExit("bench.py: --shard R/N times one shard in one process (0 <= R < N, --gpus 1)")
        args.shard = (r, n)
    if args.graph and args.config in ("ragged", "c5"):
        raise SystemExit("bench.py: --graph needs a resident config (headline, c2, ragged64)")
    import _mrnnt_lib as L
    if args.tune:
        with L.use(L.load_dev()):
            for kv in args.tune:
                k, v = kv.split("=")
                if L.tune(k, int(v)) < 0:
                    raise SystemExit(f"unknown knob {k}")
            run(args, world)
    else:
        run(args, world)


def run(args, world):
    import torch
    import torch.distributed as dist
    import monotonic_rnnt_op as op
    import _mrnnt_lib as L

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

    def coll(x):  # gloo collectives run on host tensors
        return x.cpu() if gloo else x

    # which device each rank drives (LOCAL_RANK -> device index, PCI bus): under RCCL every rank owns its own GPU
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "local_rank": local_rank, "device": dev_index,
          "pci_bus": getattr(props, "pci_bus_id", None), "pci_device": getattr(props, "pci_device_id", None)}
    rank_devices = [me]
    if world > 1:
        rank_devices = [None] * world
        dist.all_gather_object(rank_devices, me)
        if not gloo and len({(d["device"], d["pci_bus"], d["pci_device"]) for d in rank_devices}) != world:
            raise SystemExit(f"bench.py: ranks share a GPU under RCCL: {rank_devices}")

    def barrier():
        if world > 1:
            dist.barrier()

    cfg_rank, cfg_world = (rank, world) if not args.shard else args.shard
    T, S, V, workload, scaling = lengths_for(args.config, cfg_rank, cfg_world)
    if args.shard:
        workload += f"; shard {cfg_rank} of {cfg_world} timed alone on this GPU"
    B = len(T)
    elem = {"f32": 4, "bf16": 2, "f16": 2}[args.acts_dtype]
    rows_u = T.astype(np.int64) * (S + 1)
    rows = int(rows_u.sum())
    n_band = int(np.sum((S.astype(np.int64) + 1) * (T - S + 1) - 1))  # in-band rows N_v
    # global row offset of this rank's first utterance, so every rank streams different synthetic data
    all_rows = [rows]
    if world > 1:
        t = coll(torch.tensor([rows], dtype=torch.int64, device=dev))
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        all_rows = [int(x.item()) for x in g]
    row0 = sum(all_rows[:rank])
    if args.shard:  # the global row offset of shard R: every shard streams its own part of the synthetic batch
        row0 = sum(int(np.sum(lengths_for(args.config, i, cfg_world)[0].astype(np.int64) *
                              (lengths_for(args.config, i, cfg_world)[1] + 1))) for i in range(cfg_rank))

    # memory plan: acts + grads resident (autograd path), else grads in place, else chunks of utterances
    free, _ = torch.cuda.mem_get_info(dev)
    budget = args.hbm_budget_gb * 1e9 if args.hbm_budget_gb > 0 else free - 6e9
    ws_per_row = 48  # workspace bytes per lattice row (den fp32 + lpb/lpe/alpha/beta fp64, rounded up)
    need = rows * V * elem
    if 2 * need + rows * ws_per_row <= budget:
        mode, chunks = "resident", [(0, B)]
    else:
        mode = "inplace"
        chunks, lo, acc = [], 0, 0
        for b in range(B):
            nb = int(rows_u[b]) * (V * elem + ws_per_row)
            if acc and acc + nb > budget:
                chunks.append((lo, b))
                lo, acc = b, 0
            acc += nb
        chunks.append((lo, B))
        if args.acts_dtype != "f32":
            raise SystemExit("the in-place / chunked modes regenerate fp32 logits; use --acts-dtype f32")
    crow = np.concatenate([[0], np.cumsum(rows_u)])
    max_chunk_rows = max(int(crow[hi] - crow[lo]) for lo, hi in chunks)

    stream_h = torch.cuda.current_stream(dev).cuda_stream
    normal = args.acts_dist == "normal"
    acts_buf = torch.empty((max_chunk_rows, V), dtype=torch.float32, device=dev)
    labels_all = labels_for(args.config, scaling, cfg_rank, cfg_world, B, max(1, int(S.max())), V)
    labels_dev = torch.from_numpy(labels_all).to(dev)

    def synth(lo, hi):
        n = int(crow[hi] - crow[lo])
        L.synth_acts(acts_buf.data_ptr(), (row0 + int(crow[lo])) * V, n * V, 0, normal, stream_h)
        return acts_buf[:n]

    align = n_window = None
    if args.align_k is not None:
        if mode != "resident":
            raise SystemExit("--align-k needs a resident config")
        al_np, n_window = synthetic_alignment(labels_all, T, S, args.align_k)
        align = torch.from_numpy(al_np).to(dev)
        workload += f", alignment-restricted (k={args.align_k}, labels evenly spaced)"

    T_h, S_h = torch.from_numpy(T), torch.from_numpy(S)
    T_g, S_g = T_h.to(dev), S_h.to(dev)
    device_lengths = not args.host_lengths
    T_t, S_t = (T_g, S_g) if device_lengths else (T_h, S_h)
    prof_steps = min(args.steps, 100) if args.graph else args.steps  # steps the per-kernel times cover
    lengths_ab = None
    if args.graph and mode != "resident":
        raise SystemExit("--graph needs a resident config")
    if mode == "resident":
        acts = synth(0, B)
        if args.acts_dtype != "f32":
            acts = acts.to(torch.bfloat16 if args.acts_dtype == "bf16" else torch.float16)
            del acts_buf
            torch.cuda.empty_cache()
        acts.requires_grad_(True)
        torch.cuda.synchronize()

        def loss_and_grad(Tl, Sl):
            costs = op.monotonic_rnnt_loss(acts, labels_dev, Tl, Sl, align, args.align_k or 0, blank_label=0)
            loss = costs.sum()
            loss.backward()
            return loss

        def reduce(loss):
            if world > 1:
                tot = coll(loss.detach().clone())
                dist.all_reduce(tot)  # the one RCCL exchange of the path: 4 bytes over xGMI

        def make_steps(Tl, Sl):
            def eager_step():
                acts.grad = None
                loss = loss_and_grad(Tl, Sl)
                reduce(loss)
                return loss

            if not args.graph:
                return eager_step, eager_step
            # forward + backward captured once in a HIP graph (torch.cuda.graph) and replayed: no host work per
            # step beyond one graph launch; acts.grad lives in the graph's pool and is rewritten by every replay
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    eager_step()
            torch.cuda.current_stream(dev).wait_stream(side)
            acts.grad = None
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                g_loss = loss_and_grad(Tl, Sl)

            def replay_step():
                graph.replay()
                reduce(g_loss)
                return g_loss

            return replay_step, eager_step

        def timed_steps(step, n):
            torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            for _ in range(n):
                loss = step()
            torch.cuda.synchronize()
            barrier()
            return time.perf_counter() - t0, loss

        step, eager_step = make_steps(T_t, S_t)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        barrier()
        L.profile_enable(not args.graph)
        elapsed, loss = timed_steps(step, args.steps)
        loss_val = loss.detach().reshape(1).double()
        if args.graph:  # replays launch no kernels from the host: per-kernel times from eager steps after timing
            L.profile_enable(True)
            for _ in range(prof_steps):
                eager_step()
            torch.cuda.synchronize()
        prof_main = L.profile_read()
        L.profile_enable(False)
        if not args.no_lengths_ab:
            # the other lengths form, same process, buffers and step count, after the measured steps (not in `value`)
            other = (T_h, S_h) if device_lengths else (T_g, S_g)
            step_o, _ = make_steps(*other)
            for _ in range(args.warmup):
                step_o()
            el_o, _ = timed_steps(step_o, args.steps)
            el_m, _ = timed_steps(step, args.steps)  # this form again, right after it (drift check)
            ms = {("device" if device_lengths else "host"): round(elapsed * 1e3 / args.steps, 4),
                  ("host" if device_lengths else "device"): round(el_o * 1e3 / args.steps, 4)}
            lengths_ab = {"ms_per_step": ms, "measured_form_again_ms": round(el_m * 1e3 / args.steps, 4),
                          "device_over_host": round(ms["device"] / ms["host"], 4)}
    else:
        costs_c = torch.zeros(B, dtype=torch.float32, device=dev)
        T_d, S_d = T_g, S_g

        def chunk_step(lo, hi):
            """Regenerate the chunk's logits (not timed), then one timed forward + in-place backward."""
            a = synth(lo, hi)
            torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(a, labels_dev[lo:hi], T_d[lo:hi], S_d[lo:hi], costs_c[lo:hi],
                                                     a, 0)
            if world > 1 and hi == B:
                tot = coll(costs_c.sum().reshape(1))
                dist.all_reduce(tot)  # the loss all-reduce, once per step
            torch.cuda.synchronize()
            barrier()
            return time.perf_counter() - t0

        for _ in range(args.warmup):
            for lo, hi in chunks:
                chunk_step(lo, hi)
        L.profile_enable(True)
        elapsed = 0.0
        for _ in range(args.steps):
            for lo, hi in chunks:
                elapsed += chunk_step(lo, hi)
        loss_val = costs_c.double().sum().reshape(1)
        acts = None
        prof_main = L.profile_read()
        L.profile_enable(False)
    # the whole batch's summed loss (every rank's share, the same all-reduce the step performs), for checks
    loss_val = coll(loss_val)
    if world > 1:
        dist.all_reduce(loss_val)
    loss_val = float(loss_val.item())
    prof = prof_main
    el = coll(torch.tensor([elapsed], dtype=torch.float64, device=dev))
    rank_elapsed = [float(el.item())]
    if world > 1:
        g = [torch.zeros_like(el) for _ in range(world)]
        dist.all_gather(g, el)
        rank_elapsed = [float(x.item()) for x in g]
    elapsed = max(rank_elapsed)
    ar_us = allreduce_latency_us(dist, coll, torch, dev, world)
    total_utts = coll(torch.tensor([B], dtype=torch.int64, device=dev))
    if world > 1:
        dist.all_reduce(total_utts)
    total_utts = int(total_utts.item())

    # live rows: in-band rows whose gradient is not exactly zero in fp32 -- the only acts rows the gradient
    # kernel reads (occupancy skip); counted once after the timed region
    live = 0
    for lo, hi in chunks:
        a = acts.detach() if mode == "resident" else synth(lo, hi)
        live += live_rows(op, L, a, labels_dev[lo:hi], T_h[lo:hi], S_h[lo:hi], dev, align, args.align_k or 0)
    grad_bytes = (live + rows) * V * elem  # algorithmic: read live acts rows once, write every grads row once
    formula_grad_bytes = (n_band + rows) * V * elem  # SURVEY.md §8d formula: every in-band row read
    n_read = n_band if n_window is None else n_window  # rows the log-softmax pass reads
    softmax_bytes = n_read * V * elem
    step_bytes = (n_read + live + rows) * V * elem
    n_chunks = len(chunks)

    def tot_ms(name):
        ms, n = prof[name]
        return (ms, n) if n else (None, 0)

    g_ms, g_n = tot_ms("grad")
    s_ms, s_n = tot_ms("log_softmax")
    d_ms, d_n = tot_ms("alpha_beta")
    c_ms, c_n = tot_ms("chase")
    # the bytes of all gradient launches of the timed steps over their summed duration
    achieved = grad_bytes * prof_steps / (g_ms * 1e-3) / 1e9 if g_ms else None
    g_avg = g_ms / g_n if g_ms else None

    traffic = traffic_source = None  # PMC traffic is counted by rocprofv3 in its own run (tools/gpu_profile.sh)
    pmc_path = os.path.join(ROOT, "profiles", "pmc_grad_traffic.json")
    if os.path.exists(pmc_path) and mode == "resident" and not args.tune:
        try:
            pm = json.load(open(pmc_path))
            ek = {"f32": "IoF32", "bf16": "IoBF16", "f16": "IoF16"}[args.acts_dtype]
            # the counter record belongs to this exact workload only: same config and acts dtype, and the same
            # live-row bytes per launch (an alignment band, a shard or chunking all change those)
            # workload, measured on a library built from these very sources (source_sha256: csrc/ + include/ +
            # Makefile + ROCm release; the build is path-independent) or this very binary (lib_sha256)
            if (pm.get("config") == args.config and pm.get("dtype") == args.acts_dtype
                    and pm.get("kernel", "").startswith(f"grad_staged_kernel<{ek}")
                    and pm.get("algorithmic_bytes_per_launch") == grad_bytes // n_chunks
                    and (pm.get("source_sha256") == L.source_sha256()
                         or pm.get("lib_sha256") == lib_sha256(L.LIB_PATH))):
                traffic = pm.get("hbm_bytes_per_launch")
                traffic_source = {"file": os.path.relpath(pmc_path, ROOT), "run": pm.get("source"),
                                  "source_sha256": pm.get("source_sha256"), "lib_sha256": pm.get("lib_sha256"),
                                  "measured_in_this_run": False}
        except Exception:
            traffic = None

    copy_gbps = acts_read_gbps = None
    if mode == "resident" and acts.grad is not None:
        copy_gbps = same_buffers_copy_gbps(L, dev, acts.detach(), acts.grad)
        acts_read_gbps = acts_read_probe_gbps(L, dev, acts.detach())

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0 and args.acts_dtype == "f32":
        cpu = cpu_baseline(op, T, S, V, labels_all, row0, args.cpu_sample, args.cpu_threads, normal)

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
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.acts_dtype,
            "data": f"synthetic: counter-hash {'N(0,1)-like' if normal else 'U[0,1)'} acts (seed 0), labels U[1,V-1] (seed 1+rank; configs[3]: seed 1 over the global batch); inputs resident in HBM",
            "config": {"workload": workload, "utterances_per_gpu": B, "global_batch": total_utts,
                       "rows_per_gpu": rows, "inband_rows_per_gpu": n_band, "V": V,
                       "acts_dist": args.acts_dist, "memory_mode": mode, "chunks_per_step": n_chunks,
                       "execution": "hip_graph_replay" if args.graph else "eager",
                       "lengths": "device" if (device_lengths or mode != "resident") else "host",
                       "rank_devices": rank_devices,
                       **({"window_rows_per_gpu": n_window} if n_window is not None else {}),
                       "parallelism": f"dp{world} (batch-sharded, one 4-byte "
                                      f"{'gloo (rehearsal)' if gloo else 'RCCL'} loss all-reduce)"},
            "achieved_hbm_gbps_step": round(step_bytes * args.steps / elapsed / 1e9, 1),
            "roofline": {"kernel": "logit gradient", "bound": "hbm",
                         "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_source,
                         "algorithmic_bytes_per_launch": grad_bytes // n_chunks,
                         "avg_launch_ms": round(g_avg, 4) if g_avg else None,
                         "live_rows": live, "inband_rows": n_band,
                         "formula_bytes_per_launch": formula_grad_bytes // n_chunks,
                         "formula_gbps": round(formula_grad_bytes * prof_steps / (g_ms * 1e-3) / 1e9, 1) if g_ms else None,
                         "copy_gbps_same_buffers": copy_gbps,
                         "frac_of_copy_same_buffers": round(achieved / copy_gbps, 4) if achieved and copy_gbps else None},
            "kernels": {
                "log_softmax": {"avg_ms": round(s_ms / s_n, 4) if s_ms else None,
                                "gbps": round(softmax_bytes * prof_steps / (s_ms * 1e-3) / 1e9, 1) if s_ms else None,
                                "acts_read_probe_gbps": acts_read_gbps,
                                "frac_of_acts_read_probe": round(softmax_bytes * prof_steps / (s_ms * 1e-3) / 1e9 /
                                                                 acts_read_gbps, 4)
                                if s_ms and acts_read_gbps else None},
                "alpha_beta": {"avg_ms": round(d_ms / d_n, 4) if d_ms else None},
                "chase": {"avg_ms": round(c_ms / c_n, 4) if c_ms else None,
                          "note": "log-softmax + alpha/beta in one launch (mrnnt_chase.hip), where it pays"},
                "grad": {"avg_ms": round(g_avg, 4) if g_avg else None, "gbps": round(achieved, 1) if achieved else None},
            },
            "cpu_baseline": cpu,
            # what the driver needs to compare N > 1 with N = 1: every rank's own step time (value uses the max),
            # their spread, and the loss all-reduce's own latency (timed alone after the steps, max over ranks)
            "ranks": {"n": world, "ms_per_step": [round(e * 1e3 / args.steps, 4) for e in rank_elapsed],
                      "max_ms_per_step": round(max(rank_elapsed) * 1e3 / args.steps, 4),
                      "min_ms_per_step": round(min(rank_elapsed) * 1e3 / args.steps, 4),
                      "balance_min_over_max": round(min(rank_elapsed) / max(rank_elapsed), 4),
                      "devices_distinct": len({(d["device"], d["pci_bus"], d["pci_device"])
                                               for d in rank_devices}) == world,
                      "allreduce_4byte_us": ar_us,
                      "collective": "none" if world == 1 else ("gloo (rehearsal)" if gloo else "RCCL")},
            "lengths_ab": lengths_ab,
            "grads_placement": placement_log(),
            "tune": args.tune or None,
            "loss_check": loss_val,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def allreduce_latency_us(dist, coll, torch, dev, world, reps=50):
    """Average latency of the step's one collective -- a 4-byte sum all-reduce -- each one completed before the next
    (synchronised), max over ranks; None at world size 1."""
    if world == 1:
        return None
    x = coll(torch.ones(1, dtype=torch.float32, device=dev))
    for _ in range(5):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(x)
        torch.cuda.synchronize()
    t = coll(torch.tensor([(time.perf_counter() - t0) / reps * 1e6], dtype=torch.float64, device=dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return round(float(t.item()), 2)


def lib_sha256(path):
    """sha256 of the product library file: a PMC record counts only for the build it was measured on."""
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def placement_log():
    """The gradient-buffer placement decisions of this process (pytorch_binding/_grads_placement.py): per decision
    the fill rate of each candidate block and the one kept; None when no call was large enough."""
    import _grads_placement as GP
    if not GP.enabled():
        return "disabled"
    return {"decisions": GP.ARENA.log or None, **GP.ARENA.stats,
            "fired": GP.ARENA.stats["handed_out"] > 0}


def same_buffers_copy_gbps(L, dev, src_t, dst_t, gib=8, reps=5):
    """Device-copy rate on THIS run's own buffers (mrnnt_copy_probe: the gradient pass's access pattern,
    nontemporal, read + write bytes / time, HIP events on the stream it runs on), acts -> grads, after the timed
    region. HBM streaming rates depend on where a buffer sits physically (profiles/r01/grad_placement_study.json),
    so the gradient kernel is compared with a plain copy between the same two buffers. None if too small."""
    import torch
    n = min(gib << 30, src_t.numel() * src_t.element_size(), dst_t.numel() * dst_t.element_size())
    n -= n % 16
    if n < (1 << 30):
        return None
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    tools = L.devtools()

    def run():
        if tools.mrnnt_copy_probe(ctypes.c_void_p(dst_t.data_ptr()), ctypes.c_void_p(src_t.data_ptr()), n, sp):
            raise RuntimeError("copy probe failed")

    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return round(2 * n / (ms * 1e-3) / 1e9, 1)


def acts_read_probe_gbps(L, dev, acts_t, reps=3):
    """Nontemporal read rate of THIS run's whole acts buffer (mrnnt_read_probe, the log-softmax pass's load stream,
    HIP events on the stream it runs on), after the timed region: like a grads buffer, an acts
    allocation reads at a rate set by its physical placement, which the caller -- not the library -- chose, so
    the log-softmax kernel is also reported against the rate of its own input. None below 1 GiB."""
    import torch
    n = acts_t.numel() * acts_t.element_size()
    n -= n % 16
    if n < (1 << 30):
        return None
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    sink = torch.zeros(4, dtype=torch.uint8, device=dev)
    tools = L.devtools()

    def run():
        if tools.mrnnt_read_probe(ctypes.c_void_p(acts_t.data_ptr()), n, ctypes.c_void_p(sink.data_ptr()), sp):
            raise RuntimeError("read probe failed")

    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    return round(n / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9, 1)


def synthetic_alignment(labels, T, S, k):
    """[B, T_max] alignment with label i of utterance b at frame floor((i + 0.5) T_b / S_b) (blank = 0 elsewhere),
    and the number of lattice rows the log-softmax pass reads under it (the alignment window of each column:
    mrnnt_device.h align_window, from the band of gpu_workspace_manager.h:191-219)."""
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
    import torch
    prep = op._Prepared(acts, labels, T, S, align, k, 0)
    _, ws = op._forward(prep, with_beta=True)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    L.check(L.load().mrnnt_grad_live_rows(ctypes.byref(prep.problem), ctypes.c_void_p(ws.data_ptr()),
                                          ctypes.c_void_p(cnt.data_ptr()), prep.stream()), "grad_live_rows")
    return int(cnt.item())


# ---------------------------------------------------------------------------------------------------------
# CPU baseline

def host_cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 cpu.max quota when there is one
    (the GPU box shows the whole machine's CPUs in nproc / os.cpu_count but grants a share per GPU)."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        quota = None
    env = os.environ.get("OMP_NUM_THREADS")
    share = min(aff, quota) if quota else aff
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota,
            "omp_num_threads_env": int(env) if env and env.isdigit() else None, "share": share}


def cpu_worker(job):
    """One reference call in its own process (bench.py --cpu-worker JSON): regenerate the sample's logits on the
    host with the GPU run's generator, then time the reference's cost_and_grad (or the oracle port)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    T = np.asarray(job["T"], np.int32)
    S = np.asarray(job["S"], np.int32)
    V = int(job["V"])
    labels = np.asarray(job["labels"], np.int32)
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = O.synth_acts(int(job["begin"]), rows * V, seed=0, normal=bool(job.get("normal", True))).reshape(rows, V)
    fn = O.ref_rnnt if job["kind"] == "reference" else O.oracle_rnnt
    t0 = time.perf_counter()
    costs, _ = fn(acts, labels, T, S, precision="f32", num_threads=int(job["threads"]))
    dt = time.perf_counter() - t0
    print(json.dumps({"seconds": dt, "utterances": len(T), "finite": bool(np.all(np.isfinite(costs)))}), flush=True)
    return 0


def cpu_baseline(op, T, S, V, labels, row0, n_sample, threads_arg=0, normal=True):
    """Time the reference CPU path on the first n_sample utterances of the same synthetic workload, using the
    host's CPU share. The reference indexes acts with 32-bit offsets (cpu_workspace_manager.h:48,125-135) and
    parallelises over utterances only (cpu_rnnt.h:54-57), so one call takes at most 2^31 / (rows per utterance
    * V) utterances (10 at the headline) with one busy thread each: the sample runs as concurrent calls in
    separate processes, together using every core of the share."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": f"oracle unavailable: {e}"}
    host = host_cpu_share()
    cores = threads_arg if threads_arg > 0 else host["share"]
    kind = "reference" if O.ref_available() else "port"
    n = min(n_sample, len(T))
    rows_u = T[:n].astype(np.int64) * (S[:n] + 1)
    per_call_cap = max(1, int((2 ** 31 - 1) // (int(rows_u.max()) * V)))  # int32 offsets of one call
    calls = min(n, max(math.ceil(n / per_call_cap), math.ceil(cores / per_call_cap)))
    bounds = np.linspace(0, n, calls + 1).astype(int)
    threads = [max(1, min(int(bounds[c + 1] - bounds[c]), cores // calls)) for c in range(calls)]
    crow = np.concatenate([[0], np.cumsum(rows_u)])
    procs = []
    for c in range(calls):
        lo, hi = int(bounds[c]), int(bounds[c + 1])
        job = {"T": T[lo:hi].tolist(), "S": S[lo:hi].tolist(), "V": V,
               "labels": labels[lo:hi, :max(1, int(S[lo:hi].max()))].tolist(),
               "begin": int((row0 + crow[lo]) * V), "kind": kind, "threads": threads[c], "normal": normal}
        env = dict(os.environ, OMP_NUM_THREADS=str(threads[c]))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", json.dumps(job)],
                                      stdout=subprocess.PIPE, env=env, text=True))
    res = []
    for p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            return {"error": f"cpu worker exited with {p.returncode}"}
        res.append(json.loads(out.strip().splitlines()[-1]))
    wall = max(r["seconds"] for r in res)
    done = sum(r["utterances"] for r in res)
    out = {"value": round(done / wall, 4), "unit": "utt/s", "cores": sum(threads), "kind": kind, "host": host,
           "concurrent_calls": calls, "threads_per_call": threads,
           "sample": f"{done} utterances of the same workload (first T={int(T[0])}, S={int(S[0])}, V={V}): "
                     f"{calls} concurrent reference calls in separate processes (<= {per_call_cap} utterances per "
                     f"call: 32-bit offsets), cost_and_grad at fp32, OpenMP over utterances, slowest call "
                     f"{wall:.2f} s",
           "finite": all(r["finite"] for r in res)}
    out["product_cpu"] = product_cpu_rate(op, T[:n], S[:n], V, labels[:n], row0, cores, normal)
    return out


def product_cpu_rate(op, T, S, V, labels, row0, threads, normal=True):
    """The library's own host implementation (RNNT_CPU, cpu_monotonic_rnnt) on the same sample: one call,
    OpenMP over lattice columns on every core of the share. Reported next to the reference baseline."""
    import torch
    import oracle as O
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = torch.from_numpy(O.synth_acts(row0 * V, rows * V, seed=0, normal=normal).reshape(rows, V))
    grads = torch.empty_like(acts)
    costs = torch.zeros(len(T))
    lab = torch.from_numpy(np.ascontiguousarray(labels[:, :max(1, int(S.max()))]))
    args = (acts, lab, torch.from_numpy(T), torch.from_numpy(S), costs, grads, 0, threads)
    t0 = time.perf_counter()
    op.monotonic_rnnt_cpp.cpu_monotonic_rnnt(*args)
    dt = time.perf_counter() - t0
    return {"value": round(len(T) / dt, 4), "unit": "utt/s", "threads": threads, "seconds": round(dt, 3),
            "finite": bool(torch.isfinite(costs).all())}


if __name__ == "__main__":
    main()
