"""Strong scaling of the batch-sharded configs[3] (B = 512 ragged, V = 1024), emulated on ONE MI355X.

    python tools/shard_scaling.py [--worlds 1,2,4,8] [--steps 5] [--warmup 2] [--out FILE]

The sharded path has no data-path collective: rank r of N runs the whole single-GPU path on its
contiguous slice of utterances (distributed.shard_bounds, balanced by rows) and the only exchange is one 4-byte
loss all-reduce (~10-30 us, not included). So the N-GPU step is the slowest rank's slice, and each slice can be
timed alone: `bench.py --config ragged --shard r/N`, one fresh process per slice (so every slice also draws its
own buffers, as every GPU of a node allocates its own). A slice whose acts + grads do not fit HBM writes the
gradient in place over the logits; at N = 1 (292 GB of acts) the batch runs as utterance chunks.
Prints one JSON object: per N the per-rank ms/step, the emulated step (max), utt/s and the rank balance.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {}
    for n in [int(x) for x in a.worlds.split(",")]:
        ranks = []
        for r in range(n):
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "ragged", "--shard", f"{r}/{n}",
                   "--steps", str(a.steps), "--warmup", str(a.warmup), "--no-cpu"]
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                raise SystemExit(f"shard {r}/{n} failed:\n{out.stderr[-3000:]}")
            line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
            ranks.append({"rank": r, "utterances": line["config"]["utterances_per_gpu"],
                          "rows": line["config"]["rows_per_gpu"], "memory_mode": line["config"]["memory_mode"],
                          "chunks": line["config"]["chunks_per_step"], "ms_per_step": line["ms_per_step"],
                          "grad_ms": line["kernels"]["grad"]["avg_ms"], "softmax_ms": line["kernels"]["log_softmax"]["avg_ms"],
                          "grads_placement": line.get("grads_placement")})
            print(json.dumps({"n": n, **ranks[-1]}), file=sys.stderr, flush=True)
        step = max(x["ms_per_step"] for x in ranks)
        utts = sum(x["utterances"] for x in ranks)
        res[n] = {"step_ms_max_over_ranks": step, "utt_per_s": round(utts / (step * 1e-3), 1),
                  "balance_min_over_max": round(min(x["ms_per_step"] for x in ranks) / step, 3), "ranks": ranks}
    text = json.dumps({"config": "configs[3]: B=512 ragged, V=1024, strong scaling (emulated, one GPU)",
                       "results": res}, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main()
