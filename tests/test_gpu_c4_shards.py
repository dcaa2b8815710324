"""configs[3] at full size as the two rank shards of an N = 2 run: B = 512 ragged utterances (T ~ U[200, 1600],
S ~ U[20, min(300, T)], V = 1024, 292 GB of logits in all), each shard (~146 GB) ONE in-place call on the GPU --
what every rank of `bench.py --config ragged --gpus 2` runs. Checked: finite costs, sum_v grad = 0 in every row,
the first and last utterance of each shard element by element against the fp64 oracle, and (opt-in,
MRNNT_FULL_BATCH=1) every one of the 512 costs against the oracle. Its own module, so the headline module's
105 GB are released before a shard is allocated.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _c4_batch():
    """configs[3] as bench.py draws it (lengths seed 0, labels seed 1 over the global batch)."""
    rng = np.random.default_rng(0)
    Tg = rng.integers(200, 1601, 512).astype(np.int32)
    Sg = np.array([rng.integers(20, min(300, t) + 1) for t in Tg], np.int32)
    labels = np.random.default_rng(1).integers(1, 1024, (512, int(Sg.max()))).astype(np.int32)
    return Tg, Sg, labels


@pytest.fixture(scope="module", params=[0, 1], ids=["shard0", "shard1"])
def c4_shard(request):
    """One rank shard of configs[3] at N = 2 (distributed.shard_bounds: the contiguous row-balanced split bench.py
    uses), ~146 GB of logits generated on the device at their global offsets, run as ONE in-place call
    (gpu_monotonic_rnnt with grads = acts, the per-rank form of bench.py --config ragged)."""
    import _mrnnt_lib as L
    import monotonic_rnnt_op as op
    from distributed import shard_bounds
    dev = torch.device("cuda:0")
    V = 1024
    Tg, Sg, labels = _c4_batch()
    rows_u = Tg.astype(np.int64) * (Sg + 1)
    lo, hi = shard_bounds(rows_u, 2)[request.param]
    r0, nrows = int(rows_u[:lo].sum()), int(rows_u[lo:hi].sum())
    acts = torch.empty((nrows, V), dtype=torch.float32, device=dev)
    L.synth_acts(acts.data_ptr(), r0 * V, nrows * V, 8, 1, torch.cuda.current_stream().cuda_stream)
    costs = torch.empty(hi - lo, dtype=torch.float32)
    # lengths on the device, as bench.py --config ragged passes them (the reference's convention; B = 256 > 64: the
    # setup-kernel planning with the log-softmax's work stealing)
    T, S = torch.from_numpy(Tg[lo:hi]).to(dev), torch.from_numpy(Sg[lo:hi]).to(dev)
    lab = torch.from_numpy(np.ascontiguousarray(labels[lo:hi])).to(dev)
    assert op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(acts, lab, T, S, costs, acts, 0) == 0
    torch.cuda.synchronize()
    d = dict(grads=acts, costs=costs.numpy().astype(np.float64), lo=lo, hi=hi, r0=r0, rows_u=rows_u, Tg=Tg, Sg=Sg,
             labels=labels, V=V)
    yield d
    d.clear()  # pytest keeps the yielded value until after teardown: drop the 146 GB here
    del acts
    torch.cuda.empty_cache()


def test_config_c4_shard_rows_and_oracle(c4_shard):
    """Per rank shard of configs[3] (256 utterances, one call): finite costs, every gradient row sums to zero (in
    row blocks: no full-size fp64 temporary), and the first and last utterance of the shard against the oracle
    (logits regenerated on the host by the bit-identical twin of the device generator)."""
    c, g, V = c4_shard["costs"], c4_shard["grads"], c4_shard["V"]
    assert np.all(np.isfinite(c)) and np.all(c > 0)
    worst = 0.0
    for a in range(0, g.shape[0], 1 << 20):
        worst = max(worst, g[a: a + (1 << 20)].sum(dim=1, dtype=torch.float64).abs().max().item())
    assert worst < 1e-4
    lo, hi, r0, rows_u = c4_shard["lo"], c4_shard["hi"], c4_shard["r0"], c4_shard["rows_u"]
    pick = [lo, hi - 1]
    offs = [int(rows_u[:b].sum()) for b in pick]
    ns = [int(rows_u[b]) for b in pick]
    host = np.concatenate([O.synth_acts(o * V, n * V, seed=8).reshape(n, V) for o, n in zip(offs, ns)])
    cr, gr = O.oracle_rnnt(host, c4_shard["labels"][pick], c4_shard["Tg"][pick], c4_shard["Sg"][pick],
                           precision="f64", num_threads=2)
    del host
    assert np.all(np.abs(c[np.array(pick) - lo] - cr) <= 1e-4 * np.abs(cr))
    h0 = 0
    for o, n in zip(offs, ns):
        assert np.abs(g[o - r0: o - r0 + n].cpu().numpy() - gr[h0: h0 + n]).max() <= 1e-4
        h0 += n


@pytest.mark.skipif(os.environ.get("MRNNT_FULL_BATCH", "0") != "1",
                    reason="opt-in (MRNNT_FULL_BATCH=1): every configs[3] cost against the oracle, minutes on the "
                           "box's 16 cores; its last run is recorded under profiles/r03/tests/")
def test_config_c4_all_costs_match_oracle(c4_shard):
    """Every cost of the shard against the fp64 oracle (costs only), in groups of 16 utterances."""
    c, V = c4_shard["costs"], c4_shard["V"]
    lo, hi, rows_u = c4_shard["lo"], c4_shard["hi"], c4_shard["rows_u"]
    threads = int(os.environ.get("MRNNT_FULL_BATCH_THREADS", "16"))
    worst = 0.0
    for b0 in range(lo, hi, 16):
        b1 = min(hi, b0 + 16)
        off, n = int(rows_u[:b0].sum()), int(rows_u[b0:b1].sum())
        host = O.synth_acts(off * V, n * V, seed=8).reshape(n, V)
        cr, _ = O.oracle_rnnt(host, c4_shard["labels"][b0:b1], c4_shard["Tg"][b0:b1], c4_shard["Sg"][b0:b1],
                              precision="f64", grads=False, num_threads=threads)
        del host
        worst = max(worst, float(np.max(np.abs(c[b0 - lo: b1 - lo] - cr) / np.abs(cr))))
        print(f"utterances [{b0}, {b1}): worst rel err so far {worst:.3e}", flush=True)  # progress for long runs
    import _mrnnt_lib as L
    print(f"configs[3] utterances [{lo}, {hi}): costs max rel err {worst:.3e} (device lengths; library sha256 "
          f"{L.library_sha256()})")
    assert worst <= 1e-4
