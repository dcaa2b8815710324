"""configs[4] at full size: (B, T, S, V) = (64, 1000, 200, 10000), 514.6 GB of logits -- more than one MI355X holds,
so it runs as bench.py --config c5 runs it: four in-place calls of 16 utterances (~128.6 GB each, gradients written
over the logits). Checked for the whole batch: finite costs and sum_v grad = 0 in every one of the 12.9 M rows;
with MRNNT_FULL_BATCH=1 also every one of the 64 costs against the fp64 oracle (one utterance per oracle call, its
frames over the box's 16 cores). Element-by-element gradients at this V are covered by
test_gpu_surface.py::test_configs4_full_utterance_vs_oracle.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

B, T, S, V, CHUNK, SEED = 64, 1000, 200, 10000, 16, 12


def test_config_c5_whole_batch_in_place_chunks():
    import _mrnnt_lib as L
    import monotonic_rnnt_op as op
    dev = torch.device("cuda:0")
    full = os.environ.get("MRNNT_FULL_BATCH", "0") == "1"
    threads = int(os.environ.get("MRNNT_FULL_BATCH_THREADS", "16"))
    rows_u = T * (S + 1)
    labels = np.random.default_rng(5).integers(1, V, (B, S)).astype(np.int32)
    acts = torch.empty((CHUNK * rows_u, V), dtype=torch.float32, device=dev)
    worst_rs = worst_c = 0.0
    costs_all = np.zeros(B)
    for b0 in range(0, B, CHUNK):
        L.synth_acts(acts.data_ptr(), b0 * rows_u * V, CHUNK * rows_u * V, SEED, 1,
                     torch.cuda.current_stream().cuda_stream)
        costs = torch.empty(CHUNK, dtype=torch.float32)
        lab = torch.from_numpy(np.ascontiguousarray(labels[b0: b0 + CHUNK])).to(dev)
        # lengths on the device, as bench.py --config c5 passes them (planned inside the log-softmax launch)
        Tt = torch.full((CHUNK,), T, dtype=torch.int32, device=dev)
        St = torch.full((CHUNK,), S, dtype=torch.int32, device=dev)
        assert op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(acts, lab, Tt, St, costs, acts, 0) == 0
        for a in range(0, acts.shape[0], 1 << 18):
            worst_rs = max(worst_rs, acts[a: a + (1 << 18)].sum(dim=1, dtype=torch.float64).abs().max().item())
        costs_all[b0: b0 + CHUNK] = costs.numpy()
        print(f"utterances [{b0}, {b0 + CHUNK}): row sums worst {worst_rs:.3e}", flush=True)
    del acts
    torch.cuda.empty_cache()
    assert np.all(np.isfinite(costs_all)) and np.all(costs_all > 0)
    assert worst_rs < 1e-4
    if not full:
        return
    for b in range(B):
        host = O.synth_acts(b * rows_u * V, rows_u * V, seed=SEED).reshape(rows_u, V)
        cr, _ = O.oracle_rnnt(host, labels[b: b + 1], [T], [S], precision="f64", grads=False, num_threads=threads)
        del host
        worst_c = max(worst_c, abs(costs_all[b] - cr[0]) / abs(cr[0]))
        print(f"utterance {b}: cost {costs_all[b]:.6f} oracle {cr[0]:.6f}; worst rel err so far {worst_c:.3e}",
              flush=True)
    print(f"configs[4] all 64 costs: max rel err {worst_c:.3e} (device lengths; library sha256 {L.library_sha256()})")
    assert worst_c <= 1e-4
