"""The oracle (oracle/rnnt_oracle.c) pinned against the reference: golden vectors produced by the
reference's own CpuRNNTComputer (tests/golden/make_golden.py) and the reference tests' known answers
(tests/test_cpu.cpp, pytorch_binding/test.py, README.md:117-174). CPU only."""
import glob
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(glob.glob(os.path.join(GOLD, "*.npz")))


def load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def run(fx, precision, grads=True, debug=False):
    return O.oracle_rnnt(fx["acts"], fx["labels"], fx["T"], fx["S"], blank=int(fx["blank"]),
                         alignment=fx.get("alignment"), max_shift=int(fx.get("max_shift", 0)),
                         precision=precision, grads=grads, debug=debug)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_oracle_matches_reference_golden_bitexact(path):
    fx = dict(np.load(path))
    c, g, d, a, b = run(fx, "f64", debug=True)
    np.testing.assert_array_equal(c, fx["costs_f64"])
    np.testing.assert_array_equal(g, fx["grads_f64"])
    np.testing.assert_array_equal(d, fx["denom_f64"])
    np.testing.assert_array_equal(a, fx["alpha_f64"])
    np.testing.assert_array_equal(b, fx["beta_f64"])
    c32, g32 = run(fx, "f32")
    np.testing.assert_array_equal(c32, fx["costs_f32"])
    np.testing.assert_array_equal(g32, fx["grads_f32"])
    cc, none = run(fx, "f64", grads=False)
    assert none is None
    np.testing.assert_array_equal(cc, fx["costs_only_f64"])


def test_known_answers_toy():
    # tests/test_cpu.cpp:57 (cost), :114-192 (grads, 1e-2), pytorch_binding/test.py:64-66
    fx = load("toy")
    c, g = run(fx, "f64")
    assert abs(c[0] - (-np.log(0.363))) < 1e-4
    expected = np.array([0.04, -0.14, 0.1, 0, 0, 0, 0, 0, 0, 0.13, -0.19, 0.06, -0.04, 0.04, -0.01, 0, 0, 0,
                         0.06, -0.1, 0.04, 0.01, 0.07, -0.08, -0.06, 0.04, 0.02, 0, 0, 0, 0.14, 0.05, -0.19,
                         -0.11, 0.05, 0.05]).reshape(12, 3)
    assert np.abs(g - expected).max() < 1e-2
    # exact fp32 values captured from the reference
    assert abs(g[0, 0] - 0.041322) < 1e-6 and abs(g[11, 0] - (-0.105785)) < 1e-6


def test_known_answers_multibatch():
    # tests/test_cpu.cpp:291-294
    c, _ = run(load("multibatch"), "f64")
    assert abs(c[0] - (-np.log(0.39))) < 1e-4 and abs(c[1] - (-np.log(0.363))) < 1e-4


@pytest.mark.parametrize("k,p", [(2, 0.363), (0, 0.072), (1, 0.2958)])
def test_known_answers_align(k, p):
    # tests/test_cpu.cpp:406-433
    c, _ = run(load(f"align_toy_k{k}"), "f64")
    assert abs(c[0] - (-np.log(p))) < 1e-4


@pytest.mark.parametrize("k,p0,p1", [(3, 0.363, 0.363), (0, 0.072, 0.0672), (1, 0.2958, 0.192)])
def test_known_answers_align_multibatch(k, p0, p1):
    # tests/test_cpu.cpp:512-547
    c, _ = run(load(f"align_multibatch_k{k}"), "f64")
    assert abs(c[0] - (-np.log(p0))) < 1e-4 and abs(c[1] - (-np.log(p1))) < 1e-4


def test_known_answers_pytorch_binding():
    # pytorch_binding/test.py:110 (k=1 -> 1.22) and :128 (alignment [1,2,0,0], k=0 -> 2.7)
    assert abs(run(load("align_toy_k1"), "f64")[0][0] - 1.22) < 1e-2
    assert abs(run(load("align_toy_1202_k0"), "f64")[0][0] - 2.7) < 1e-2


def test_infnan():
    # tests/test_cpu.cpp:297-333
    c, g = run(load("infnan_T50_S10_V15"), "f64")
    assert np.all(np.isfinite(c)) and np.all(np.isfinite(g))


def test_invalid_lengths():
    acts = np.zeros((12, 3), np.float32)
    with pytest.raises(O.OracleError):
        O.oracle_rnnt(acts, [[1, 2, 1]], [2], [3])  # T < S -> RNNT_STATUS_INVALID_VALUE


@pytest.mark.skipif(not O.ref_available(), reason="reference build (oracle/_ref) not present")
def test_oracle_vs_reference_random_bitexact():
    rng = np.random.default_rng(7)
    for trial in range(25):
        B = int(rng.integers(1, 5))
        T = rng.integers(1, 30, B).astype(np.int32)
        S = np.array([rng.integers(0, min(t, 8) + 1) for t in T], np.int32)
        V = int(rng.integers(2, 20))
        rows = int(np.sum(T * (S + 1)))
        acts = rng.standard_normal((rows, V)).astype(np.float32)
        labels = rng.integers(1, V, (B, max(1, S.max()))).astype(np.int32)
        blank = 0 if trial % 3 else int(rng.integers(0, V))
        for prec in ("f64", "f32"):
            c, g = O.oracle_rnnt(acts, labels, T, S, blank=blank, precision=prec)
            cr, gr = O.ref_rnnt(acts, labels, T, S, blank=blank, precision=prec)
            np.testing.assert_array_equal(c, cr)
            np.testing.assert_array_equal(g, gr)


def test_synth_generator_deterministic():
    a = O.synth_acts(1000, 4096, seed=3)
    b = O.synth_acts(1000 + 96, 4000, seed=3)
    np.testing.assert_array_equal(a[96:], b)
    assert abs(a.mean()) < 0.1 and abs(a.std() - 1.0) < 0.05
    u = O.synth_acts(0, 4096, seed=1, normal=False)
    assert u.min() >= 0 and u.max() < 1
