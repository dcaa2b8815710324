"""Shared parity helpers: the tolerances of the north star and the comparison rules.

    costs : |dc| <= 1e-4 * max(1, |c|)      (relative for large costs: 1e-4 abs is < 1 ulp at |c| ~ 1e3)
    grads : max |dg| <= 1e-4                 (absolute, fp32)
Non-finite entries must be non-finite in the same places (the reference's inf / NaN semantics).
"""
import contextlib
import glob
import os

import numpy as np

COST_TOL = 1e-4
GRAD_TOL = 1e-4
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(glob.glob(os.path.join(GOLD, "*.npz")))


def assert_costs(c, ref):
    c = np.asarray(c, np.float64)
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(c), fin), (c, ref)
    if fin.any():
        err = np.abs(c[fin] - ref[fin]) / np.maximum(1.0, np.abs(ref[fin]))
        assert err.max() <= COST_TOL, (err.max(), c, ref)


def assert_grads(g, ref, tol=GRAD_TOL):
    assert g.shape == ref.shape
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(g), fin)
    err = np.abs(g[fin] - ref[fin]).max() if fin.any() else 0.0
    assert err <= tol, err


def random_problem(rng, B, Trange, Smax, V, dist="normal", force=None):
    T = rng.integers(Trange[0], Trange[1] + 1, B).astype(np.int32)
    S = np.array([rng.integers(0, min(t, Smax) + 1) for t in T], np.int32)
    for b, (t, s) in (force or {}).items():
        T[b], S[b] = t, s
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = (rng.standard_normal((rows, V)) if dist == "normal" else rng.random((rows, V))).astype(np.float32)
    labels = rng.integers(1, V, (B, max(1, int(S.max())))).astype(np.int32)
    return acts, labels, T, S


def band_mask(T, S):
    """Rows (t, s) of the monotonic band max(0, t-(T-S)) <= s <= min(t, S), packed row order."""
    out = []
    for Tb, Sb in zip(np.asarray(T), np.asarray(S)):
        t = np.arange(Tb)[:, None]
        s = np.arange(Sb + 1)[None, :]
        out.append(((s >= np.maximum(0, t - (Tb - Sb))) & (s <= np.minimum(t, Sb))).reshape(-1))
    return np.concatenate(out)


def assert_state(den, alpha, beta, fx, window=None, beta_too=True, rel=1e-4, den_rel=1e-5):
    """Workspace read-out vs the reference's own per-row state (golden denom_f64 / alpha_f64 / beta_f64 from
    cpu_rnnt.h<double>): denominators on the rows the forward reduced (the band, or `window`), alpha / beta
    on every row (-inf outside the band in both), each within rel (den_rel) * max(1, |ref|)."""
    rows = band_mask(fx["T"], fx["S"]) if window is None else window
    ref_den = fx["denom_f64"]
    fin = rows & np.isfinite(ref_den)
    if fin.any():
        err = np.abs(den[fin].astype(np.float64) - ref_den[fin]) / np.maximum(1.0, np.abs(ref_den[fin]))
        assert err.max() <= den_rel, err.max()
    for got, ref in ((alpha, fx["alpha_f64"]),) + (((beta, fx["beta_f64"]),) if beta_too else ()):
        assert np.array_equal(np.isfinite(got), np.isfinite(ref)), np.argwhere(np.isfinite(got) != np.isfinite(ref))
        f = np.isfinite(ref)
        if f.any():
            err = np.abs(got[f] - ref[f]) / np.maximum(1.0, np.abs(ref[f]))
            assert err.max() <= rel, err.max()


def used_rows(fx):
    """Rows whose log-softmax the reference's recursion combines with finite state: row (t, s) enters alpha(t, s)
    (blank) and alpha(t, s+1) (label) with alpha(t-1, s), and beta(t, s) with beta(t+1, .). A subset of the rows
    any implementation must reduce."""
    a, b = np.isfinite(fx["alpha_f64"]), np.isfinite(fx["beta_f64"])
    out, r = [], 0
    for Tb, Sb in zip(fx["T"], fx["S"]):
        n = int(Tb) * (int(Sb) + 1)
        aa = a[r:r + n].reshape(Tb, Sb + 1)
        prev = np.zeros_like(aa)  # alpha(t-1, s) finite; alpha(-1, s) = [s == 0]
        prev[0, 0] = True
        prev[1:] = aa[:-1]
        nxt = np.zeros_like(aa)
        nxt[:, :-1] = aa[:, 1:]
        out.append((((aa | nxt) & prev) | b[r:r + n].reshape(Tb, Sb + 1)).reshape(-1))
        r += n
    return np.concatenate(out) if out else np.zeros(0, bool)


@contextlib.contextmanager
def knobs(**kv):
    """Run the block through the development build (libmonotonic_rnnt_amd_dev.so) with launch knobs set,
    restoring them afterwards. The product library has no knobs: it always runs the tuned defaults."""
    import _mrnnt_lib as L
    with L.use(L.load_dev()):
        saved = {k: L.tune(k) for k in kv}
        try:
            for k, v in kv.items():
                assert L.tune(k, int(v)) >= 0, k
            yield
        finally:
            for k, v in saved.items():
                L.tune(k, v)
