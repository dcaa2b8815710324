"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

The reference's CpuRNNTComputer (include/cpu_rnnt.h) is compiled in place from /root/reference by
oracle/Makefile into oracle/_ref/libref_rnnt.so; this script drives it through oracle/oracle.py:ref_rnnt
at double (the parity golden: cpu_rnnt.h<double> on fp32 inputs) and at float (cpu_rnnt.h<float>, to
quantify the reference's own fp32 noise). Only data is written: inputs and expected outputs.

Run (in the container that has /root/reference):  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

TOY_PROBS = np.array([
    0.6, 0.3, 0.1, 0.7, 0.1, 0.2, 0.5, 0.1, 0.4,
    0.5, 0.4, 0.1, 0.5, 0.1, 0.4, 0.8, 0.1, 0.1,
    0.4, 0.3, 0.3, 0.5, 0.1, 0.4, 0.7, 0.2, 0.1,
    0.8, 0.1, 0.1, 0.3, 0.1, 0.6, 0.8, 0.1, 0.1], np.float32).reshape(12, 3)


def toy_logits():
    return np.log(TOY_PROBS).astype(np.float32)


def valid_alignment(rng, T, S, labels, blank, Tmax):
    al = np.full((len(T), Tmax), blank, np.int32)
    for b in range(len(T)):
        pos = np.sort(rng.choice(T[b], S[b], replace=False))
        al[b, pos] = labels[b, : S[b]]
    return al


def random_case(rng, B, Trange, Smax, V, blank=0, dist="normal", force=None):
    T = rng.integers(Trange[0], Trange[1] + 1, B).astype(np.int32)
    S = np.array([rng.integers(0, min(t, Smax) + 1) for t in T], np.int32)
    if force:
        for b, (t, s) in force.items():
            T[b], S[b] = t, s
    rows = int(np.sum(T.astype(np.int64) * (S + 1)))
    acts = (rng.standard_normal((rows, V)) if dist == "normal" else rng.random((rows, V))).astype(np.float32)
    L = max(1, int(S.max()))
    choices = np.array([v for v in range(V) if v != blank], np.int32)
    labels = choices[rng.integers(0, len(choices), (B, L))].astype(np.int32)
    return acts, labels, T, S


def cases():
    rng = np.random.default_rng(20261015)
    out = []
    # tests/test_cpu.cpp:10-192 and README.md:83-174
    out.append(dict(name="toy", acts=toy_logits(), labels=np.array([[1, 2]], np.int32), T=[4], S=[2], blank=0))
    # tests/test_cpu.cpp:194-295 (ragged B=2, labels padded {1,0,1,2})
    p = np.concatenate([TOY_PROBS[[0, 1, 3, 4]], TOY_PROBS], 0)
    out.append(dict(name="multibatch", acts=np.log(p).astype(np.float32), labels=np.array([[1, 0], [1, 2]], np.int32),
                    T=[2, 4], S=[1, 2], blank=0))
    # tests/test_cpu.cpp:335-438 / pytorch_binding/test.py:71-130
    for k in (0, 1, 2):
        out.append(dict(name=f"align_toy_k{k}", acts=toy_logits(), labels=np.array([[1, 2]], np.int32), T=[4], S=[2],
                        blank=0, alignment=np.array([[0, 1, 0, 2]], np.int32), max_shift=k))
    out.append(dict(name="align_toy_1202_k0", acts=toy_logits(), labels=np.array([[1, 2]], np.int32), T=[4], S=[2],
                    blank=0, alignment=np.array([[1, 2, 0, 0]], np.int32), max_shift=0))
    # tests/test_cpu.cpp:440-552
    for k in (0, 1, 3):
        out.append(dict(name=f"align_multibatch_k{k}", acts=np.concatenate([toy_logits(), toy_logits()], 0),
                        labels=np.array([[1, 2], [1, 2]], np.int32), T=[4, 4], S=[2, 2], blank=0,
                        alignment=np.array([[0, 1, 0, 2], [1, 2, 0, 0]], np.int32), max_shift=k))
    # tests/test_cpu.cpp:297-333 shape (T=50, S=10, V=15), uniform [0,1) like tests/random.cpp:4-20
    acts = rng.random((50 * 11, 15)).astype(np.float32)
    lab = rng.integers(1, 15, (1, 10)).astype(np.int32)
    lab[0, 4] = lab[0, 5] = lab[0, 6]  # forced repeats, as tests/random.cpp:32-35 does
    out.append(dict(name="infnan_T50_S10_V15", acts=acts, labels=lab, T=[50], S=[10], blank=0))
    # ragged, odd V (scalar path), S=0 and T=S edge cases
    a, l, T, S = random_case(rng, 5, (1, 24), 7, 7, force={0: (5, 0), 1: (6, 6), 2: (1, 0), 3: (1, 1)})
    out.append(dict(name="ragged_v7_edges", acts=a, labels=l, T=T, S=S, blank=0))
    a, l, T, S = random_case(rng, 4, (3, 30), 8, 8, blank=7)
    out.append(dict(name="ragged_v8_blank_last", acts=a, labels=l, T=T, S=S, blank=7))
    a, l, T, S = random_case(rng, 3, (9, 31), 7, 16, force={2: (9, 0)})
    out.append(dict(name="ragged_v16", acts=a, labels=l, T=T, S=S, blank=0))
    a, l, T, S = random_case(rng, 3, (12, 40), 9, 64, dist="uniform")
    al = valid_alignment(rng, T, S, l, 0, int(T.max()))
    out.append(dict(name="align_ragged_v64_k2", acts=a, labels=l, T=T, S=S, blank=0, alignment=al, max_shift=2))
    out.append(dict(name="align_ragged_v64_k0", acts=a, labels=l, T=T, S=S, blank=0, alignment=al, max_shift=0))
    a, l, T, S = random_case(rng, 2, (60, 60), 12, 32, force={0: (60, 12), 1: (60, 12)})
    out.append(dict(name="medium_T60_S12_V32", acts=a, labels=l, T=T, S=S, blank=0))
    a, l, T, S = random_case(rng, 1, (200, 200), 40, 4, force={0: (200, 40)})
    out.append(dict(name="long_T200_S40_V4", acts=a, labels=l, T=T, S=S, blank=0))
    a, l, T, S = random_case(rng, 2, (12, 12), 4, 256, force={0: (12, 4), 1: (10, 3)})
    out.append(dict(name="v256", acts=a, labels=l, T=T, S=S, blank=0))
    a, l, T, S = random_case(rng, 1, (6, 6), 3, 1024, force={0: (6, 3)})
    a = (a * 3.0).astype(np.float32)
    out.append(dict(name="v1024_wide_logits", acts=a, labels=l, T=T, S=S, blank=0))
    # labels that contain the blank inside S (cpu_rnnt.h:224-230: the blank branch wins)
    a, l, T, S = random_case(rng, 1, (7, 7), 3, 5, force={0: (7, 3)})
    l[0, 1] = 0
    out.append(dict(name="label_equals_blank", acts=a, labels=l, T=T, S=S, blank=0))
    return out


def main():
    if not O.ref_available():
        O.build(ref=True)
    manifest = []
    for c in cases():
        kw = dict(blank=c["blank"], alignment=c.get("alignment"), max_shift=c.get("max_shift", 0))
        c64, g64, d64, a64, b64 = O.ref_rnnt(c["acts"], c["labels"], c["T"], c["S"], precision="f64", debug=True, **kw)
        c32, g32 = O.ref_rnnt(c["acts"], c["labels"], c["T"], c["S"], precision="f32", **kw)
        cc64, _ = O.ref_rnnt(c["acts"], c["labels"], c["T"], c["S"], precision="f64", grads=False, **kw)
        rec = dict(acts=c["acts"], labels=np.asarray(c["labels"], np.int32), T=np.asarray(c["T"], np.int32),
                   S=np.asarray(c["S"], np.int32), blank=np.int32(c["blank"]),
                   costs_f64=c64, grads_f64=g64, denom_f64=d64, alpha_f64=a64, beta_f64=b64,
                   costs_f32=c32, grads_f32=g32, costs_only_f64=cc64)
        if c.get("alignment") is not None:
            rec["alignment"] = np.asarray(c["alignment"], np.int32)
            rec["max_shift"] = np.int32(c["max_shift"])
        np.savez_compressed(os.path.join(HERE, c["name"] + ".npz"), **rec)
        with np.errstate(invalid="ignore"):
            dg = float(np.nanmax(np.abs(g64 - g32))) if g64.size else 0.0
        manifest.append(dict(name=c["name"], B=len(c["T"]), V=int(c["acts"].shape[1]), rows=int(c["acts"].shape[0]),
                             costs_f64=[float(x) for x in c64], f32_vs_f64_max_abs_grad=dg,
                             finite=bool(np.all(np.isfinite(c64)))))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(dict(generator="oracle/_ref/libref_rnnt.so (reference include/cpu_rnnt.h compiled in place)",
                       cases=manifest), f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
