"""ctypes bindings for the CPU checkers (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product package (monotonic-rnnt_amd/) never imports it.

  oracle_rnnt(...)   -> our C restatement (oracle/rnnt_oracle.c), precision "f64" (golden) or "f32"
  ref_rnnt(...)      -> the reference's own CpuRNNTComputer compiled in place (oracle/_ref), when built
  synth_acts(...)    -> host twin of the device synthetic generator (bit-identical)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(HERE, "liboracle.so")
_REF = os.path.join(HERE, "_ref", "libref_rnnt.so")

_lib = None
_ref = None


def build(ref: bool = True) -> None:
    """Compile the checkers (gcc). The reference build only happens where its sources exist."""
    subprocess.run(["make", "-s", "-C", HERE, "all" if ref else os.path.join(HERE, "liboracle.so")], check=True)


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build(ref=False)
        _lib = ctypes.CDLL(_LIB)
        for name in ("mrnnt_oracle_f64", "mrnnt_oracle_f32"):
            fn = getattr(_lib, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                           ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_int]
        _lib.mrnnt_oracle_synth_acts.restype = None
        _lib.mrnnt_oracle_synth_acts.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                                 ctypes.c_int]
    return _lib


def ref_available() -> bool:
    return os.path.exists(_REF)


def _load_ref():
    global _ref
    if _ref is None:
        _ref = ctypes.CDLL(_REF)
        for name in ("ref_rnnt_f32", "ref_rnnt_f64"):
            fn = getattr(_ref, name)
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return _ref


class OracleError(RuntimeError):
    pass


def _prep(acts, labels, T, S):
    acts = np.ascontiguousarray(acts, dtype=np.float32)
    T = np.ascontiguousarray(T, dtype=np.int32).reshape(-1)
    S = np.ascontiguousarray(S, dtype=np.int32).reshape(-1)
    labels = np.ascontiguousarray(labels, dtype=np.int32)
    if labels.ndim == 1:
        labels = labels.reshape(len(T), -1) if labels.size else np.zeros((len(T), 0), np.int32)
    return acts, labels, T, S


def oracle_rnnt(acts, labels, T, S, blank=0, alignment=None, max_shift=0, align_blank=None, precision="f64",
                grads=True, num_threads=0, debug=False):
    """Restatement of cpu_rnnt.h. Returns (costs, grads|None[, denom, alpha, beta]) as numpy arrays.

    labels: [B, L] with the true row stride L (the reference uses max(S) -- identical when L == max(S)).
    alignment: [B, L_T] int, max_shift: k, align_blank: blank used to parse the alignment (default: blank).
    """
    acts, labels, T, S = _prep(acts, labels, T, S)
    B = len(T)
    V = acts.shape[1] if acts.ndim == 2 else int(acts.size // max(1, int(np.sum(T.astype(np.int64) * (S + 1)))))
    rows = int(np.sum(T.astype(np.int64) * (S.astype(np.int64) + 1)))
    dt = np.float64 if precision == "f64" else np.float32
    fn = _load().mrnnt_oracle_f64 if precision == "f64" else _load().mrnnt_oracle_f32
    costs = np.zeros(B, dt)
    g = np.zeros((rows, V), dt) if grads else None
    den = np.zeros(rows, dt) if debug else None
    al = np.zeros(rows, dt) if debug else None
    be = np.zeros(rows, dt) if debug else None
    if alignment is not None:
        alignment = np.ascontiguousarray(alignment, dtype=np.int32)
        if alignment.ndim == 1:
            alignment = alignment.reshape(B, -1)
        astride = alignment.shape[1]
    else:
        astride = 0
    st = fn(_p(acts), _p(labels), labels.shape[1], B, _p(T), _p(S), V, blank, _p(alignment), astride, max_shift,
            blank if align_blank is None else align_blank, _p(costs), _p(g), _p(den), _p(al), _p(be), num_threads)
    if st != 0:
        raise OracleError(f"oracle status {st}")
    if debug:
        return costs, g, den, al, be
    return costs, g


def ref_rnnt(acts, labels, T, S, blank=0, alignment=None, max_shift=0, align_blank=None, precision="f64",
             grads=True, num_threads=0, debug=False):
    """The reference's own CpuRNNTComputer (oracle/_ref). Same return convention as oracle_rnnt.

    Re-packs labels with stride max(S) and the alignment with stride max(T), as the reference expects.
    """
    acts, labels, T, S = _prep(acts, labels, T, S)
    B = len(T)
    V = acts.shape[1]
    rows = int(np.sum(T.astype(np.int64) * (S.astype(np.int64) + 1)))
    smax = int(S.max())
    lab = np.ascontiguousarray(labels[:, :smax]) if smax > 0 else np.zeros((B, 1), np.int32)
    dt = np.float64 if precision == "f64" else np.float32
    fn = _load_ref().ref_rnnt_f64 if precision == "f64" else _load_ref().ref_rnnt_f32
    costs = np.zeros(B, dt)
    g = np.zeros((rows, V), dt) if grads else None
    den = np.zeros(rows, dt) if debug else None
    al = np.zeros(rows, dt) if debug else None
    be = np.zeros(rows, dt) if debug else None
    if alignment is not None:
        alignment = np.ascontiguousarray(alignment, dtype=np.int32).reshape(B, -1)
        alignment = np.ascontiguousarray(alignment[:, : int(T.max())])
    st = fn(_p(acts), _p(lab), B, _p(T), _p(S), V, blank, _p(alignment), max_shift,
            blank if align_blank is None else align_blank, _p(costs), _p(g), _p(den), _p(al), _p(be), num_threads)
    if st != 0:
        raise OracleError(f"reference status {st}")
    if debug:
        return costs, g, den, al, be
    return costs, g


def synth_acts(begin: int, count: int, seed: int = 0, normal: bool = True) -> np.ndarray:
    out = np.empty(count, np.float32)
    _load().mrnnt_oracle_synth_acts(_p(out), begin, count, seed, 1 if normal else 0)
    return out
