"""ctypes binding of libmonotonic_rnnt_amd.so (the flat C ABI in include/mrnnt.h).

There is no fallback: if the HIP library is missing or fails to load, importing this module raises.
Build it with `python __graft_entry__.py` (or `make -C monotonic-rnnt_amd`). MRNNT_LIB=<path> loads another
build of the same ABI instead (A/B measurements of compile-time variants, tools/); MRNNT_TUNE="key=value,..."
sets launch knobs (mrnnt_tune) at load.
"""
from __future__ import annotations

import ctypes
import os
import threading

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MRNNT_LIB") or os.path.join(PKG_DIR, "libmonotonic_rnnt_amd.so")

RNNT_STATUS_SUCCESS = 0
RNNT_STATUS_MEMOPS_FAILED = 1
RNNT_STATUS_INVALID_VALUE = 2
RNNT_STATUS_EXECUTION_FAILED = 3
RNNT_STATUS_UNKNOWN_ERROR = 4
STATUS_NAMES = {0: "no error", 1: "device memcpy or memset failed", 2: "invalid value", 3: "execution failed",
                4: "unknown error"}

# acts / grads element types (MRNNT_F32 / MRNNT_BF16 / MRNNT_F16 in include/mrnnt.h)
MRNNT_F32 = 0
MRNNT_BF16 = 1
MRNNT_F16 = 2

# kernel-family order of mrnnt_profile_read
KERNELS = ("band", "log_softmax", "alpha_beta", "grad", "setup", "joint_fwd", "joint_bwd", "joint_reduce")


class MrnntProblem(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int),
        ("V", ctypes.c_int),
        ("blank", ctypes.c_int),
        ("max_shift", ctypes.c_int),
        ("T_host", ctypes.c_void_p),
        ("S_host", ctypes.c_void_p),
        ("T_dev", ctypes.c_void_p),
        ("S_dev", ctypes.c_void_p),
        ("acts", ctypes.c_void_p),
        ("labels", ctypes.c_void_p),
        ("label_stride", ctypes.c_int64),
        ("alignment", ctypes.c_void_p),
        ("align_stride", ctypes.c_int64),
        ("align_blank", ctypes.c_int),
        ("num_rows", ctypes.c_int64),
        # version 2 (zero = the reference contract: packed fp32 acts)
        ("acts_dtype", ctypes.c_int),
        ("pad_T", ctypes.c_int64),
        ("pad_S1", ctypes.c_int64),
    ]


class MrnntJointProblem(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int),
        ("V", ctypes.c_int),
        ("H", ctypes.c_int),
        ("blank", ctypes.c_int),
        ("T_host", ctypes.c_void_p),
        ("S_host", ctypes.c_void_p),
        ("T_dev", ctypes.c_void_p),
        ("S_dev", ctypes.c_void_p),
        ("labels", ctypes.c_void_p),
        ("label_stride", ctypes.c_int64),
        ("enc", ctypes.c_void_p),
        ("enc_stride", ctypes.c_int64),
        ("pred", ctypes.c_void_p),
        ("pred_stride", ctypes.c_int64),
        ("weight", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("alignment", ctypes.c_void_p),
        ("align_stride", ctypes.c_int64),
        ("align_blank", ctypes.c_int),
        ("max_shift", ctypes.c_int),
        ("hact_ld", ctypes.c_int64),
    ]


class MrnntError(RuntimeError):
    def __init__(self, status: int, where: str, message: str):
        self.status = status
        super().__init__(f"{where}: {STATUS_NAMES.get(status, status)} ({message})")


_lib = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"monotonic RNN-T HIP library not built: {LIB_PATH} is missing "
                              "(run `python __graft_entry__.py` or `make -C monotonic-rnnt_amd`)")
        lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER(MrnntProblem)
        JP = ctypes.POINTER(MrnntJointProblem)
        vp, i, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
        sig = {
            "mrnnt_workspace_size": (i, [P, ctypes.POINTER(sz)]),
            "mrnnt_forward": (i, [P, vp, sz, vp, i, vp]),
            "mrnnt_backward": (i, [P, vp, vp, vp, vp]),
            "mrnnt_cost_and_grad": (i, [P, vp, sz, vp, vp, vp, vp]),
            "mrnnt_read_loglik": (i, [P, vp, vp, vp, vp]),
            "mrnnt_grad_live_rows": (i, [P, vp, vp, vp]),
            "mrnnt_joint_workspace_size": (i, [JP, ctypes.POINTER(sz)]),
            "mrnnt_joint_forward": (i, [JP, vp, sz, vp, i, vp]),
            "mrnnt_joint_live_rows": (i, [JP, vp, vp, vp]),
            "mrnnt_joint_backward": (i, [JP, vp, i64, vp, vp, vp, vp, vp, vp]),
            "mrnnt_joint_reduce": (i, [JP, vp, i64, vp, vp, vp, vp, vp]),
            "mrnnt_last_error": (ctypes.c_char_p, []),
            "mrnnt_version": (i, []),
            "mrnnt_profile_enable": (None, [i]),
            "mrnnt_profile_read": (i, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64), i]),
            "mrnnt_synth_acts": (i, [vp, i64, i64, ctypes.c_uint64, i, vp]),
            "mrnnt_copy_probe": (i, [vp, vp, sz, vp]),
            "mrnnt_tune": (i, [ctypes.c_char_p, i]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.mrnnt_version() < 3:
            raise ImportError(f"{LIB_PATH} is a stale build (ABI version {lib.mrnnt_version()} < 3); "
                              "rebuild with `make -C monotonic-rnnt_amd`")
        for kv in filter(None, os.environ.get("MRNNT_TUNE", "").split(",")):
            k, v = kv.split("=")
            if lib.mrnnt_tune(k.strip().encode(), int(v)) < 0:
                raise ValueError(f"MRNNT_TUNE: unknown knob {k!r}")
        _lib = lib
        return lib


def check(status: int, where: str) -> None:
    if status != RNNT_STATUS_SUCCESS:
        msg = load().mrnnt_last_error()
        raise MrnntError(status, where, msg.decode() if msg else "")


def tune(key: str, value: int = -1) -> int:
    """Set a launch-shape knob (mrnnt_tune); returns the previous value (-1 = unknown key)."""
    return load().mrnnt_tune(key.encode(), int(value))


def profile_enable(on: bool = True) -> None:
    load().mrnnt_profile_enable(1 if on else 0)


def profile_read() -> dict:
    n = len(KERNELS)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    load().mrnnt_profile_read(ms, cnt, n)
    return {k: (ms[j], cnt[j]) for j, k in enumerate(KERNELS)}
