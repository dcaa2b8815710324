"""ctypes binding of libmonotonic_rnnt_amd.so (the flat C ABI in include/mrnnt.h).

There is no fallback: if the library is missing or fails to load, importing this module raises.
Build it with `python __graft_entry__.py` (or `make -C monotonic-rnnt_amd`).

Besides the product library, two development builds sit next to it (never loaded by the product path):
  libmonotonic_rnnt_amd_dev.so : the same kernels with the launch knobs exported (mrnnt_tune); load_dev(),
                                 and `with use(load_dev()):` routes this module's callers through it (tests
                                 of the launch variants, tools/kbench.py)
  libmrnnt_devtools.so         : synthetic logits and a copy probe for bench.py / tests (devtools())
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

# One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so, and a library of ours loaded before
# torch would bind the system copy first, leaving torch's device calls on a second runtime ("no ROCm-capable
# device is detected" in whichever loses). Importing torch first makes every library here share torch's.
import torch  # noqa: F401

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MRNNT_LIB_PATH: load another build of the library in place of the product -- the host-only sanitizer build
# (`make -C monotonic-rnnt_amd asan`, CPU entry points only; tests/test_sanitizers.py) or the product with its host
# orchestration sanitized (`asan-gpu`; tests/test_gpu_host_asan.py)
HOST_ONLY_PATH = os.environ.get("MRNNT_LIB_PATH") or None
LIB_PATH = HOST_ONLY_PATH or os.path.join(PKG_DIR, "libmonotonic_rnnt_amd.so")
DEV_PATH = os.path.join(PKG_DIR, "libmonotonic_rnnt_amd_dev.so")
TOOLS_PATH = os.path.join(PKG_DIR, "libmrnnt_devtools.so")

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
KERNELS = ("band", "log_softmax", "alpha_beta", "grad", "setup", "joint_fwd", "joint_bwd", "joint_reduce", "chase",
           "joint_dpre")


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
        # version 4
        ("lattice", ctypes.c_void_p),
        # version 6
        ("grad_scale_broadcast", ctypes.c_int),
        # version 7
        ("lengths_on_device", ctypes.c_int),
        ("status_host", ctypes.c_void_p),
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
        ("dbias", ctypes.c_void_p),
        # version 9
        ("reduce_scratch", ctypes.c_void_p),
        ("reduce_scratch_bytes", ctypes.c_size_t),
        # version 12
        ("live_count_dev", ctypes.c_void_p),
    ]


class MrnntError(RuntimeError):
    def __init__(self, status: int, where: str, message: str):
        self.status = status
        super().__init__(f"{where}: {STATUS_NAMES.get(status, status)} ({message})")


_lib = None
_dev = None
_tools = None
_override = None
_lock = threading.Lock()


def _bind(path: str, dev: bool = False) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(f"monotonic RNN-T library not built: {path} is missing "
                          "(run `python __graft_entry__.py` or `make -C monotonic-rnnt_amd`)")
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER(MrnntProblem)
    JP = ctypes.POINTER(MrnntJointProblem)
    vp, i, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
    sig = {
        "mrnnt_workspace_size": (i, [P, ctypes.POINTER(sz)]),
        "mrnnt_forward": (i, [P, vp, sz, vp, i, vp]),
        "mrnnt_lattice_bytes": (i, [P, ctypes.POINTER(sz)]),
        "mrnnt_lattice_host": (i, [P, vp, sz]),
        "mrnnt_backward": (i, [P, vp, vp, vp, vp]),
        "mrnnt_cost_and_grad": (i, [P, vp, sz, vp, vp, vp, vp]),
        "mrnnt_read_loglik": (i, [P, vp, vp, vp, vp]),
        "mrnnt_grad_live_rows": (i, [P, vp, vp, vp]),
        "mrnnt_read_state": (i, [P, vp, vp, vp, vp, vp]),
        "mrnnt_cpu_read_state": (i, [P, vp, vp, vp, vp]),
        "mrnnt_read_denoms": (i, [P, vp, vp, vp]),
        "mrnnt_read_band": (i, [P, vp, vp, vp, i64, vp]),
        "mrnnt_status_word": (ctypes.POINTER(ctypes.c_int), []),
        "mrnnt_cpu_workspace_size": (i, [P, ctypes.POINTER(sz)]),
        "mrnnt_cpu_forward": (i, [P, vp, sz, vp, i, i]),
        "mrnnt_cpu_backward": (i, [P, vp, vp, vp, i]),
        "mrnnt_joint_workspace_size": (i, [JP, ctypes.POINTER(sz)]),
        "mrnnt_joint_forward": (i, [JP, vp, sz, vp, i, vp]),
        "mrnnt_joint_live_rows": (i, [JP, vp, vp, vp]),
        "mrnnt_joint_backward": (i, [JP, vp, i64, vp, vp, vp, vp, vp, vp]),
        "mrnnt_joint_reduce": (i, [JP, vp, i64, vp, vp, vp, vp, vp]),
        "mrnnt_joint_reduce_pre": (i, [JP, vp, i64, vp, vp, vp, vp]),
        "mrnnt_joint_reduce_scratch_bytes": (i, [JP, ctypes.POINTER(sz)]),
        "mrnnt_joint_row_bound": (i, [JP, ctypes.POINTER(i64)]),
        "mrnnt_joint_dpre": (i, [JP, i64, vp, vp, vp, vp, vp]),
        "mrnnt_last_error": (ctypes.c_char_p, []),
        "mrnnt_version": (i, []),
        "mrnnt_fill_zero": (i, [vp, sz, vp]),
        "mrnnt_profile_enable": (None, [i]),
        "mrnnt_profile_read": (i, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64), i]),
    }
    if dev:
        sig["mrnnt_tune"] = (i, [ctypes.c_char_p, i])
        sig["mrnnt_chase_helped"] = (ctypes.c_ulonglong, [i])
        sig["mrnnt_chase_trace"] = (i, [ctypes.POINTER(ctypes.c_ulonglong), i])
        sig["mrnnt_chase_walk_trace"] = (i, [ctypes.POINTER(ctypes.c_ulonglong), i])
        sig["mrnnt_joint_trace"] = (i, [ctypes.POINTER(ctypes.c_ulonglong), i])
        sig["mrnnt_joint_reduce_trace"] = (i, [ctypes.POINTER(ctypes.c_ulonglong), i])
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None and path == HOST_ONLY_PATH and not name.startswith(("mrnnt_cpu", "mrnnt_lattice", "mrnnt_last",
                                                                          "mrnnt_version")):
            continue  # a host-only build: the GPU entry points are absent, and a call to one fails loudly
        if fn is None:
            raise ImportError(f"{path} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    if lib.mrnnt_version() < 12:
        raise ImportError(f"{path} is a stale build (ABI version {lib.mrnnt_version()} < 12); "
                          "rebuild with `make -C monotonic-rnnt_amd`")
    return lib


def load() -> ctypes.CDLL:
    """The library every call of this package goes through: the product build (or, inside `use(...)`, the
    library given there)."""
    global _lib
    if _override is not None:
        return _override
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            _lib = _bind(LIB_PATH)
        return _lib


def load_dev() -> ctypes.CDLL:
    """The development build (same kernels, launch knobs exported through mrnnt_tune)."""
    global _dev
    with _lock:
        if _dev is None:
            _dev = _bind(DEV_PATH, dev=True)
        return _dev


@contextlib.contextmanager
def use(lib: ctypes.CDLL):
    """Route load() -- hence every op of this package -- through `lib` (e.g. load_dev()) inside the block."""
    global _override
    prev = _override
    _override = lib
    try:
        yield lib
    finally:
        _override = prev


def select_dev() -> ctypes.CDLL:
    """Route this whole process through the development build (A/B tools with launch knobs; never the product)."""
    global _override
    _override = load_dev()
    return _override


def devtools() -> ctypes.CDLL:
    """libmrnnt_devtools.so: mrnnt_synth_acts / mrnnt_copy_probe / mrnnt_read_probe / mrnnt_write_probe (bench and tests only)."""
    global _tools
    with _lock:
        if _tools is None:
            if not os.path.exists(TOOLS_PATH):
                raise ImportError(f"{TOOLS_PATH} is missing (run `make -C monotonic-rnnt_amd`)")
            t = ctypes.CDLL(TOOLS_PATH)
            t.mrnnt_synth_acts.restype = ctypes.c_int
            t.mrnnt_synth_acts.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_void_p]
            t.mrnnt_copy_probe.restype = ctypes.c_int
            t.mrnnt_copy_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
            t.mrnnt_write_probe.restype = ctypes.c_int
            t.mrnnt_write_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
            t.mrnnt_read_probe.restype = ctypes.c_int
            t.mrnnt_read_probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
            t.mrnnt_dispatch_probe.restype = ctypes.c_int
            t.mrnnt_dispatch_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
            t.mrnnt_occupy.restype = ctypes.c_int
            t.mrnnt_occupy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
            _tools = t
        return _tools


def synth_acts(out_ptr: int, begin: int, count: int, seed: int, normal: bool, stream: int) -> None:
    """Fill a device fp32 buffer with the counter-based synthetic generator (devtools)."""
    rc = devtools().mrnnt_synth_acts(ctypes.c_void_p(out_ptr), begin, count, seed, 1 if normal else 0,
                                     ctypes.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"mrnnt_synth_acts failed ({rc})")


def check(status: int, where: str) -> None:
    if status != RNNT_STATUS_SUCCESS:
        msg = load().mrnnt_last_error()
        raise MrnntError(status, where, msg.decode() if msg else "")


def tune(key: str, value: int = -1) -> int:
    """Set a launch-shape knob of the current library (needs the development build: `with use(load_dev()):`);
    returns the previous value (-1 = unknown key)."""
    lib = load()
    if not hasattr(lib, "mrnnt_tune") or lib.mrnnt_tune.restype is not ctypes.c_int:
        raise RuntimeError("launch knobs need the development build: `with _mrnnt_lib.use(_mrnnt_lib.load_dev()):`")
    return lib.mrnnt_tune(key.encode(), int(value))


def library_sha256(path: str = LIB_PATH) -> str:
    """sha256 of a built library file (test logs name the product build they ran on)."""
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def source_sha256() -> str:
    """sha256 over what the product library is built from -- csrc/, include/, the Makefile (names and bytes, sorted)
    -- and the ROCm release the build uses. The Makefile's build is path-independent (-ffile-prefix-map, fixed
    -cuid), so equal sources and toolchain give an equal library; a PMC record keyed by this hash stays valid across a
    rebuild in another checkout (bench.py's roofline.traffic)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    root = os.path.dirname(PKG_DIR)
    files = sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*")) + glob.glob(os.path.join(root, "include", "*")) +
                   [os.path.join(PKG_DIR, "Makefile")])
    for f in files:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    rocm = "/opt/rocm/.info/version"
    h.update(b"rocm " + (open(rocm, "rb").read().strip() if os.path.exists(rocm) else b"unknown"))
    return h.hexdigest()


def profile_enable(on: bool = True) -> None:
    load().mrnnt_profile_enable(1 if on else 0)


def profile_read() -> dict:
    n = len(KERNELS)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    load().mrnnt_profile_read(ms, cnt, n)
    return {k: (ms[j], cnt[j]) for j, k in enumerate(KERNELS)}
