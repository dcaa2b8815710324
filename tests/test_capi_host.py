"""Host-side tests of the C-ABI library (no GPU needed): it loads, exports every symbol the headers in
include/ declare, and the host-only planning/validation behaves like the reference
(cpu_workspace_manager.h:99-107 / gpu_workspace_manager.h:228-239)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIB = os.path.join(ROOT, "monotonic-rnnt_amd", "libmonotonic_rnnt_amd.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "monotonic-rnnt_amd")], check=True)
    import _mrnnt_lib
    return _mrnnt_lib.load()


def _exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    dem = subprocess.run(["c++filt"], input=out, capture_output=True, text=True, check=True).stdout
    return dem


def _declared_c_functions():
    names = set()
    for h in ("mrnnt.h", "rnnt_entrypoint.h"):
        src = open(os.path.join(INC, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"\b(mrnnt_\w+|compute_rnnt_loss)\s*\(", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_c_symbol(lib):
    exported = _exported()
    declared = _declared_c_functions()
    assert "compute_rnnt_loss" in declared and "mrnnt_forward" in declared
    missing = [n for n in sorted(declared) if not re.search(r"\sT\s" + n + r"\b", exported)]
    assert not missing, missing


def test_library_exports_reference_cpp_classes(lib):
    exported = _exported()
    for method in ["GpuRNNTWorkspaceManager<float>::GpuRNNTWorkspaceManager(float const*, int const*, int, int const*, int const*, int)",
                   "GpuRNNTWorkspaceManager<float>::get_workspace_size(unsigned long*) const",
                   "GpuRNNTWorkspaceManager<float>::set_workspace(void*)",
                   "GpuRNNTWorkspaceManager<float>::create_workspace()",
                   "GpuRNNTWorkspaceManager<float>::free_workspace()",
                   "GpuRNNTWorkspaceManager<float>::restrict_to_alignment(int const*, int, int)",
                   "GpuRNNTComputer<float>::cost_and_grad(float*, float*)",
                   "GpuRNNTComputer<float>::cost(float*)",
                   "GpuRNNTComputer<float>::GpuRNNTComputer(GpuRNNTWorkspaceManager<float>&, int, ihipStream_t*)",
                   "CpuRNNTWorkspaceManager<float>::CpuRNNTWorkspaceManager(float const*, int const*, int, int const*, int const*, int)",
                   "CpuRNNTWorkspaceManager<float>::get_workspace_size(unsigned long*) const",
                   "CpuRNNTWorkspaceManager<float>::set_workspace(void*)",
                   "CpuRNNTWorkspaceManager<float>::create_workspace()",
                   "CpuRNNTWorkspaceManager<float>::free_workspace()",
                   "CpuRNNTWorkspaceManager<float>::restrict_to_alignment(int const*, int, int)",
                   "CpuRNNTComputer<float>::cost_and_grad(float*, float*)",
                   "CpuRNNTComputer<float>::cost(float*)",
                   "CpuRNNTComputer<float>::CpuRNNTComputer(CpuRNNTWorkspaceManager<float>&, int, int)"]:
        assert method in exported, method


def test_c_header_compiles_as_c():
    # the flat ABI header must be consumable from plain C (cgo / JNI / N-API stubs)
    src = '#include "mrnnt.h"\nint main(void){ mrnnt_problem p; (void)p; return (int)RNNT_STATUS_SUCCESS; }\n'
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", INC, "-x", "c", "-", "-fsyntax-only"],
                       input=src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _problem(T, S, V=8, blank=0, rows=-1):
    import _mrnnt_lib as L
    T = np.asarray(T, np.int32)
    S = np.asarray(S, np.int32)
    p = L.MrnntProblem()
    p.B, p.V, p.blank = len(T), V, blank
    p.T_host, p.S_host = T.ctypes.data, S.ctypes.data
    p.label_stride = int(S.max(initial=0))
    p.num_rows = rows
    return p, (T, S)


def test_workspace_size_and_validation(lib):
    import _mrnnt_lib as L
    n = ctypes.c_size_t(0)
    p, keep = _problem([4, 7], [2, 7])
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_SUCCESS
    rows = 4 * 3 + 7 * 8
    assert n.value >= rows * (4 + 4 * 8)  # den + lpb/lpe/alpha/beta
    for T, S in (([4], [5]), ([0], [0]), ([3], [-1])):  # T < S, T == 0, S < 0 -> INVALID_VALUE
        p, keep = _problem(T, S)
        assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
        assert b"invalid lengths" in lib.mrnnt_last_error()
    p, keep = _problem([4], [2], rows=11)  # acts rows disagree with lengths
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    p, keep = _problem([4], [2], V=3, blank=3)  # blank out of range
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    p, keep = _problem([2100], [2047])  # the largest label length the recursion covers (S + 1 = 2048)
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_SUCCESS
    p, keep = _problem([2100], [2048])
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    assert b"exceeds 2047" in lib.mrnnt_last_error()


def test_forward_rejects_bad_arguments_without_touching_gpu(lib):
    import _mrnnt_lib as L
    p, keep = _problem([4], [2])  # no device pointers -> INVALID_VALUE before any HIP call
    assert lib.mrnnt_forward(ctypes.byref(p), None, 0, None, 1, None) == L.RNNT_STATUS_INVALID_VALUE


def test_status_strings_match_reference_enum():
    src = open(os.path.join(INC, "status.h")).read()
    for name, val in (("SUCCESS", 0), ("MEMOPS_FAILED", 1), ("INVALID_VALUE", 2), ("EXECUTION_FAILED", 3),
                      ("UNKNOWN_ERROR", 4)):
        assert re.search(rf"RNNT_STATUS_{name}\s*=\s*{val}", src)


def test_torch_op_device_dispatch_checks():
    """CPU tensors run the host implementation (tests/test_cpu_parity.py); the gpu_* extension functions keep
    the reference's TORCH_CHECK that every input is a GPU tensor (monotonic_rnnt.cu:85-88)."""
    import torch
    import monotonic_rnnt_op as op
    acts = torch.zeros(12, 3)
    lab, T, S = torch.tensor([[1, 2]], dtype=torch.int32), torch.tensor([4]), torch.tensor([2])
    with pytest.raises(RuntimeError, match="GPU"):
        op.monotonic_rnnt_cpp.gpu_monotonic_rnnt(acts, lab, T, S, torch.zeros(1), torch.zeros(0), 0, 0)
    with pytest.raises(Exception):
        op.monotonic_rnnt_cpp.cpu_monotonic_rnnt(acts, None, None, None, None, None, 0, 0)
    with pytest.raises(RuntimeError, match="float32"):
        op.monotonic_rnnt_loss(acts.to(torch.bfloat16), lab, T, S)


def test_product_library_has_no_development_hooks(lib):
    """Launch knobs and bench helpers live in the development builds only (libmonotonic_rnnt_amd_dev.so,
    libmrnnt_devtools.so); the product library exports neither."""
    import _mrnnt_lib as L
    exported = _exported()
    for name in ("mrnnt_tune", "mrnnt_synth_acts", "mrnnt_copy_probe"):
        assert not re.search(r"\s" + name + r"\b", exported), name
    assert L.load_dev().mrnnt_tune(b"occ_skip", -1) == 1
    assert L.devtools().mrnnt_synth_acts
    with pytest.raises(RuntimeError, match="development build"):
        L.tune("occ_skip")
    with L.use(L.load_dev()):
        assert L.tune("occ_skip") == 1


def test_label_and_alignment_strides_validated(lib):
    """A labels / alignment row narrower than max S / max T would make the kernels read past the row."""
    import _mrnnt_lib as L
    n = ctypes.c_size_t(0)
    p, keep = _problem([4, 7], [2, 5])
    p.label_stride = 4
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    assert b"label row stride" in lib.mrnnt_last_error()
    assert lib.mrnnt_cpu_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    p.label_stride = 5
    al = np.zeros(2 * 6, np.int32)
    p.alignment, p.align_stride = al.ctypes.data, 6
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    assert b"alignment row stride" in lib.mrnnt_last_error()
    p.align_stride = 7
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_SUCCESS


@pytest.mark.parametrize("cname,pyname", [("mrnnt_problem", "MrnntProblem"),
                                          ("mrnnt_joint_problem", "MrnntJointProblem")])
def test_ctypes_problem_struct_matches_c_layout(cname, pyname):
    """The ctypes mirrors of the ABI structs have the C header's size and field offsets (checked with gcc)."""
    import _mrnnt_lib as L
    cls = getattr(L, pyname)
    fields = [f for f, _ in cls._fields_]
    body = "".join(f'printf("%zu\\n", offsetof({cname}, {f}));' for f in fields)
    src = ('#include <stddef.h>\n#include <stdio.h>\n#include "mrnnt.h"\n'
           f'int main(void){{ printf("%zu\\n", sizeof({cname})); {body} return 0; }}\n')
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "layout")
        r = subprocess.run(["gcc", "-std=c11", "-I", INC, "-x", "c", "-", "-o", exe], input=src,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        vals = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(cls)
    assert vals[1:] == [getattr(cls, f).offset for f in fields]


def test_padded_layout_and_dtype_validation(lib):
    import _mrnnt_lib as L
    n = ctypes.c_size_t(0)
    p, keep = _problem([4, 7], [2, 5])
    p.pad_T, p.pad_S1 = 7, 6
    p.num_rows = 2 * 7 * 6
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_SUCCESS
    p.pad_S1 = 5  # < max S + 1
    p.num_rows = 2 * 7 * 5
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    assert b"padded layout" in lib.mrnnt_last_error()
    p.pad_T, p.pad_S1, p.num_rows = 7, 6, 2 * 7 * 6 - 1  # wrong row count for the padded layout
    assert lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    p.num_rows = 2 * 7 * 6
    for dt, ok in ((L.MRNNT_F32, True), (L.MRNNT_BF16, True), (L.MRNNT_F16, True), (3, False), (-1, False)):
        p.acts_dtype = dt
        st = lib.mrnnt_workspace_size(ctypes.byref(p), ctypes.byref(n))
        assert (st == L.RNNT_STATUS_SUCCESS) == ok, dt


def test_joint_workspace_size_and_validation(lib):
    import _mrnnt_lib as L
    T = np.array([4, 7], np.int32)
    S = np.array([2, 5], np.int32)
    p = L.MrnntJointProblem()
    p.B, p.V, p.H, p.blank = 2, 64, 256, 0
    p.T_host, p.S_host = T.ctypes.data, S.ctypes.data
    p.enc_stride, p.pred_stride = 7 * 256, 6 * 256
    p.label_stride = 5
    n = ctypes.c_size_t(0)
    assert lib.mrnnt_joint_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_SUCCESS
    assert n.value >= (4 * 3 + 7 * 6) * (4 + 4 * 8)
    p.H = 200  # unsupported hidden size
    assert lib.mrnnt_joint_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    assert b"joint H" in lib.mrnnt_last_error()
    p.H, p.pred_stride = 256, 5 * 256  # fewer label positions than max S + 1
    assert lib.mrnnt_joint_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    p.pred_stride = 6 * 256 + 4  # not a multiple of 8
    assert lib.mrnnt_joint_workspace_size(ctypes.byref(p), ctypes.byref(n)) == L.RNNT_STATUS_INVALID_VALUE
    p.pred_stride = 6 * 256
    assert lib.mrnnt_joint_forward(ctypes.byref(p), None, 0, None, 1, None) == L.RNNT_STATUS_INVALID_VALUE
