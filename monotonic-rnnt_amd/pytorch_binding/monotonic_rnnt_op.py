"""PyTorch autograd surface of the MI355X monotonic RNN-T loss.

Same public names, signatures and return conventions as the reference's
pytorch_binding/monotonic_rnnt_op.py:
  MonotonicRNNTFunction.apply(acts, labels, input_lengths, label_lengths,
                              alignment=None, max_distance_from_alignment=0, blank_label=0) -> costs [B]
  monotonic_rnnt_loss(...)                    (reference :121-163)
  MonotonicRNNTLoss(blank_label=0)            (reference :166-217)
  monotonic_rnnt_cpp.gpu_monotonic_rnnt(...) / .gpu_monotonic_rnnt_align_restrict(...)
                                              (reference pybind names, monotonic_rnnt.cu:81-152)

Execution goes through the C ABI of libmonotonic_rnnt_amd.so: GPU tensors run the HIP kernels on the current
torch stream; CPU tensors run the library's own multithreaded host implementation (mrnnt_cpu_*, the
reference's cpu_monotonic_rnnt path). There is no eager-PyTorch fallback.

Behavioural differences from the reference, all deliberate:
  * forward runs the log-softmax reduce and the alpha/beta recursion; the logit gradient is produced
    in backward with dL/dcost[b] fused into the kernel (the reference writes grads in forward into a
    zeros_like(acts) and rescales them in backward: 3 extra passes over an N x V tensor, :32-36, :96-118);
  * costs are computed on the device (the reference computes into a host tensor and copies, :37, :90);
  * labels / alignment use their true row strides (the reference assumes max(S) / max(T)); strides below
    max(S) / max(T), and (for host labels) labels outside [0, V), are rejected;
  * acts without requires_grad take the cost-only path on both devices (the reference's CPU path segfaults
    writing into its empty grads tensor);
  * MonotonicRNNTLoss.forward uses self.blank_label (the reference reads a missing self.blank, :214).

Extensions beyond the reference: bf16/fp16 acts (costs stay fp32) and the padded
[B, pad_T, pad_S1, V] acts layout, both read in place by the same kernels.

Lengths on the GPU (the reference's required form, monotonic_rnnt.cu:85-88) are never read back: the launch is
planned from acts.size(0) and labels.size(1) and the lattice is built and validated on the device (ABI v7
lengths_on_device), so a step makes no host synchronisation and can be captured in a HIP graph. Lengths that fail
that validation make the call's costs and gradients NaN and are reported by the next call (or check_lengths()),
as a RuntimeError, the way an asynchronous device error surfaces; MRNNT_SYNC_LENGTH_CHECK=1 checks every call
synchronously instead. Host (CPU) lengths plan the launch exactly, uploaded once per distinct shape.
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Optional

import numpy as np
import torch

try:
    from . import _mrnnt_lib as _L
    from . import _grads_placement as _GP
except ImportError:  # imported with pytorch_binding/ on sys.path, like the reference's tests do
    import _mrnnt_lib as _L
    import _grads_placement as _GP

_L.load()  # fail loudly at import if the HIP library is missing


# acts element types the kernels read (the arithmetic is fp32/fp64 in registers whatever the type)
_ELEM = {torch.float32: _L.MRNNT_F32, torch.bfloat16: _L.MRNNT_BF16, torch.float16: _L.MRNNT_F16}


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class _Lengths:
    """int32 host copies of one (T, S) pair (the plan needs them on the host), their device copies per device,
    and the workspace sizes of that shape. Cached by content: training loops repeat shapes, so the conversions,
    the pinned staging copy and its H2D transfer are paid once per distinct shape, not per call. Entries are
    never written after creation (the kernels only read them)."""

    __slots__ = ("T", "S", "T_ptr", "S_ptr", "dev", "ws")

    def __init__(self, T: np.ndarray, S: np.ndarray):
        self.T, self.S = T, S
        self.T_ptr, self.S_ptr = T.ctypes.data, S.ctypes.data
        self.dev = {}
        self.ws = {}

    def on(self, dev: torch.device):
        """Device copies of T, S and the lattice offsets (mrnnt_lattice_host: with them the forward launches no
        setup kernel), uploaded once as one pinned non-blocking copy on the current stream (no host wait); a call
        on another stream waits for that upload through an event. Returns (T_dev, S_dev, lattice_dev)."""
        hit = self.dev.get(dev)
        stream = torch.cuda.current_stream(dev)
        if hit is None and torch.cuda.is_current_stream_capturing():
            # the upload would only be captured, not run: an eager call with these lengths before the first replay
            # would read unwritten offsets
            raise RuntimeError("monotonic_rnnt: these host lengths are first seen inside HIP-graph capture; run one "
                               "warm-up call with them before capturing, or pass the lengths as GPU tensors")
        if hit is None:
            B = self.T.size
            p = _L.MrnntProblem()
            p.B, p.T_host, p.S_host = B, self.T_ptr, self.S_ptr
            n = ctypes.c_size_t(0)
            _L.check(_L.load().mrnnt_lattice_bytes(ctypes.byref(p), ctypes.byref(n)), "lattice_bytes")
            lat_off = 8 * ((2 * B * 4 + 7) // 8)
            host = torch.empty(lat_off + n.value, dtype=torch.uint8).pin_memory()
            hv = host.numpy()
            hv[:B * 4] = self.T.view(np.uint8)
            hv[B * 4:2 * B * 4] = self.S.view(np.uint8)
            _L.check(_L.load().mrnnt_lattice_host(ctypes.byref(p), ctypes.c_void_p(host.data_ptr() + lat_off), n.value),
                     "lattice_host")
            d = host.to(dev, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            hit = self.dev[dev] = (d[:B * 4].view(torch.int32), d[B * 4:2 * B * 4].view(torch.int32), d[lat_off:],
                                   ev, stream)
        elif hit[4] != stream and not torch.cuda.is_current_stream_capturing():
            # (under HIP-graph capture the wait is skipped: torch.cuda.graph synchronises the device before
            # capture begins, so an upload issued before it has landed)
            stream.wait_event(hit[3])
        return hit[0], hit[1], hit[2]


_LEN_CACHE: "dict" = {}
_LEN_CACHE_MAX = 64


def _host_int32(t: torch.Tensor) -> np.ndarray:
    t = t.detach()
    if t.is_cuda:
        t = t.cpu()  # a sync, as the reference's cudaMemcpy of the lengths (gpu_workspace_manager.h:87-96)
    return np.ascontiguousarray(t.numpy() if t.dtype == torch.int32 else t.to(torch.int32).numpy()).reshape(-1)


def _content(t: torch.Tensor) -> bytes:
    if not t.is_cuda and t.dtype == torch.int32 and t.is_contiguous():
        return ctypes.string_at(t.data_ptr(), t.numel() * 4)  # no numpy round trip for the common case
    return _host_int32(t).tobytes()


def _lengths(input_lengths: torch.Tensor, label_lengths: torch.Tensor) -> _Lengths:
    key = (_content(input_lengths), _content(label_lengths))
    hit = _LEN_CACHE.get(key)
    if hit is None:
        hit = _Lengths(np.frombuffer(key[0], np.int32).copy(), np.frombuffer(key[1], np.int32).copy())
        if len(_LEN_CACHE) >= _LEN_CACHE_MAX:
            _LEN_CACHE.pop(next(iter(_LEN_CACHE)))
        _LEN_CACHE[key] = hit
    return hit


import os as _os

_SYNC_LENGTH_CHECK = _os.environ.get("MRNNT_SYNC_LENGTH_CHECK", "0") not in ("", "0")
_STATUS = None
_DYN_WS: "dict" = {}


def _status_word():
    """The library's host-mapped status word (mrnnt_status_word): the device stores into it when device-resident
    lengths fail validation, with no copy on the stream."""
    global _STATUS
    if _STATUS is None:
        ptr = _L.load().mrnnt_status_word()
        if not ptr:
            raise RuntimeError("monotonic_rnnt: could not allocate the host-mapped status word")
        _STATUS = ptr
    return _STATUS


def check_lengths(sync: bool = True) -> None:
    """Raise if an earlier call's GPU-resident lengths failed validation on the device (their costs and gradients
    are NaN). sync=True waits for the current device's queued work first."""
    if _STATUS is None:
        return
    if sync and torch.cuda.is_available():
        torch.cuda.synchronize()
    if _STATUS[0] != 0:
        _STATUS[0] = 0
        raise _L.MrnntError(_L.RNNT_STATUS_INVALID_VALUE, "monotonic_rnnt",
                            "GPU-resident lengths of an earlier call failed validation on the device: need "
                            "T_b > 0, 0 <= S_b <= T_b, S_b <= labels.size(1), sum_b T_b (S_b+1) == acts.size(0) "
                            "(padded acts: T_b <= size(1), S_b < size(2)), T_b <= alignment.size(1); that call's "
                            "costs and gradients are NaN")


def _device_lengths(t: torch.Tensor, dev: torch.device, B: int, what: str) -> torch.Tensor:
    t = t.detach()
    if t.device != dev or t.dtype != torch.int32:
        t = t.to(dev, torch.int32, non_blocking=True)
    t = t.reshape(-1).contiguous()
    if t.numel() != B:
        raise RuntimeError(f"monotonic_rnnt: expected {B} {what}, got {t.numel()}")
    return t


class _Prepared:
    """Views of one call's inputs on the device they live on, plus the filled mrnnt_problem.

    GPU acts: device lengths / labels / alignment (host lengths plan the launch). CPU acts: every pointer on
    the host (the mrnnt_cpu_* entry points)."""

    def __init__(self, acts, labels, input_lengths, label_lengths, alignment, max_shift, blank_label,
                 num_threads=0):
        if acts.dtype not in _ELEM:
            raise RuntimeError("monotonic_rnnt: acts must be float32 (reference monotonic_rnnt.cu:19,84), "
                               f"or bfloat16 / float16 (extension, GPU only); got {acts.dtype}")
        if acts.dim() not in (2, 4):
            raise RuntimeError("monotonic_rnnt: acts must be packed 2-D [sum_b T_b (S_b+1), V] "
                               "or padded 4-D [B, max_T, max_S+1, V]")
        self.on_gpu = acts.is_cuda
        if not self.on_gpu and acts.dtype != torch.float32:
            raise RuntimeError(f"monotonic_rnnt: the CPU implementation takes float32 acts, got {acts.dtype}")
        dev = acts.device
        self.acts = acts.contiguous()
        self.num_threads = int(num_threads)
        B = labels.size(0)
        # GPU acts with GPU lengths: planned without reading the lengths back (ABI v7 lengths_on_device)
        self.dyn = self.on_gpu and (input_lengths.is_cuda or label_lengths.is_cuda)
        if self.dyn:
            self.lengths = ln = None
            self.T_host = self.S_host = None
            self.T_dev = _device_lengths(input_lengths, dev, B, "input lengths")
            self.S_dev = _device_lengths(label_lengths, dev, B, "label lengths")
        else:
            self.lengths = ln = _lengths(input_lengths, label_lengths)
            self.T_host, self.S_host = ln.T, ln.S
            if self.T_host.size != B or self.S_host.size != B:
                raise RuntimeError(f"monotonic_rnnt: expected {B} input/label lengths, "
                                   f"got {self.T_host.size}/{self.S_host.size}")
        lab = labels.detach()
        if lab.device != dev or lab.dtype != torch.int32:
            lab = lab.to(dev, torch.int32)
        if lab.dim() == 1:
            lab = lab.view(B, -1)
        self.labels = lab.contiguous() if lab.numel() else torch.zeros(B, 1, dtype=torch.int32, device=dev)
        self.lattice = None
        if self.on_gpu and not self.dyn:
            self.T_dev, self.S_dev, self.lattice = ln.on(dev)
        if self.on_gpu and not labels.is_cuda and not self.dyn:
            _check_labels(labels, self.S_host, acts.size(-1))
        self.alignment = None
        if alignment is not None:
            al = alignment.detach().to(dev, torch.int32)
            self.alignment = (al.view(B, -1) if al.dim() == 1 else al).contiguous()
        p = _L.MrnntProblem()
        p.B = B
        p.V = self.acts.size(-1)
        p.blank = int(blank_label)
        p.max_shift = int(max_shift)
        if self.dyn:
            p.lengths_on_device = 1
            # (first allocated outside graph capture; a capture that comes first fails closed without the report)
            if _STATUS is not None or not torch.cuda.is_current_stream_capturing():
                p.status_host = ctypes.cast(_status_word(), ctypes.c_void_p).value
        else:
            p.T_host = ln.T_ptr
            p.S_host = ln.S_ptr
        if self.on_gpu:
            p.T_dev = self.T_dev.data_ptr()
            p.S_dev = self.S_dev.data_ptr()
            p.lattice = self.lattice.data_ptr() if self.lattice is not None else None
        p.acts = self.acts.data_ptr()
        p.labels = self.labels.data_ptr()
        p.label_stride = self.labels.size(1)
        p.alignment = self.alignment.data_ptr() if self.alignment is not None else None
        p.align_stride = self.alignment.size(1) if self.alignment is not None else 0
        p.align_blank = int(blank_label)  # the reference parses the alignment with the same blank (monotonic_rnnt.cu:144)
        p.acts_dtype = _ELEM[self.acts.dtype]
        if self.acts.dim() == 4:
            if self.acts.size(0) != B:
                raise RuntimeError(f"monotonic_rnnt: padded acts has {self.acts.size(0)} utterances, labels {B}")
            p.pad_T, p.pad_S1 = self.acts.size(1), self.acts.size(2)
            p.num_rows = B * p.pad_T * p.pad_S1
        else:
            p.num_rows = self.acts.size(0)
        self.problem = p
        self.device = dev

    def workspace(self) -> torch.Tensor:
        p = self.problem
        # the plan also depends on V and the acts element type (whether the chase launch applies, and so whether the
        # workspace holds its ready flags) and on the device (its CU count bounds the chase)
        key = (self.on_gpu, self.alignment is not None, _L.load(), p.V, p.acts_dtype, str(self.device), p.pad_T,
               p.pad_S1)
        if self.dyn:  # sized from bounds: the shapes of acts and labels
            key = key + (p.B, p.num_rows, p.label_stride)
            cache = _DYN_WS
        else:
            cache = self.lengths.ws  # with the key above, a function of the lengths
        n = cache.get(key)
        if n is None:
            c = ctypes.c_size_t(0)
            if self.on_gpu:  # the plan reads the CU count of the CURRENT device: make it this call's
                with _on_device(self.device):
                    _L.check(_L.load().mrnnt_workspace_size(ctypes.byref(self.problem), ctypes.byref(c)),
                             "workspace_size")
            else:
                _L.check(_L.load().mrnnt_cpu_workspace_size(ctypes.byref(self.problem), ctypes.byref(c)),
                         "workspace_size")
            n = cache[key] = max(1, c.value)
            if self.dyn and len(_DYN_WS) > 256:
                _DYN_WS.clear()
        return torch.empty(n, dtype=torch.uint8, device=self.device)

    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)


def _check_labels(labels: torch.Tensor, S_host: np.ndarray, V: int) -> None:
    """Host labels: every label inside the lattice (s < S_b) must be in [0, V). (Device labels are not read back;
    the kernels never index past a row with them, and an out-of-range label yields a non-finite cost.)"""
    lab = labels.detach().to(torch.int32).numpy()
    lab = lab.reshape(len(S_host), -1) if lab.size else lab.reshape(len(S_host), 0)
    if lab.shape[1] < int(S_host.max(initial=0)):
        return  # the stride check in the library reports this
    mask = np.arange(lab.shape[1])[None, :] < S_host[:, None]
    bad = mask & ((lab < 0) | (lab >= V))
    if bad.any():
        b, s = map(int, np.argwhere(bad)[0])
        raise _L.MrnntError(_L.RNNT_STATUS_INVALID_VALUE, "monotonic_rnnt",
                            f"label {int(lab[b, s])} at ({b}, {s}) outside [0, V = {V})")


_NULL_CTX = contextlib.nullcontext()


def _on_device(dev: torch.device):
    """torch.cuda.device(dev) only when dev is not already current (the context manager costs microseconds)."""
    return _NULL_CTX if torch.cuda.current_device() == dev.index else torch.cuda.device(dev)


def _forward(prep: _Prepared, with_beta: bool):
    lib = _L.load()
    ws = prep.workspace()
    costs = torch.empty(prep.problem.B, dtype=torch.float32, device=prep.device)
    if not prep.on_gpu:
        _L.check(lib.mrnnt_cpu_forward(ctypes.byref(prep.problem), _ptr(ws), ws.numel(), _ptr(costs),
                                       1 if with_beta else 0, prep.num_threads), "mrnnt_cpu_forward")
        return costs, ws
    if prep.dyn:
        check_lengths(sync=False)  # an earlier call's failed validation surfaces here (no wait)
    with _on_device(prep.device):  # kernels go to this device's current stream
        _L.check(lib.mrnnt_forward(ctypes.byref(prep.problem), _ptr(ws), ws.numel(), _ptr(costs),
                                   1 if with_beta else 0, prep.stream()), "mrnnt_forward")
        if prep.dyn and _SYNC_LENGTH_CHECK and not torch.cuda.is_current_stream_capturing():
            torch.cuda.current_stream(prep.device).synchronize()
            check_lengths(sync=False)
    return costs, ws


def _backward(prep: _Prepared, ws: torch.Tensor, grad_scale: Optional[torch.Tensor],
              grads: Optional[torch.Tensor] = None) -> torch.Tensor:
    if grads is None:  # large GPU gradients: a fast-writing buffer, kept across calls (_grads_placement)
        grads = _GP.grads_like(prep.acts) if prep.on_gpu else torch.empty_like(prep.acts)
    prep.problem.grad_scale_broadcast = 0
    if grad_scale is not None:
        grad_scale = grad_scale.detach()
        if (grad_scale.dim() == 1 and grad_scale.numel() > 1 and grad_scale.stride(0) == 0
                and grad_scale.dtype == torch.float32 and grad_scale.device == prep.device):
            # the backward of costs.sum() / .mean(): one value expanded over B -- read it in place (ABI v6)
            # instead of materialising the [B] vector (a copy kernel per step)
            prep.problem.grad_scale_broadcast = 1
        else:
            grad_scale = grad_scale.to(prep.device, torch.float32).contiguous()
    if not prep.on_gpu:
        _L.check(_L.load().mrnnt_cpu_backward(ctypes.byref(prep.problem), _ptr(ws), _ptr(grad_scale), _ptr(grads),
                                              prep.num_threads), "mrnnt_cpu_backward")
        return grads
    with _on_device(prep.device):
        _L.check(_L.load().mrnnt_backward(ctypes.byref(prep.problem), _ptr(ws), _ptr(grad_scale), _ptr(grads),
                                          prep.stream()), "mrnnt_backward")
    return grads


class MonotonicRNNTFunction(torch.autograd.Function):
    """reference pytorch_binding/monotonic_rnnt_op.py:18-118"""

    @staticmethod
    def forward(ctx, acts: torch.Tensor, labels: torch.Tensor, input_lengths: torch.Tensor,
                label_lengths: torch.Tensor, alignment: Optional[torch.Tensor] = None,
                max_distance_from_alignment: int = 0, blank_label: int = 0) -> torch.Tensor:
        prep = _Prepared(acts, labels, input_lengths, label_lengths, alignment, max_distance_from_alignment,
                         blank_label)
        need_grad = bool(ctx.needs_input_grad[0])
        costs, ws = _forward(prep, with_beta=need_grad)
        if need_grad:
            # acts is re-read by the gradient kernel (saving it lets autograd catch in-place edits); the workspace
            # (den / lp / alpha / beta) is a saved tensor too, so autograd frees it after the last backward and
            # keeps it for another one under retain_graph=True (the reference saves its grads, :92)
            ctx.save_for_backward(acts, ws)
            ctx.prep = prep
        return costs

    @staticmethod
    def backward(ctx, grad_outputs):
        _, ws = ctx.saved_tensors
        grads = _backward(ctx.prep, ws, grad_outputs)
        return grads, None, None, None, None, None, None


def monotonic_rnnt_loss(acts: torch.Tensor, labels: torch.Tensor, input_lengths: torch.Tensor,
                        label_lengths: torch.Tensor, alignment: Optional[torch.Tensor] = None,
                        max_distance_from_alignment: int = 0, blank_label: int = 0) -> torch.Tensor:
    """Computes the monotonic RNN-T loss between a sequence of activations and a ground truth labeling.

    Args (reference monotonic_rnnt_op.py:130-160):
        acts:           packed 2-D float32 tensor of logits (GPU: HIP kernels; CPU: host implementation), (sum_b T_b*(S_b+1), V), utterance b
                        contiguous, then t-major, then s. Softmax is applied internally.
                        Extensions (GPU): bfloat16 / float16 elements (fp32 math; grads in the same type), and
                        the padded 4-D joint-network layout [B, pad_T >= max T, pad_S1 >= max S + 1, V]
                        read in place (no packing copy; grads of padding rows are 0).
        labels:         2-D int tensor [B, max_b S_b] of padded label sequences.
        input_lengths:  1-D int tensor [B] of T_b.
        label_lengths:  1-D int tensor [B] of S_b.
        alignment:      optional [B, max_b T_b] int tensor; restricts paths to within
                        max_distance_from_alignment frames of it.
        blank_label:    index of the blank symbol.
    Returns:
        1-D float tensor [B] of costs (negative log probabilities) on acts.device.
    """
    result = MonotonicRNNTFunction.apply(acts, labels, input_lengths, label_lengths, alignment,
                                         max_distance_from_alignment, blank_label)
    assert result is not None
    return result


class MonotonicRNNTLoss(torch.nn.Module):
    """reference monotonic_rnnt_op.py:166-217 (with the self.blank -> self.blank_label fix)."""

    def __init__(self, blank_label: int = 0) -> None:
        super().__init__()
        self.blank_label = blank_label
        self.loss = MonotonicRNNTFunction.apply

    def forward(self, acts: torch.Tensor, labels: torch.Tensor, input_lengths: torch.Tensor,
                label_lengths: torch.Tensor, alignment: Optional[torch.Tensor] = None,
                max_distance_from_alignment: int = 0) -> torch.Tensor:
        loss = self.loss(acts, labels, input_lengths, label_lengths, alignment, max_distance_from_alignment,
                         self.blank_label)
        assert loss is not None
        return loss


class _Ext:
    """The reference's pybind extension functions (monotonic_rnnt.cu:155-164), same argument order.

    gpu_*: acts on the GPU (the reference's TORCH_CHECK, :85; labels / lengths may be host or device tensors,
    the reference requires device ones); costs may live on any device (the reference takes a host tensor);
    grads [N, V] on the GPU, an empty tensor = cost only.
    cpu_*: every tensor on the host (the reference's cpu_monotonic_rnnt, :16-77); num_threads > 0 sets the
    thread count of the call. grads may also be acts itself (gradient written in place over the logits).
    Return 0 (RNNT_STATUS_SUCCESS) or raise RuntimeError.
    """

    @staticmethod
    def _run(acts, labels, input_lengths, label_lengths, alignment, k, costs, grads, blank_label, num_threads,
             want_gpu):
        if acts.is_cuda != want_gpu:  # labels / lengths may live on either device (copied as needed)
            raise RuntimeError(f"{'gpu' if want_gpu else 'cpu'}_monotonic_rnnt: acts must be a "
                               f"{'GPU' if want_gpu else 'CPU'} tensor")
        prep = _Prepared(acts, labels, input_lengths, label_lengths, alignment, k, blank_label, num_threads)
        want = grads is not None and grads.numel() > 0
        if want:
            if grads.device != prep.device or grads.dtype != prep.acts.dtype or not grads.is_contiguous():
                raise RuntimeError(f"grads must be a contiguous {prep.acts.dtype} tensor on {prep.device}")
            if grads.shape != prep.acts.shape:
                raise RuntimeError(f"grads must have the shape of acts {tuple(prep.acts.shape)}")
        c, ws = _forward(prep, with_beta=want)
        if want:
            _backward(prep, ws, None, grads)
        costs.copy_(c)
        return _L.RNNT_STATUS_SUCCESS

    def gpu_monotonic_rnnt(self, acts, labels, input_lengths, label_lengths, costs, grads, blank_label,
                           num_threads=0):
        return self._run(acts, labels, input_lengths, label_lengths, None, 0, costs, grads, blank_label, 0, True)

    def gpu_monotonic_rnnt_align_restrict(self, acts, labels, input_lengths, label_lengths, alignment,
                                          max_distance_from_alignment, costs, grads, blank_label, num_threads=0):
        return self._run(acts, labels, input_lengths, label_lengths, alignment, max_distance_from_alignment,
                         costs, grads, blank_label, 0, True)

    def cpu_monotonic_rnnt(self, acts, labels, input_lengths, label_lengths, costs, grads, blank_label,
                           num_threads=0):
        return self._run(acts, labels, input_lengths, label_lengths, None, 0, costs, grads, blank_label,
                         num_threads, False)

    def cpu_monotonic_rnnt_align_restrict(self, acts, labels, input_lengths, label_lengths, alignment,
                                          max_distance_from_alignment, costs, grads, blank_label, num_threads=0):
        return self._run(acts, labels, input_lengths, label_lengths, alignment, max_distance_from_alignment,
                         costs, grads, blank_label, num_threads, False)


monotonic_rnnt_cpp = _Ext()

__all__ = ["MonotonicRNNTFunction", "monotonic_rnnt_loss", "MonotonicRNNTLoss", "monotonic_rnnt_cpp", "check_lengths"]
