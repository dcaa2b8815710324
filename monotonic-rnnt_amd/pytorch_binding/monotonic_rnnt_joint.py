"""Fused joint network + monotonic RNN-T loss (extension).

    costs = monotonic_rnnt_joint_loss(enc, pred, weight, bias, labels, input_lengths, label_lengths, blank_label=0)

computes the loss of `monotonic_rnnt_loss(acts, ...)` for the packed logits

    acts[(b, t, s), :] = weight @ tanh(enc[b, t] + pred[b, s]) + bias      (t < T_b, s <= S_b)

without materialising them: the HIP kernels of `mrnnt_joint.hip` form each tile of logits on the matrix cores
(bf16 operands, fp32 accumulation) inside the log-softmax pass and again, for the live lattice rows only,
inside the gradient pass. Backward returns gradients for enc, pred, weight and bias: the fused kernel writes
the logit gradient G and the activations tanh(enc + pred) of the live rows (bf16); dweight = G^T Hact (split-K
batched GEMM, fp32 out; Hact carries a ones column when dbias is needed, so dbias = sum G comes out of the same
GEMM) is a library GEMM over those rows (hipBLASLt through torch); dpre = (G weight) (1 - Hact^2) is one
hand-written MFMA pass (mrnnt_joint_dpre; H = 256 / 512 -- other widths take dH from hipBLASLt and multiply in the
reduce), and mrnnt_joint_reduce folds dpre into denc (sum over s) and dpred (sum over t) in one pass.

Shapes: enc [B, T_slots >= max T, H], pred [B, S_slots >= max S + 1, H], weight [V, H] (torch.nn.Linear
layout), bias [V] or None; H in {128, 256, 384, 512, 640}. Inputs of other floating dtypes are cast to bf16
(the cast is differentiable, so their gradients come back in their own dtype). Costs are fp32 on the device.
There is no CPU or eager fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np
import torch

try:
    from . import _mrnnt_lib as _L
    from .monotonic_rnnt_op import _check_labels, _lengths
except ImportError:
    import _mrnnt_lib as _L
    from monotonic_rnnt_op import _check_labels, _lengths

_L.load()

JOINT_H = (128, 256, 384, 512, 640)


def _vp(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class _JointPrepared:
    def __init__(self, enc, pred, weight, bias, labels, input_lengths, label_lengths, blank_label, alignment=None,
                 max_shift=0):
        for name, x in (("enc", enc), ("pred", pred), ("weight", weight)):
            if not x.is_cuda:
                raise RuntimeError(f"monotonic_rnnt_joint: {name} must be a GPU tensor (no CPU implementation)")
            if x.dtype != torch.bfloat16:
                raise RuntimeError(f"monotonic_rnnt_joint: {name} must be bfloat16 here")
        if enc.dim() != 3 or pred.dim() != 3 or weight.dim() != 2:
            raise RuntimeError("monotonic_rnnt_joint: expected enc [B, T, H], pred [B, S+1, H], weight [V, H]")
        B, _, H = enc.shape
        V = weight.size(0)
        if pred.size(0) != B or pred.size(2) != H or weight.size(1) != H:
            raise RuntimeError(f"monotonic_rnnt_joint: shape mismatch enc {tuple(enc.shape)}, "
                               f"pred {tuple(pred.shape)}, weight {tuple(weight.shape)}")
        if H not in JOINT_H:
            raise RuntimeError(f"monotonic_rnnt_joint: H = {H} not supported (one of {JOINT_H})")
        dev = enc.device
        self.enc = enc.contiguous()
        self.pred = pred.contiguous()
        self.weight = weight.contiguous()
        self.bias = None if bias is None else bias.detach().to(dev, torch.float32).contiguous()
        ln = _lengths(input_lengths, label_lengths)
        self.T_host, self.S_host = ln.T, ln.S
        if self.T_host.size != B or self.S_host.size != B:
            raise RuntimeError(f"monotonic_rnnt_joint: expected {B} input/label lengths")
        if B and (self.T_host.max() > enc.size(1) or self.S_host.max() + 1 > pred.size(1)):
            raise RuntimeError("monotonic_rnnt_joint: enc/pred have fewer frames/label positions than the lengths")
        self.T_dev, self.S_dev, _ = ln.on(dev)
        if not labels.is_cuda:
            _check_labels(labels, self.S_host, V)
        lab = labels.detach().to(dev, torch.int32)
        if lab.dim() == 1:
            lab = lab.view(B, -1)
        self.labels = lab.contiguous() if lab.numel() else torch.zeros(B, 1, dtype=torch.int32, device=dev)
        p = _L.MrnntJointProblem()
        p.B, p.V, p.H, p.blank = B, V, H, int(blank_label)
        p.T_host, p.S_host = ln.T_ptr, ln.S_ptr
        p.T_dev, p.S_dev = self.T_dev.data_ptr(), self.S_dev.data_ptr()
        p.labels, p.label_stride = self.labels.data_ptr(), self.labels.size(1)
        p.enc, p.enc_stride = self.enc.data_ptr(), self.enc.size(1) * H
        p.pred, p.pred_stride = self.pred.data_ptr(), self.pred.size(1) * H
        p.weight = self.weight.data_ptr()
        p.bias = self.bias.data_ptr() if self.bias is not None else None
        self.alignment = None
        if alignment is not None:
            al = alignment.detach().to(dev, torch.int32)
            self.alignment = (al.view(B, -1) if al.dim() == 1 else al).contiguous()
            p.alignment, p.align_stride = self.alignment.data_ptr(), self.alignment.size(1)
            p.align_blank, p.max_shift = int(blank_label), int(max_shift)
        self.problem = p
        self.device = dev
        self.B, self.V, self.H = B, V, H

    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def forward(self, with_beta: bool):
        lib = _L.load()
        n = ctypes.c_size_t(0)
        _L.check(lib.mrnnt_joint_workspace_size(ctypes.byref(self.problem), ctypes.byref(n)), "joint_workspace_size")
        with torch.cuda.device(self.device):
            ws = torch.empty(max(1, n.value), dtype=torch.uint8, device=self.device)
            costs = torch.empty(self.B, dtype=torch.float32, device=self.device)
            _L.check(lib.mrnnt_joint_forward(ctypes.byref(self.problem), _vp(ws), ws.numel(), _vp(costs),
                                             1 if with_beta else 0, self.stream()), "mrnnt_joint_forward")
        return costs, ws

    def backward_rows(self, ws, grad_scale, with_index=False, bias_column=False, dbias=None, capturable=False):
        """The fused gradient pass over the live rows: (G [n, V], Hact [n, H]) and, with_index, the enc / pred
        row of each live row (bt_idx, bs_idx). bias_column: Hact is [n, _HACT_LD[H]] with column H = 1 (and zeros
        after it), so G^T Hact carries dbias = sum_i G[i] in column H (no separate pass over G).
        capturable: no device-to-host read -- n is the host-known bound on the live rows (mrnnt_joint_row_bound: the
        in-band rows), the kernels take the live count from the device (ABI v12 live_count_dev) and rows past it are
        zeros, so the step can be captured in a HIP graph; the GEMMs downstream then run over the bound."""
        lib = _L.load()
        with torch.cuda.device(self.device):
            cnt = torch.zeros(1, dtype=torch.int64, device=self.device)
            _L.check(lib.mrnnt_joint_live_rows(ctypes.byref(self.problem), _vp(ws), _vp(cnt), self.stream()),
                     "mrnnt_joint_live_rows")
            if capturable:
                nb = ctypes.c_int64(0)
                _L.check(lib.mrnnt_joint_row_bound(ctypes.byref(self.problem), ctypes.byref(nb)), "joint_row_bound")
                n = nb.value
                self.live_count = cnt  # referenced by the problem until the backward's last kernel is queued
                self.problem.live_count_dev = cnt.data_ptr()
            else:
                n = int(cnt.item())  # one 8-byte read-back sizes the row buffers
                self.problem.live_count_dev = None
            G = torch.empty(max(1, n), self.V, dtype=torch.bfloat16, device=self.device)
            ld = _HACT_LD[self.H] if bias_column else self.H
            self.problem.hact_ld = ld  # mrnnt_joint_reduce reads Hact with the same stride
            Hact = torch.empty(max(1, n), ld, dtype=torch.bfloat16, device=self.device)
            bt = bs = None
            if with_index:
                bt = torch.empty(max(1, n), dtype=torch.int64, device=self.device)
                bs = torch.empty(max(1, n), dtype=torch.int64, device=self.device)
            if grad_scale is not None:
                grad_scale = grad_scale.detach().to(self.device, torch.float32).contiguous()
            self.problem.dbias = _vp(dbias)  # the gradient pass adds sum_i G[i] into it (zeroed by the caller)
            _L.check(lib.mrnnt_joint_backward(ctypes.byref(self.problem), _vp(ws), n, _vp(grad_scale), _vp(G),
                                              _vp(Hact), _vp(bt), _vp(bs), self.stream()), "mrnnt_joint_backward")
        if with_index:
            return G[:n], Hact[:n], bt[:n], bs[:n]
        return G[:n], Hact[:n]

    def dpre(self, G, Hact):
        """dpre = (G weight) * (1 - Hact^2), bf16 [n, H], on the library's hand-written MFMA tiles (mrnnt_joint_dpre)."""
        n = G.shape[0]
        wt = self.weight.t().contiguous()  # [H, V]: k = v contiguous, as G's rows (1 MB at H = 512, V = 1024)
        out = torch.empty(max(1, n), self.H, dtype=torch.bfloat16, device=self.device)
        with torch.cuda.device(self.device):
            _L.check(_L.load().mrnnt_joint_dpre(ctypes.byref(self.problem), n, _vp(G), _vp(wt), _vp(Hact), _vp(out),
                                                self.stream()), "mrnnt_joint_dpre")
        return out[:n]

    def reduce(self, ws, dH, Hact, need_enc, need_pred, scratch=None):
        """d_enc / d_pred (fp32) from dH = G weight over the live rows (mrnnt_joint_reduce); Hact None: dH is already
        dpre (mrnnt_joint_dpre), summed by mrnnt_joint_reduce_pre. scratch: a dead device buffer (G, once dH exists) for the blocked form; a fresh one is
        allocated when it is too small."""
        d_enc = torch.zeros(self.enc.shape, dtype=torch.float32, device=self.device)
        d_pred = torch.zeros(self.pred.shape, dtype=torch.float32, device=self.device)
        need = ctypes.c_size_t(0)
        _L.check(_L.load().mrnnt_joint_reduce_scratch_bytes(ctypes.byref(self.problem), ctypes.byref(need)),
                 "joint_reduce_scratch_bytes")
        if scratch is None or scratch.numel() * scratch.element_size() < need.value:
            scratch = torch.empty(need.value, dtype=torch.uint8, device=self.device)
        self.problem.reduce_scratch = scratch.data_ptr()
        self.problem.reduce_scratch_bytes = scratch.numel() * scratch.element_size()
        with torch.cuda.device(self.device):
            if Hact is None:  # dH holds dpre (mrnnt_joint_dpre)
                _L.check(_L.load().mrnnt_joint_reduce_pre(ctypes.byref(self.problem), _vp(ws), dH.shape[0], _vp(dH),
                                                          _vp(d_enc), _vp(d_pred), self.stream()),
                         "mrnnt_joint_reduce_pre")
            else:
                _L.check(_L.load().mrnnt_joint_reduce(ctypes.byref(self.problem), _vp(ws), dH.shape[0], _vp(dH),
                                                      _vp(Hact), _vp(d_enc), _vp(d_pred), self.stream()),
                         "mrnnt_joint_reduce")
        return d_enc if need_enc else None, d_pred if need_pred else None


_BIAS_SUM = os.environ.get("MRNNT_JOINT_BIAS_SUM") == "1"
_CAPTURABLE = os.environ.get("MRNNT_JOINT_CAPTURABLE") == "1"
# dH: a library GEMM (hipBLASLt) and the reduce's own multiply by default; MRNNT_JOINT_DH=mfma takes the library's
# hand-written MFMA kernel with the tanh derivative fused (mrnnt_joint_dpre: H = 256 / 512, V % 8 == 0) -- opt-in
# while it is slower than the GEMM it replaces (6.1 vs 3.8 ms at H = 512, the reduce 2.7 -> 2.1 ms)
_DH_BLAS = os.environ.get("MRNNT_JOINT_DH", "blas") != "mfma"


def _dpre_ok(H, V):
    return not _DH_BLAS and H in (256, 512) and V % 8 == 0
# dbias source per H: the 16x16x32 gradient pass sums G's columns at H = 256, 384, 512 (measured faster than the
# ones column at 256 / 384, profiles/r03/joint/dbias/); the ones column stays at H = 128 (the pass's column sums cost
# more there) and H = 640 (32x32x16 gradient pass). MRNNT_JOINT_DBIAS=pass / column forces one (A/B).
_DBIAS_MODE = os.environ.get("MRNNT_JOINT_DBIAS", "")


def _dbias_lds_fits(H, V):
    """The gradient pass keeps one column-sum row per wave (8) beside two weight tiles and the bias row in the CU's
    160 KiB of LDS (mrnnt_joint.hip joint_dbias_lds_bytes)."""
    return 2 * 32 * H * 2 + 9 * 4 * ((V + 31) // 32 * 32) <= 160 * 1024


def _dbias_in_pass(H, V):
    if _DBIAS_MODE == "column" and H in _HACT_LD:
        return False
    if not _bwd_sums_columns(H) or not _dbias_lds_fits(H, V):
        return False
    return _DBIAS_MODE == "pass" or H >= 256


def _bwd_sums_columns(H):
    """Whether the gradient pass runs on the 16x16x32 tile, which can add sum_i G[i] into dbias: H <= 512 (the
    product library always; the development build unless its joint_bwd_mfma knob selects the 32x32x16 tile)."""
    if H > 512:
        return False
    lib = _L.load()
    if hasattr(lib, "mrnnt_tune") and lib.mrnnt_tune.restype is ctypes.c_int:
        return _L.tune("joint_bwd_mfma") == 16
    return True
# Hact row stride when it carries the dbias ones column: the widths at which hipBLASLt's split-K dW GEMM (n = 3.9 M
# live rows, V = 1024) costs least over the plain H-wide one -- some widths pick much slower kernels
# (profiles/r01/joint_bias_column_gemm.json). H = 512 keeps the separate G.sum: its cheapest wider GEMM (640) costs
# +1.3 ms against 1.5 ms for G.sum, and the wider Hact store takes the rest (joint step +0.4 ms measured).
_HACT_LD = {128: 192, 256: 288, 384: 392, 640: 656}


def _split_k_weight_grad(G, Hact, chunks=32):
    """dW = G^T Hact over n live rows (K = n, output [V, H]): split K into batched GEMMs with fp32 outputs, then
    sum (a single long-K GEMM leaves most of the chip idle)."""
    n = G.shape[0]
    m = n // chunks
    if m < 1024:
        return torch.mm(G.t(), Hact, out_dtype=torch.float32)
    head = chunks * m
    part = torch.bmm(G[:head].view(chunks, m, -1).transpose(1, 2), Hact[:head].view(chunks, m, -1),
                     out_dtype=torch.float32).sum(0)
    if head < n:
        part += torch.mm(G[head:].t(), Hact[head:], out_dtype=torch.float32)
    return part


class MonotonicRNNTJointFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc, pred, weight, bias, labels, input_lengths, label_lengths, blank_label=0, alignment=None,
                max_distance_from_alignment=0, capturable=None):
        prep = _JointPrepared(enc, pred, weight, bias, labels, input_lengths, label_lengths, blank_label, alignment,
                              max_distance_from_alignment)
        need = any(ctx.needs_input_grad[:4])
        costs, ws = prep.forward(with_beta=need)
        if need:
            # the workspace is a saved tensor: freed after the last backward, kept under retain_graph=True
            ctx.save_for_backward(enc, pred, weight, ws)
            ctx.prep = prep
            ctx.bias_dtype = None if bias is None else bias.dtype
            ctx.capturable = capturable
        return costs

    @staticmethod
    def backward(ctx, grad_costs):
        prep, ws = ctx.prep, ctx.saved_tensors[3]
        need_b = ctx.bias_dtype is not None and ctx.needs_input_grad[3]
        # dbias rides on the dweight GEMM (a ones column in Hact); MRNNT_JOINT_BIAS_SUM=1: a separate G.sum (A/B)
        in_pass = need_b and not _BIAS_SUM and _dbias_in_pass(prep.H, prep.V)
        bias_col = need_b and ctx.needs_input_grad[2] and not _BIAS_SUM and prep.H in _HACT_LD and not in_pass
        # the 16x16x32 gradient pass (H <= 512, LDS permitting) sums G's columns itself: no separate pass over G
        fused_b = (need_b and not bias_col and not _BIAS_SUM and _bwd_sums_columns(prep.H)
                   and _dbias_lds_fits(prep.H, prep.V))
        db = torch.zeros(prep.V, dtype=torch.float32, device=prep.device) if fused_b else None
        # capturable (no host read of the live-row count): asked for, MRNNT_JOINT_CAPTURABLE=1, or inside HIP-graph capture
        cap = ctx.capturable if ctx.capturable is not None else (_CAPTURABLE or torch.cuda.is_current_stream_capturing())
        G, Hact = prep.backward_rows(ws, grad_costs, bias_column=bias_col, dbias=db, capturable=cap)
        d_enc = d_pred = d_w = d_b = None
        H = prep.H
        if ctx.needs_input_grad[2]:
            dw = _split_k_weight_grad(G, Hact)  # [V, H] (+ dbias, zeros when Hact is wider)
            d_w = dw[:, :H].to(prep.weight.dtype)
            if bias_col:
                d_b = dw[:, H].to(ctx.bias_dtype)
        if fused_b:
            d_b = db.to(ctx.bias_dtype)
        elif need_b and not bias_col:
            d_b = G.sum(0, dtype=torch.float32).to(ctx.bias_dtype)
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            if _dpre_ok(H, prep.V):
                # dpre = (G W) * (1 - Hact^2) in one hand-written MFMA pass; the reduce then reads it alone
                dH, h_in = prep.dpre(G, Hact), None
            else:
                # [n, H] bf16 (hipBLASLt), with W^T stored [H, V] (1 MB copy): hipBLASLt's kernel for that layout runs
                # 3.9 vs 4.4 ms at H = 512 (profiles/r04/joint/gemm_probe.json)
                dH, h_in = G @ prep.weight.t().contiguous().t(), Hact
            # G is dead once dH exists (dweight / dbias came first): the reduce's scratch (stream-ordered after the GEMM)
            d_enc, d_pred = prep.reduce(ws, dH, h_in, ctx.needs_input_grad[0], ctx.needs_input_grad[1], scratch=G)
            del G
            d_enc = None if d_enc is None else d_enc.to(prep.enc.dtype)
            d_pred = None if d_pred is None else d_pred.to(prep.pred.dtype)
        return d_enc, d_pred, d_w, d_b, None, None, None, None, None, None, None


def monotonic_rnnt_joint_loss(enc: torch.Tensor, pred: torch.Tensor, weight: torch.Tensor,
                              bias: Optional[torch.Tensor], labels: torch.Tensor, input_lengths: torch.Tensor,
                              label_lengths: torch.Tensor, blank_label: int = 0,
                              alignment: Optional[torch.Tensor] = None,
                              max_distance_from_alignment: int = 0, capturable: Optional[bool] = None) -> torch.Tensor:
    """Monotonic RNN-T loss of the joint network tanh(enc + pred) @ weight.T + bias, fused (see module doc).
    alignment / max_distance_from_alignment restrict the paths as in monotonic_rnnt_loss. capturable: the backward
    reads no live-row count back to the host (row buffers and GEMMs sized by the in-band rows instead of the live
    ones: slower, graph-capturable); None = only inside HIP-graph capture (or MRNNT_JOINT_CAPTURABLE=1). A step
    captured with it replays bit for bit what an eager capturable=True step computes."""
    cast = lambda x: x if x is None or x.dtype == torch.bfloat16 else x.to(torch.bfloat16)  # noqa: E731
    return MonotonicRNNTJointFunction.apply(cast(enc), cast(pred), cast(weight), bias, labels, input_lengths,
                                            label_lengths, blank_label, alignment, max_distance_from_alignment,
                                            capturable)


__all__ = ["MonotonicRNNTJointFunction", "monotonic_rnnt_joint_loss"]
