"""Training-path linear layers of the renderer MLP on split-fp16 MFMA.

When the renderer needs gradients (stage-1 training, training_utils.py:396-451)
its networks run op by op as the reference does (FiLMSiren / LinearLayer,
sdf_model.py:23-69, NGPSIRENGenerator :1566-1592): F.linear over ~196 K samples
per chunk, forward and backward.  ``linear`` routes those products to the HIP
kernels of ``csrc/linear_f16x3.hip`` (three fp16 MFMA terms per fp32 product,
fp32 accumulation, power-of-two row / column scaling: fp32-level accuracy):

  FiLM forward     s = sin(g (x W^T + b) + be) sdfr_film_linear_f16x3 (GEMM + epilogue)
  FiLM backward    dy, dg, dbe, db             sdfr_film_backward (one elementwise pass)
  forward          out = x W^T + b             sdfr_linear_f16x3 (B = W)
  input gradient   gx  = gy W                  sdfr_linear_f16x3 (B = W^T)
  weight gradient  gW  = gy^T x                sdfr_linear_wgrad_f16x3
  bias gradient    gb  = gy.sum(0)             (torch reduction)
  narrow heads     J <= 4 outputs (sigma 1, rgb 3): sdfr_linear_head_forward / _backward
                   (HBM-streaming fp32 FMA kernels in place of rocBLAS's N = 1..3 GEMMs)

Shapes the kernels take: out features 256 with in features 32 / 256 / 259..288
(the networks' input_linear, dense and views layers), and J <= 4 outputs with K <= 256
(the 3- and 1-wide heads).  Everything else (the per-face gamma / beta layers on the
styles, CPU tensors, inference) stays on F.linear.  ``set_train_gemm("torch")`` turns
the routing off.

The backward is first-order only (``once_differentiable``), so only the ngp network
routes here (``NGPSIRENGenerator`` marks its layers ``train_kernels = True``): its
eikonal term leaves autograd inside the grid encoder's backward (grid.py:65-89) and
carries no gradient (as in the reference), so nothing differentiates these ops twice.
The SIREN network's eikonal loss does reach its weights through a double backward
(the points feed the MLP directly), so SirenGenerator keeps F.linear.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.autograd.function import once_differentiable

from . import _lib

_MODE = {"gemm": "f16x3"}


def set_train_gemm(mode: str) -> None:
    """'f16x3' (default): renderer-MLP training GEMMs on the HIP kernels; 'torch':
    F.linear (rocBLAS fp32)."""
    if mode not in ("f16x3", "torch"):
        raise ValueError(f"train gemm must be 'f16x3' or 'torch', got {mode!r}")
    _MODE["gemm"] = mode


def train_gemm() -> str:
    return _MODE["gemm"]


def _pack(w: torch.Tensor, transposed: bool) -> torch.Tensor:
    """Split-fp16 fragments + row scales of B = w (or w^T) for sdfr_linear_f16x3."""
    L = _lib.lib()
    N, K = (w.shape[1], w.shape[0]) if transposed else (w.shape[0], w.shape[1])
    buf = torch.empty(L.sdfr_linear_pack_bytes(N, K), dtype=torch.uint8, device=w.device)
    _lib.check(L.sdfr_linear_pack(_lib.ptr(w), N, K, int(transposed), _lib.ptr(buf),
                                  _lib.stream_of(w)), "sdfr_linear_pack")
    return buf


def _a16(t):
    """t, or a 16-B aligned copy (the kernels read bias / gamma / beta as 16-B vectors)."""
    if t is None:
        return None
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _gemm(x2: torch.Tensor, packed: torch.Tensor, bias, N: int) -> torch.Tensor:
    M, K = x2.shape
    out = torch.empty(M, N, device=x2.device, dtype=torch.float32)
    _lib.check(_lib.lib().sdfr_linear_f16x3(_lib.ptr(out), _lib.ptr(x2), _lib.ptr(packed),
                                            _lib.ptr(bias), M, N, K, _lib.stream_of(x2)),
               "sdfr_linear_f16x3")
    return out


def _wgrad(gy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    L = _lib.lib()
    M, N = gy2.shape
    K = x2.shape[1]
    nws = L.sdfr_linear_wgrad_ws_bytes(M, N, K)
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=gy2.device)
    gw = torch.empty(N, K, device=gy2.device, dtype=torch.float32)
    _lib.check(L.sdfr_linear_wgrad_f16x3(_lib.ptr(gw), _lib.ptr(gy2), _lib.ptr(x2), M, N, K,
                                         _lib.ptr(ws), nws, _lib.stream_of(gy2)),
               "sdfr_linear_wgrad_f16x3")
    return gw


class _LinearF16x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        N, K = weight.shape
        lead = x.shape[:-1]
        x2 = _a16(x.reshape(-1, K))
        w = weight.contiguous()
        out = _gemm(x2, _pack(w, False), _a16(bias), N)
        ctx.save_for_backward(x2, w)
        ctx.has_bias = bias is not None
        ctx.lead = lead
        return out.view(*lead, N)

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        N, K = w.shape
        gy2 = _a16(gy.reshape(-1, N))
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = _gemm(gy2, _pack(w, True), None, K).view(*ctx.lead, K)
        if ctx.needs_input_grad[1]:
            gw = _wgrad(gy2, x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy2.sum(0)
        return gx, gw, gb


class _FiLMLinearF16x3(torch.autograd.Function):
    """sin(gamma[f] * (x W^T + b) + beta[f]) over F faces of equal row count: the GEMM
    with the FiLM activation in its epilogue (y = x W^T + b saved), and a backward whose
    elementwise part is one HIP kernel (dy, dgamma, dbeta, db) before the two GEMMs."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta):
        N, K = weight.shape
        F_ = gamma.shape[0]
        lead = x.shape[:-1]
        x2 = _a16(x.reshape(-1, K))
        M = x2.shape[0]
        w = weight.contiguous()
        g2, b2 = _a16(gamma.reshape(F_, N)), _a16(beta.reshape(F_, N))
        out = torch.empty(M, N, device=x.device, dtype=torch.float32)
        y = torch.empty(M, N, device=x.device, dtype=torch.float32)
        _lib.check(_lib.lib().sdfr_film_linear_f16x3(
            _lib.ptr(out), _lib.ptr(y), _lib.ptr(x2), _lib.ptr(_pack(w, False)),
            _lib.ptr(_a16(bias)), _lib.ptr(g2),
            _lib.ptr(b2), M, N, K, M // F_, _lib.stream_of(x2)), "sdfr_film_linear_f16x3")
        ctx.save_for_backward(x2, w, y, g2, b2)
        ctx.meta = (lead, bias is not None, gamma.shape, beta.shape)
        return out.view(*lead, N)

    @staticmethod
    @once_differentiable
    def backward(ctx, ds):
        x2, w, y, g2, b2 = ctx.saved_tensors
        lead, has_bias, gshape, bshape = ctx.meta
        N, K = w.shape
        M, F_ = x2.shape[0], g2.shape[0]
        ds2 = _a16(ds.reshape(-1, N))
        L = _lib.lib()
        dy = torch.empty(M, N, device=ds.device, dtype=torch.float32)
        dg = torch.empty(F_, N, device=ds.device, dtype=torch.float32)
        db_ = torch.empty(F_, N, device=ds.device, dtype=torch.float32)
        dbf = torch.empty(F_, N, device=ds.device, dtype=torch.float32)
        nws = L.sdfr_film_backward_ws_bytes(M, N, M // F_)
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=ds.device)
        _lib.check(L.sdfr_film_backward(
            _lib.ptr(dy), _lib.ptr(dg), _lib.ptr(db_), _lib.ptr(dbf), _lib.ptr(ds2), _lib.ptr(y),
            _lib.ptr(g2), _lib.ptr(b2), M, N, M // F_, _lib.ptr(ws), nws, _lib.stream_of(ds2)),
            "sdfr_film_backward")
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = _gemm(dy, _pack(w, True), None, K).view(*lead, K)
        if ctx.needs_input_grad[1]:
            gw = _wgrad(dy, x2)
        if has_bias and ctx.needs_input_grad[2]:
            gb = dbf.sum(0)
        gg = dg.view(gshape) if ctx.needs_input_grad[3] else None
        gbt = db_.view(bshape) if ctx.needs_input_grad[4] else None
        return gx, gw, gb, gg, gbt


class _LinearHead(torch.autograd.Function):
    """x W^T + b for the narrow heads (J <= 4 outputs): HBM-streaming HIP kernels."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        J, K = weight.shape
        lead = x.shape[:-1]
        x2 = _a16(x.reshape(-1, K))
        w = _a16(weight)
        M = x2.shape[0]
        out = torch.empty(M, J, device=x.device, dtype=torch.float32)
        _lib.check(_lib.lib().sdfr_linear_head_forward(
            _lib.ptr(out), _lib.ptr(x2), _lib.ptr(w), _lib.ptr(bias.contiguous() if bias is not None
                                                               else None),
            M, J, K, _lib.stream_of(x2)), "sdfr_linear_head_forward")
        ctx.save_for_backward(x2, w)
        ctx.has_bias = bias is not None
        ctx.lead = lead
        return out.view(*lead, J)

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        J, K = w.shape
        M = x2.shape[0]
        gy2 = gy.reshape(-1, J).contiguous()
        L = _lib.lib()
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        gx = torch.empty(M, K, device=gy.device, dtype=torch.float32) if need_x else None
        gw = torch.empty(J, K, device=gy.device, dtype=torch.float32) if need_w else None
        gb = torch.empty(J, device=gy.device, dtype=torch.float32) if need_b else None
        nws = L.sdfr_linear_head_ws_bytes(M, J, K) if (need_w or need_b) else 0
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=gy.device)
        _lib.check(L.sdfr_linear_head_backward(
            _lib.ptr(gx), _lib.ptr(gw), _lib.ptr(gb), _lib.ptr(gy2), _lib.ptr(x2), _lib.ptr(w),
            M, J, K, _lib.ptr(ws), nws, _lib.stream_of(gy2)), "sdfr_linear_head_backward")
        return (gx.view(*ctx.lead, K) if gx is not None else None), gw, gb


def film_linear(x, weight, bias, gamma, beta, kernels=True):
    """FiLMSiren's ``sin(gamma * F.linear(x, weight, bias) + beta)`` (sdf_model.py:62-67),
    gamma / beta [F, 1, ..., 1, N] broadcast over each face's samples: fused on the HIP
    kernels for the renderer MLP's training shapes (and ``kernels``), the reference's
    ops otherwise."""
    F_ = gamma.shape[0]
    if (kernels and _routable(x, weight) and x.shape[0] == F_ and gamma.shape[-1] == weight.shape[0]
            and gamma.numel() == F_ * weight.shape[0] and beta.shape == gamma.shape
            and weight.shape[1] > 32):
        return _FiLMLinearF16x3.apply(x, weight, bias, gamma, beta)
    return torch.sin(gamma * linear(x, weight, bias, kernels) + beta)


def _routable(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if _MODE["gemm"] != "f16x3" or not x.is_cuda or not torch.is_grad_enabled():
        return False
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() < 2:
        return False
    N, K = weight.shape
    if N != 256 or K % 4 or not (K <= 32 or K == 256 or 256 < K <= 288):
        return False
    return x.numel() // K >= 1024            # the per-face gamma / beta layers stay on F.linear


def _head_routable(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if _MODE["gemm"] != "f16x3" or not x.is_cuda or not torch.is_grad_enabled():
        return False
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() < 2:
        return False
    J, K = weight.shape
    return J <= 4 and K % 4 == 0 and K <= 256 and x.numel() // K >= 1024


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None, kernels=True) -> torch.Tensor:
    """F.linear(x, weight, bias), on the split-fp16 MFMA kernels for the renderer MLP's
    training shapes (module docstring) or the narrow-head kernels when ``kernels``, on
    F.linear otherwise."""
    if kernels and _routable(x, weight):
        return _LinearF16x3.apply(x, weight, bias)
    if kernels and _head_routable(x, weight):
        return _LinearHead.apply(x, weight, bias)
    return F.linear(x, weight, bias)
