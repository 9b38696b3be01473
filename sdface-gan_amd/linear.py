"""Training-path linear layers of the renderer MLP on split-fp16 MFMA.

When the renderer needs gradients (stage-1 training, training_utils.py:396-451)
its networks run op by op as the reference does (FiLMSiren / LinearLayer,
sdf_model.py:23-69, NGPSIRENGenerator :1566-1592): F.linear over ~196 K samples
per chunk, forward and backward.  ``linear`` routes those products to the HIP
kernels of ``csrc/linear_f16x3.hip`` (three fp16 MFMA terms per fp32 product,
fp32 accumulation, power-of-two row / column scaling: fp32-level accuracy):

  forward          out = x W^T + b             sdfr_linear_f16x3 (B = W)
  input gradient   gx  = gy W                  sdfr_linear_f16x3 (B = W^T)
  weight gradient  gW  = gy^T x                sdfr_linear_wgrad_f16x3
  bias gradient    gb  = gy.sum(0)             (torch reduction)

Shapes the kernels take: out features 256 with in features 32 / 256 / 259..288
(the networks' input_linear, dense and views layers).  Everything else (the
3- and 1-wide heads, the per-face gamma / beta layers on the styles, CPU tensors,
inference) stays on F.linear.  ``set_train_gemm("torch")`` turns the routing off.

The backward is first-order only (``once_differentiable``): SDFace-GAN never
differentiates through it twice -- the eikonal term leaves autograd inside the
grid encoder's backward (grid.py:65-89), so it carries no gradient (as in the
reference), and R1 / path-length regularisation touch only D and the decoder.
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
        x2 = x.reshape(-1, K).contiguous()
        w = weight.contiguous()
        out = _gemm(x2, _pack(w, False), bias.contiguous() if bias is not None else None, N)
        ctx.save_for_backward(x2, w)
        ctx.has_bias = bias is not None
        ctx.lead = lead
        return out.view(*lead, N)

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        N, K = w.shape
        gy2 = gy.reshape(-1, N).contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = _gemm(gy2, _pack(w, True), None, K).view(*ctx.lead, K)
        if ctx.needs_input_grad[1]:
            gw = _wgrad(gy2, x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy2.sum(0)
        return gx, gw, gb


def _routable(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if _MODE["gemm"] != "f16x3" or not x.is_cuda or not torch.is_grad_enabled():
        return False
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() < 2:
        return False
    N, K = weight.shape
    if N != 256 or K % 4 or not (K <= 32 or K == 256 or 256 < K <= 288):
        return False
    return x.numel() // K >= 1024            # the per-face gamma / beta layers stay on F.linear


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None) -> torch.Tensor:
    """F.linear(x, weight, bias), on the split-fp16 MFMA kernels for the renderer MLP's
    training shapes (module docstring), on F.linear otherwise."""
    if _routable(x, weight):
        return _LinearF16x3.apply(x, weight, bias)
    return F.linear(x, weight, bias)
