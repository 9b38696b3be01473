"""Drop-in GridEncoder / SHEncoder on the HIP kernels of libsdfr.

Interface parity with the reference modules:
  * ``GridEncoder``  <- im2scene/sdf/models/gridencoder/grid.py:96-184
    (same constructor arguments, attributes, ``embeddings`` / ``offsets``
    state-dict entries and ``forward(inputs, bound)``);
  * ``grid_encode``  <- grid.py:24-93 (autograd Function: [L,B,C] kernel
    output permuted to [B, L*C]; optional dy_dx for input gradients);
  * ``SHEncoder`` / ``sh_encode`` <- shencoder/sphere_harmonics.py:14-86.

Device tensors only: CPU inputs raise the same "must be a CUDA tensor" error
the reference's TORCH_CHECK raises (gridencoder.cu:15, 449).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
from torch.autograd import Function

from . import _lib
from .linear import _edge, _wanted

_gridtype_to_id = {"hash": 0, "tiled": 1}
_interp_to_id = {"linear": 0, "smoothstep": 1}


def _check_cuda(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")


class _GridEncode(Function):
    @staticmethod
    def forward(ctx, inputs, embeddings, offsets, per_level_scale, base_resolution,
                calc_grad_inputs=False, gridtype=0, align_corners=False, interpolation=0):
        inputs = inputs.contiguous()
        for t, n in ((inputs, "inputs"), (embeddings, "embeddings"), (offsets, "offsets")):
            _check_cuda(t, n)
        if inputs.dtype != torch.float32 or embeddings.dtype != torch.float32:
            raise RuntimeError("sdface-gan_amd GridEncoder computes in fp32 (inputs and embeddings)")
        if offsets.dtype != torch.int32:
            raise RuntimeError("offsets must be an int tensor")
        B, D = inputs.shape
        L = offsets.shape[0] - 1
        C = embeddings.shape[1]
        S = float(np.log2(per_level_scale))
        H = int(base_resolution)
        outputs = torch.empty(L, B, C, device=inputs.device, dtype=embeddings.dtype)
        dy_dx = (torch.empty(B, L * D * C, device=inputs.device, dtype=embeddings.dtype)
                 if calc_grad_inputs else None)
        _lib.check(_lib.lib().sdfr_grid_encode_forward(
            _lib.ptr(inputs), _lib.ptr(embeddings.contiguous()), _lib.ptr(offsets.contiguous()),
            _lib.ptr(outputs), B, D, C, L, S, H, _lib.ptr(dy_dx), gridtype, int(align_corners),
            interpolation, _lib.stream_of(inputs)), "sdfr_grid_encode_forward")
        outputs = outputs.permute(1, 0, 2).reshape(B, L * C)
        ctx.save_for_backward(inputs, embeddings, offsets, dy_dx)
        ctx.dims = (B, D, C, L, S, H, gridtype, interpolation, bool(align_corners))
        ctx.table_edge = _edge(embeddings)
        return outputs

    @staticmethod
    def backward(ctx, grad):
        inputs, embeddings, offsets, dy_dx = ctx.saved_tensors
        B, D, C, L, S, H, gridtype, interpolation, align_corners = ctx.dims
        grad = grad.view(B, L, C).permute(1, 0, 2).contiguous()
        grad_inputs = torch.zeros_like(inputs, dtype=embeddings.dtype) if dy_dx is not None else None
        # a backward pass that does not use the table gradient (the eikonal term's
        # autograd.grad, which returns the points' gradient only; linear._wanted, scoped to
        # that graph task) would discard it: skip it
        skip = grad_inputs is not None and not _wanted(ctx.needs_input_grad[1], ctx.table_edge)
        grad_embeddings = None if skip else torch.zeros_like(embeddings)
        # binned table gradient (csrc/encoders.hip) in a workspace from torch's allocator
        L_ = _lib.lib()
        wsb = 0 if skip else L_.sdfr_grid_encode_backward_ws_bytes(B, D, C, L, S, H,
                                                                   int(align_corners))
        ws = torch.empty(wsb, dtype=torch.uint8, device=grad.device) if wsb else None
        _lib.check(L_.sdfr_grid_encode_backward_ws(
            _lib.ptr(grad), _lib.ptr(inputs), _lib.ptr(embeddings), _lib.ptr(offsets),
            _lib.ptr(grad_embeddings), B, D, C, L, S, H, _lib.ptr(dy_dx), _lib.ptr(grad_inputs),
            gridtype, int(align_corners), interpolation, _lib.ptr(ws), wsb, _lib.stream_of(grad)),
            "sdfr_grid_encode_backward")
        if grad_inputs is not None:
            grad_inputs = grad_inputs.to(inputs.dtype)
        return grad_inputs, grad_embeddings, None, None, None, None, None, None, None


grid_encode = _GridEncode.apply


def grid_offsets(input_dim, num_levels, base_resolution, per_level_scale, log2_hashmap_size,
                 align_corners):
    """Per-level row offsets (grid.py:117-128): min(2^log2, (res+1)^D), rounded up to 8."""
    max_params = 2 ** log2_hashmap_size
    offsets, offset = [], 0
    for i in range(num_levels):
        res = int(np.ceil(base_resolution * per_level_scale ** i))
        n = min(max_params, (res if align_corners else res + 1) ** input_dim)
        n = int(np.ceil(n / 8) * 8)
        offsets.append(offset)
        offset += n
    offsets.append(offset)
    return offsets


class GridEncoder(nn.Module):
    def __init__(self, input_dim=3, num_levels=16, level_dim=2, per_level_scale=2,
                 base_resolution=16, log2_hashmap_size=19, desired_resolution=None,
                 gridtype="hash", align_corners=False, interpolation="linear"):
        super().__init__()
        if desired_resolution is not None:
            per_level_scale = np.exp2(np.log2(desired_resolution / base_resolution) /
                                      (num_levels - 1))
        self.input_dim = input_dim
        self.num_levels = num_levels
        self.level_dim = level_dim
        self.per_level_scale = per_level_scale
        self.log2_hashmap_size = log2_hashmap_size
        self.base_resolution = base_resolution
        self.output_dim = num_levels * level_dim
        self.gridtype = gridtype
        self.gridtype_id = _gridtype_to_id[gridtype]
        self.interpolation = interpolation
        self.interp_id = _interp_to_id[interpolation]
        self.align_corners = align_corners
        self.max_params = 2 ** log2_hashmap_size
        offsets = grid_offsets(input_dim, num_levels, base_resolution, per_level_scale,
                               log2_hashmap_size, align_corners)
        self.register_buffer("offsets", torch.tensor(offsets, dtype=torch.int32))
        self.n_params = self.offsets[-1] * level_dim
        self.embeddings = nn.Parameter(torch.empty(offsets[-1], level_dim))
        self.reset_parameters()

    def reset_parameters(self):
        std = 1e-4
        self.embeddings.data.uniform_(-std, std)

    def __repr__(self):
        top = int(round(self.base_resolution * self.per_level_scale ** (self.num_levels - 1)))
        return (f"GridEncoder: input_dim={self.input_dim} num_levels={self.num_levels} "
                f"level_dim={self.level_dim} resolution={self.base_resolution} -> {top} "
                f"per_level_scale={self.per_level_scale:.4f} "
                f"params={tuple(self.embeddings.shape)} gridtype={self.gridtype} "
                f"align_corners={self.align_corners} interpolation={self.interpolation}")

    def forward(self, inputs, bound=1):
        inputs = (inputs + bound) / (2 * bound)
        prefix = list(inputs.shape[:-1])
        inputs = inputs.view(-1, self.input_dim)
        out = grid_encode(inputs, self.embeddings, self.offsets, self.per_level_scale,
                          self.base_resolution, inputs.requires_grad, self.gridtype_id,
                          self.align_corners, self.interp_id)
        return out.view(prefix + [self.output_dim])

    def grad_total_variation(self, weight=1e-7, inputs=None, bound=1, B=1000000):
        # kernel_grad_tv (gridencoder.cu:506-610) is never called by SDFace-GAN;
        # see SURVEY.md section 2.2.
        raise NotImplementedError("grad_total_variation is outside the SDFace-GAN hot path")


class _SHEncode(Function):
    @staticmethod
    def forward(ctx, inputs, degree, calc_grad_inputs=False):
        inputs = inputs.contiguous().float()
        _check_cuda(inputs, "inputs")
        B, input_dim = inputs.shape
        outputs = torch.empty(B, degree ** 2, dtype=inputs.dtype, device=inputs.device)
        dy_dx = (torch.empty(B, input_dim * degree ** 2, dtype=inputs.dtype, device=inputs.device)
                 if calc_grad_inputs else None)
        _lib.check(_lib.lib().sdfr_sh_encode_forward(
            _lib.ptr(inputs), _lib.ptr(outputs), B, input_dim, degree, _lib.ptr(dy_dx),
            _lib.stream_of(inputs)), "sdfr_sh_encode_forward")
        ctx.save_for_backward(inputs, dy_dx)
        ctx.dims = (B, input_dim, degree)
        return outputs

    @staticmethod
    def backward(ctx, grad):
        inputs, dy_dx = ctx.saved_tensors
        if dy_dx is None:
            return None, None, None
        grad = grad.contiguous()
        B, input_dim, degree = ctx.dims
        grad_inputs = torch.zeros_like(inputs)
        _lib.check(_lib.lib().sdfr_sh_encode_backward(
            _lib.ptr(grad), _lib.ptr(inputs), B, input_dim, degree, _lib.ptr(dy_dx),
            _lib.ptr(grad_inputs), _lib.stream_of(grad)), "sdfr_sh_encode_backward")
        return grad_inputs, None, None


sh_encode = _SHEncode.apply


class SHEncoder(nn.Module):
    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        self.input_dim = input_dim
        self.degree = degree
        self.output_dim = degree ** 2
        assert self.input_dim == 3, "SH encoder only support input dim == 3"
        assert 0 < self.degree <= 8, "SH encoder only supports degree in [1, 8]"

    def __repr__(self):
        return f"SHEncoder: input_dim={self.input_dim} degree={self.degree}"

    def forward(self, inputs, size=1):
        inputs = inputs / size
        prefix = list(inputs.shape[:-1])
        inputs = inputs.reshape(-1, self.input_dim)
        out = sh_encode(inputs, self.degree, inputs.requires_grad)
        return out.reshape(prefix + [self.output_dim])
