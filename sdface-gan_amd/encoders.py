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

from . import ops  # noqa: F401  (registers torch.ops.sdfr.*)
from .linear import _edge, _wanted

_gridtype_to_id = {"hash": 0, "tiled": 1}
_interp_to_id = {"linear": 0, "smoothstep": 1}


class _GridEncode(Function):
    """grid.py:27-93 over torch.ops.sdfr.grid_encode_forward / _backward (ops.py)."""
    @staticmethod
    def forward(ctx, inputs, embeddings, offsets, per_level_scale, base_resolution,
                calc_grad_inputs=False, gridtype=0, align_corners=False, interpolation=0):
        inputs = inputs.contiguous()
        B = inputs.shape[0]
        L = offsets.shape[0] - 1
        C = embeddings.shape[1]
        S = float(np.log2(per_level_scale))
        H = int(base_resolution)
        outputs, dy_dx = torch.ops.sdfr.grid_encode_forward(
            inputs, embeddings, offsets, S, H, bool(calc_grad_inputs), int(gridtype),
            bool(align_corners), int(interpolation))
        outputs = outputs.permute(1, 0, 2).reshape(B, L * C)
        ctx.save_for_backward(inputs, embeddings, offsets, dy_dx)
        ctx.dims = (B, C, L, S, H, gridtype, interpolation, bool(align_corners))
        ctx.table_edge = _edge(embeddings)
        return outputs

    @staticmethod
    def backward(ctx, grad):
        inputs, embeddings, offsets, dy_dx = ctx.saved_tensors
        B, C, L, S, H, gridtype, interpolation, align_corners = ctx.dims
        grad = grad.view(B, L, C).permute(1, 0, 2).contiguous()
        with_inputs = dy_dx.numel() > 0
        # a backward pass that does not use the table gradient (the eikonal term's
        # autograd.grad, which returns the points' gradient only; linear._wanted, scoped to
        # that graph task) would discard it: skip it (binned table gradient, csrc/encoders.hip)
        want_table = not with_inputs or _wanted(ctx.needs_input_grad[1], ctx.table_edge)
        # outside autograd, as the reference's backward (grid.py:65-89): under create_graph
        # (the eikonal term) its results are constants, not nodes of the double backward
        with torch.no_grad():
            grad_embeddings, grad_inputs = torch.ops.sdfr.grid_encode_backward(
                grad, inputs, embeddings, offsets, dy_dx, S, H, want_table, int(gridtype),
                bool(align_corners), int(interpolation))
        grad_embeddings = grad_embeddings if want_table else None
        grad_inputs = grad_inputs.to(inputs.dtype) if with_inputs else None
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
    """sphere_harmonics.py:14-37 over torch.ops.sdfr.sh_encode_forward / _backward."""
    @staticmethod
    def forward(ctx, inputs, degree, calc_grad_inputs=False):
        inputs = inputs.contiguous().float()
        outputs, dy_dx = torch.ops.sdfr.sh_encode_forward(inputs, int(degree),
                                                          bool(calc_grad_inputs))
        ctx.save_for_backward(inputs, dy_dx)
        ctx.degree = degree
        return outputs

    @staticmethod
    def backward(ctx, grad):
        inputs, dy_dx = ctx.saved_tensors
        if dy_dx.numel() == 0:
            return None, None, None
        with torch.no_grad():                   # (as _GridEncode.backward)
            gi = torch.ops.sdfr.sh_encode_backward(grad, inputs, dy_dx, int(ctx.degree))
        return gi, None, None


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
