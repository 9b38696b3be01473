"""torch.library registrations of the hot path's native ops (namespace ``sdfr``).

SURVEY.md §8(b)3: the reference binds its CUDA kernels through pybind11
(``grid_encode_forward`` / ``grid_encode_backward``, gridencoder.h:11-16, bindings.cpp:5-7;
``sh_encode_forward`` / ``sh_encode_backward``, shencoder.h:9-10), the caller allocates
every output and the kernels run on the current stream.  Here the same entry points are
``torch.ops.sdfr.*`` custom ops over libsdfr's C ABI (include/sdfr.h), each with a fake
(meta) implementation, so they are visible to ``torch.library.opcheck``, FakeTensor
shape propagation and ``torch.compile`` tracing; the drop-in modules call them
(encoders.py: GridEncoder / SHEncoder; renderer.py: the fused render of a plain
``VolumeFeatureRenderer`` call).  They run on ``torch.cuda.current_stream()`` and raise
``RuntimeError`` on a non-zero library status, as the reference's TORCH_CHECKs raise.

  sdfr::grid_encode_forward(inputs[B,D], embeddings[T,C], offsets[L+1] i32, S, H,
                            calc_dy_dx, gridtype, align_corners, interpolation)
        -> (outputs[L,B,C], dy_dx[B,L*D*C] or [0])
  sdfr::grid_encode_backward(grad[L,B,C], inputs, embeddings, offsets, dy_dx or [0], S, H,
                             want_table, gridtype, align_corners, interpolation)
        -> (grad_embeddings[T,C] or [0], grad_inputs[B,D] or [0])
  sdfr::sh_encode_forward(inputs[B,D], degree, calc_dy_dx) -> (outputs[B,deg^2], dy_dx or [0])
  sdfr::sh_encode_backward(grad[B,deg^2], inputs, dy_dx, degree) -> grad_inputs[B,D]
  sdfr::render_fused(kind, params[], cam, focal, near, far, styles, t_rand?, sigma_noise?,
                     pix_x, pix_y, t_vals, prepacked?, fscal[], iscal[], flags[], H, W, N)
        -> (rgb[B,3,H,W], features[B,256,H,W] or [0], sdf[B,H,W,N,1] or [0],
            mask[B,1,H,W] or [0], xyz[B,3,H,W] or [0])
     (sdfr_render_{ngp,siren,fc}_forward: kind 0 / 1 / 2; ``params`` in the order of
     ``weight_tensors``; ``flags`` = RENDER_FLAGS.)

An absent optional output is a 0-element tensor (a custom op returns tensors only).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from . import _lib

RENDER_FLAGS = ("t_rand_per_sample", "offset_sampling", "static_viewdirs", "z_normalize",
                "force_background", "with_sdf", "field_precision", "max_field_segments",
                "output_features", "return_sdf", "return_xyz")


def _check_cuda(t: Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")


def _none_if_empty(t: Tensor) -> Optional[Tensor]:
    return None if t.numel() == 0 else t


# ---------------------------------------------------------------- hash grid
@torch.library.custom_op("sdfr::grid_encode_forward", mutates_args=())
def grid_encode_forward(inputs: Tensor, embeddings: Tensor, offsets: Tensor, S: float, H: int,
                        calc_dy_dx: bool, gridtype: int, align_corners: bool,
                        interpolation: int) -> Tuple[Tensor, Tensor]:
    """kernel_grid (gridencoder.cu:88-245; entry point :448-471) as sdfr_grid_encode_forward."""
    for t, n in ((inputs, "inputs"), (embeddings, "embeddings"), (offsets, "offsets")):
        _check_cuda(t, n)
    if inputs.dtype != torch.float32 or embeddings.dtype != torch.float32:
        raise RuntimeError("sdface-gan_amd GridEncoder computes in fp32 (inputs and embeddings)")
    if offsets.dtype != torch.int32:
        raise RuntimeError("offsets must be an int tensor")
    inputs = inputs.contiguous()
    embeddings = embeddings.contiguous()
    offsets = offsets.contiguous()
    B, D = inputs.shape
    L, C = offsets.shape[0] - 1, embeddings.shape[1]
    outputs = torch.empty(L, B, C, device=inputs.device, dtype=embeddings.dtype)
    dy_dx = (torch.empty(B, L * D * C, device=inputs.device, dtype=embeddings.dtype)
             if calc_dy_dx else inputs.new_empty(0))
    _lib.check(_lib.lib().sdfr_grid_encode_forward(
        _lib.ptr(inputs), _lib.ptr(embeddings), _lib.ptr(offsets), _lib.ptr(outputs),
        B, D, C, L, S, H, _lib.ptr(_none_if_empty(dy_dx)), gridtype, int(align_corners),
        interpolation, _lib.stream_of(inputs)), "sdfr_grid_encode_forward")
    return outputs, dy_dx


@grid_encode_forward.register_fake
def _(inputs, embeddings, offsets, S, H, calc_dy_dx, gridtype, align_corners, interpolation):
    B, D = inputs.shape
    L, C = offsets.shape[0] - 1, embeddings.shape[1]
    return (inputs.new_empty(L, B, C, dtype=embeddings.dtype),
            inputs.new_empty(B, L * D * C, dtype=embeddings.dtype) if calc_dy_dx
            else inputs.new_empty(0))


@torch.library.custom_op("sdfr::grid_encode_backward", mutates_args=())
def grid_encode_backward(grad: Tensor, inputs: Tensor, embeddings: Tensor, offsets: Tensor,
                         dy_dx: Tensor, S: float, H: int, want_table: bool, gridtype: int,
                         align_corners: bool, interpolation: int) -> Tuple[Tensor, Tensor]:
    """kernel_grid_backward / kernel_input_backward (gridencoder.cu:249-369; entry point
    :473-503):
    the table gradient binned per row (deterministic, csrc/encoders.hip), the input
    gradient from dy_dx when one was saved."""
    grad = grad.contiguous()
    L, B, C = grad.shape
    D = inputs.shape[1]
    with_inputs = dy_dx.numel() > 0
    grad_inputs = torch.zeros_like(inputs, dtype=embeddings.dtype) if with_inputs else \
        inputs.new_empty(0)
    grad_embeddings = torch.zeros_like(embeddings) if want_table else embeddings.new_empty(0)
    L_ = _lib.lib()
    wsb = (L_.sdfr_grid_encode_backward_ws_bytes(B, D, C, L, S, H, int(align_corners))
           if want_table else 0)
    ws = torch.empty(wsb, dtype=torch.uint8, device=grad.device) if wsb else None
    _lib.check(L_.sdfr_grid_encode_backward_ws(
        _lib.ptr(grad), _lib.ptr(inputs), _lib.ptr(embeddings), _lib.ptr(offsets),
        _lib.ptr(_none_if_empty(grad_embeddings)), B, D, C, L, S, H,
        _lib.ptr(_none_if_empty(dy_dx)), _lib.ptr(_none_if_empty(grad_inputs)), gridtype,
        int(align_corners), interpolation, _lib.ptr(ws), wsb, _lib.stream_of(grad)),
        "sdfr_grid_encode_backward")
    return grad_embeddings, grad_inputs


@grid_encode_backward.register_fake
def _(grad, inputs, embeddings, offsets, dy_dx, S, H, want_table, gridtype, align_corners,
      interpolation):
    return (torch.empty_like(embeddings) if want_table else embeddings.new_empty(0),
            torch.empty_like(inputs, dtype=embeddings.dtype) if dy_dx.numel() > 0
            else inputs.new_empty(0))


# --------------------------------------------------------- spherical harmonics
@torch.library.custom_op("sdfr::sh_encode_forward", mutates_args=())
def sh_encode_forward(inputs: Tensor, degree: int, calc_dy_dx: bool) -> Tuple[Tensor, Tensor]:
    """kernel_sh (shencoder.cu:28-68; entry point :400-417) as sdfr_sh_encode_forward."""
    _check_cuda(inputs, "inputs")
    inputs = inputs.contiguous().float()
    B, D = inputs.shape
    outputs = torch.empty(B, degree ** 2, dtype=inputs.dtype, device=inputs.device)
    dy_dx = (torch.empty(B, D * degree ** 2, dtype=inputs.dtype, device=inputs.device)
             if calc_dy_dx else inputs.new_empty(0))
    _lib.check(_lib.lib().sdfr_sh_encode_forward(
        _lib.ptr(inputs), _lib.ptr(outputs), B, D, degree, _lib.ptr(_none_if_empty(dy_dx)),
        _lib.stream_of(inputs)), "sdfr_sh_encode_forward")
    return outputs, dy_dx


@sh_encode_forward.register_fake
def _(inputs, degree, calc_dy_dx):
    B, D = inputs.shape
    return (inputs.new_empty(B, degree ** 2, dtype=torch.float32),
            inputs.new_empty(B, D * degree ** 2, dtype=torch.float32) if calc_dy_dx
            else inputs.new_empty(0))


@torch.library.custom_op("sdfr::sh_encode_backward", mutates_args=())
def sh_encode_backward(grad: Tensor, inputs: Tensor, dy_dx: Tensor, degree: int) -> Tensor:
    """kernel_sh_backward (shencoder.cu:359-385; entry point :419-439) as sdfr_sh_encode_backward."""
    grad = grad.contiguous()
    B, D = inputs.shape
    grad_inputs = torch.zeros_like(inputs)
    _lib.check(_lib.lib().sdfr_sh_encode_backward(
        _lib.ptr(grad), _lib.ptr(inputs), B, D, degree, _lib.ptr(dy_dx),
        _lib.ptr(grad_inputs), _lib.stream_of(grad)), "sdfr_sh_encode_backward")
    return grad_inputs


@sh_encode_backward.register_fake
def _(grad, inputs, dy_dx, degree):
    return torch.empty_like(inputs)


# ---------------------------------------------------------------- fused render
def weights_struct(kind: int, ts: Sequence[Tensor], fscal: Sequence[float],
                   iscal: Sequence[int], with_sdf: bool):
    """sdfr_{ngp,siren,fc}_weights from the flat tensor list of weight_tensors (kind 0 /
    1 / 2) and the network's scalars (ngp: fscal = (log2 per-level scale, bound), iscal =
    (base resolution,); SIREN / FC: iscal = (depth, width))."""
    P = _lib.ptr
    it = iter(ts)
    nxt = lambda: P(next(it))  # noqa: E731
    if kind == 0:
        w = _lib.NgpWeights()
        emb, off = next(it), next(it)
        w.embeddings, w.offsets = P(emb), P(off)
        w.num_levels = off.shape[0] - 1
        w.log2_per_level_scale, w.bound = float(fscal[0]), float(fscal[1])
        w.base_resolution = int(iscal[0])
        w.input_w, w.input_b = nxt(), nxt()
        n_pts = 3
    elif kind == 1:
        w = _lib.SirenWeights()
        w.depth, w.width = int(iscal[0]), int(iscal[1])
        n_pts = 8
    else:
        w = _lib.FcWeights()
        w.depth, w.width = int(iscal[0]), int(iscal[1])
        w.x_in_w, w.x_in_b, w.style_w, w.style_b = nxt(), nxt(), nxt(), nxt()
        for l in range(7):
            w.pts_w[l], w.pts_b[l] = nxt(), nxt()
        w.views_w, w.views_b = nxt(), nxt()
    if kind != 2:
        for l in range(n_pts):
            w.pts_w[l], w.pts_b[l] = nxt(), nxt()
            w.pts_gw[l], w.pts_gb[l] = nxt(), nxt()
            w.pts_bw[l], w.pts_bb[l] = nxt(), nxt()
        w.views_w, w.views_b = nxt(), nxt()
        w.views_gw, w.views_gb = nxt(), nxt()
        w.views_bw, w.views_bb = nxt(), nxt()
    w.sigma_w, w.sigma_b, w.rgb_w, w.rgb_b = nxt(), nxt(), nxt(), nxt()
    beta = next(it)
    w.sigmoid_beta = P(beta) if with_sdf else None
    return w


def render_args(B, H, W, N, cam, focal, near, far, styles, pix_x, pix_y, t_vals, t_rand,
                sigma_noise, flags: dict, rgb, features, sdf, xyz, mask, ws, prepacked):
    """sdfr_ngp_render_args (shared by the three networks' entry points)."""
    P = _lib.ptr
    a = _lib.NgpRenderArgs()
    a.B, a.H, a.W, a.N = B, H, W, N
    a.cam, a.focal, a.near_, a.far_ = P(cam), P(focal), P(near), P(far)
    a.styles = P(styles)
    a.pix_x, a.pix_y, a.t_vals = P(pix_x), P(pix_y), P(t_vals)
    a.t_rand, a.sigma_noise = P(t_rand), P(sigma_noise)
    a.t_rand_per_sample = int(flags["t_rand_per_sample"])
    a.offset_sampling = int(flags["offset_sampling"])
    a.static_viewdirs = int(flags["static_viewdirs"])
    a.z_normalize = int(flags["z_normalize"])
    a.force_background = int(flags["force_background"])
    a.with_sdf = int(flags["with_sdf"])
    a.rgb, a.features, a.sdf = P(rgb), P(features), P(sdf)
    a.xyz, a.mask = P(xyz), P(mask)
    a.workspace, a.workspace_bytes = P(ws), ws.numel()
    a.field_precision = int(flags["field_precision"])
    a.max_field_segments = int(flags["max_field_segments"])
    a.prepacked = P(prepacked)
    return a


def workspace_bytes(kind: int, B: int, H: int, W: int, N: int, num_levels: int) -> int:
    L = _lib.lib()
    if kind == 2:
        return L.sdfr_render_fc_workspace_bytes(B, H, W, N)
    if kind == 1:
        return L.sdfr_render_siren_workspace_bytes(B)
    return L.sdfr_render_ngp_workspace_bytes(B, H, W, N, num_levels)


FORWARD_FN = ("sdfr_render_ngp_forward", "sdfr_render_siren_forward", "sdfr_render_fc_forward")


def _render_outputs(B, H, W, N, dev, output_features, return_sdf, return_xyz, empty):
    z = lambda: empty(0, device=dev)  # noqa: E731
    return (empty(B, 3, H, W, device=dev),
            empty(B, 256, H, W, device=dev) if output_features else z(),
            empty(B, H, W, N, 1, device=dev) if return_sdf else z(),
            empty(B, 1, H, W, device=dev) if return_xyz else z(),
            empty(B, 3, H, W, device=dev) if return_xyz else z())


@torch.library.custom_op("sdfr::render_fused", mutates_args=())
def render_fused(kind: int, params: List[Tensor], cam: Tensor, focal: Tensor, near: Tensor,
                 far: Tensor, styles: Tensor, t_rand: Optional[Tensor],
                 sigma_noise: Optional[Tensor], pix_x: Tensor, pix_y: Tensor, t_vals: Tensor,
                 prepacked: Optional[Tensor], fscal: List[float], iscal: List[int],
                 flags: List[int], H: int, W: int, N: int
                 ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """The whole render of B faces (rays, sampling, encoders, field MLP, compositing;
    sdf_model.py:166-423) in one library call: VolumeFeatureRenderer.fused_forward's
    plain case.  Inputs contiguous fp32 on one device; ``flags`` in RENDER_FLAGS order."""
    f = dict(zip(RENDER_FLAGS, flags))
    _check_cuda(cam, "cam")
    B, dev = cam.shape[0], cam.device
    num_levels = params[1].shape[0] - 1 if kind == 0 else 0
    rgb, features, sdf, mask, xyz = _render_outputs(
        B, H, W, N, dev, f["output_features"], f["return_sdf"], f["return_xyz"], torch.empty)
    ws = torch.empty(workspace_bytes(kind, B, H, W, N, num_levels), dtype=torch.uint8,
                     device=dev)
    w = weights_struct(kind, params, fscal, iscal, bool(f["with_sdf"]))
    a = render_args(B, H, W, N, cam, focal, near, far, styles, pix_x, pix_y, t_vals, t_rand,
                    sigma_noise, f, rgb, _none_if_empty(features), _none_if_empty(sdf),
                    _none_if_empty(xyz), _none_if_empty(mask), ws, prepacked)
    name = FORWARD_FN[kind]
    _lib.check(getattr(_lib.lib(), name)(ctypes.byref(w), ctypes.byref(a), _lib.stream_of(cam)),
               name)
    return rgb, features, sdf, mask, xyz


@render_fused.register_fake
def _(kind, params, cam, focal, near, far, styles, t_rand, sigma_noise, pix_x, pix_y, t_vals,
      prepacked, fscal, iscal, flags, H, W, N):
    f = dict(zip(RENDER_FLAGS, flags))
    return _render_outputs(cam.shape[0], H, W, N, cam.device, f["output_features"],
                           f["return_sdf"], f["return_xyz"],
                           lambda *s, device: cam.new_empty(s, dtype=torch.float32))
