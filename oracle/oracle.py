"""CPU ORACLE for the SDFace-GAN SDF+ngp renderer hot path -- TEST INFRASTRUCTURE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product package (``sdface-gan_amd/``) never imports it: the HIP path fails
loudly when its extension is missing instead of falling back here.

Two layers:

* ``libsdfr_oracle.so`` (``oracle/csrc/sdfr_oracle.c``): a plain-C restatement
  of the reference CUDA kernels (``gridencoder.cu``, ``shencoder.cu``) and of the
  ray-sampling float chain that must be bit-exact.  Wrapped here with numpy.
* ``render_ngp`` / ``render_ngp_torch``: a PyTorch-CPU fp32 restatement of
  ``VolumeFeatureRenderer.forward`` + ``NGPSIRENGenerator.forward``
  (``im2scene/sdf/models/sdf_model.py:143-423, 1534-1592``), op for op in the
  reference's order, with the two encoders routed to the C restatement.

Pinning: ``tests/golden/make_golden.py`` ran the *reference's own* Python code
(imported in the build container with stubs for off-path packages) with these
C encoders injected as its ``_gridencoder`` / ``_shencoder`` backends, and
committed the results under ``tests/golden/``.  ``tests/test_oracle.py`` checks
this restatement against those fixtures and the encoder KATs.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "build" / "libsdfr_oracle.so"

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32 = ctypes.c_uint32
_lib = None


def build(force: bool = False) -> Path:
    """Compile the C oracle with gcc (oracle/Makefile)."""
    if force or not LIB_PATH.exists():
        subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        L.orc_level_scale.restype = ctypes.c_float
        L.orc_level_scale.argtypes = [_u32, ctypes.c_float, _u32]
        L.orc_set_exp2_ulp.argtypes = [_i32p, _u32]
        L.orc_level_resolution.restype = _u32
        L.orc_level_resolution.argtypes = [ctypes.c_float]
        L.orc_grid_index.restype = _u32
        L.orc_grid_index.argtypes = [_u32, ctypes.c_int, _u32, _u32, _u32,
                                     ctypes.POINTER(_u32), _u32, _u32]
        L.orc_grid_encode_forward.argtypes = [_f32p, _f32p, _i32p, _f32p, _u32, _u32, _u32, _u32,
                                              ctypes.c_float, _u32, _f32p, _u32, ctypes.c_int, _u32]
        L.orc_grid_encode_backward.argtypes = [_f32p, _f32p, _f32p, _i32p, _f32p, _u32, _u32, _u32,
                                               _u32, ctypes.c_float, _u32, _f32p, _f32p, _u32,
                                               ctypes.c_int, _u32]
        L.orc_sh_encode_forward.argtypes = [_f32p, _f32p, _u32, _u32, _u32, _f32p]
        L.orc_sh_encode_backward.argtypes = [_f32p, _f32p, _u32, _u32, _u32, _f32p, _f32p]
        L.orc_sample_rays.argtypes = [_f32p] * 8 + [ctypes.c_int] * 4 + [ctypes.c_float] * 2 + \
            [_u32] * 4 + [_f32p] * 6
        _lib = L
    return _lib


def _p(a, typ=_f32p):
    if a is None:
        return ctypes.cast(None, typ)
    assert a.flags["C_CONTIGUOUS"], "oracle arrays must be C-contiguous"
    return a.ctypes.data_as(typ)


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


# --------------------------------------------------------------------------
# hash-grid encoder (gridencoder.cu / grid.py)
# --------------------------------------------------------------------------
def grid_offsets(num_levels=16, level_dim=2, base_resolution=16, log2_hashmap_size=19,
                 desired_resolution=4096, input_dim=3, align_corners=False):
    """Per-level table offsets and per_level_scale, grid.py:97-134 (float64 numpy)."""
    per_level_scale = np.exp2(np.log2(desired_resolution / base_resolution) / (num_levels - 1))
    offsets, offset = [], 0
    max_params = 2 ** log2_hashmap_size
    for i in range(num_levels):
        resolution = int(np.ceil(base_resolution * per_level_scale ** i))
        params = min(max_params, (resolution if align_corners else resolution + 1) ** input_dim)
        params = int(np.ceil(params / 8) * 8)
        offsets.append(offset)
        offset += params
    offsets.append(offset)
    return np.array(offsets, dtype=np.int32), per_level_scale


def level_table(L, S, H, offsets):
    """(scale, resolution, hashmap_size) per level, gridencoder.cu:136-139."""
    lb = lib()
    out = []
    for level in range(L):
        sc = lb.orc_level_scale(level, ctypes.c_float(S), H)
        out.append((np.float32(sc), int(lb.orc_level_resolution(ctypes.c_float(sc))),
                    int(offsets[level + 1] - offsets[level])))
    return out


def set_exp2_ulp(offsets=None):
    """Move the oracle's per-level exp2f result by ``offsets[level]`` ulps (None: back
    to the correctly rounded value) -- the exp2f sensitivity test's probe for a CUDA
    exp2f that differs from the correctly rounded one (documented <= 2 ulp)."""
    if offsets is None:
        lib().orc_set_exp2_ulp(ctypes.cast(None, _i32p), 0)
        return
    off = np.ascontiguousarray(offsets, dtype=np.int32)
    lib().orc_set_exp2_ulp(_p(off, _i32p), off.shape[0])


def grid_index(pos_grid, hashmap_size, resolution, gridtype=0, align_corners=False, C=2):
    pg = (_u32 * len(pos_grid))(*[int(v) for v in pos_grid])
    return int(lib().orc_grid_index(gridtype, int(align_corners), 0, hashmap_size, resolution,
                                    pg, len(pos_grid), C))


def grid_encode_forward(inputs, embeddings, offsets, per_level_scale, base_resolution,
                        calc_dy_dx=False, gridtype=0, align_corners=False, interp=0):
    """Returns (outputs [L,B,C], dy_dx [B, L*D*C] or None), as grid.py:27-55 sees them."""
    x = _f32(inputs)
    emb = _f32(embeddings)
    off = np.ascontiguousarray(offsets, dtype=np.int32)
    B, D = x.shape
    L = off.shape[0] - 1
    C = emb.shape[1]
    S = np.float32(np.log2(per_level_scale))
    out = np.empty((L, B, C), np.float32)
    dydx = np.empty((B, L * D * C), np.float32) if calc_dy_dx else None
    rc = lib().orc_grid_encode_forward(_p(x), _p(emb), _p(off, _i32p), _p(out), B, D, C, L,
                                       ctypes.c_float(S), int(base_resolution), _p(dydx),
                                       gridtype, int(align_corners), interp)
    if rc != 0:
        raise RuntimeError("GridEncoding: C must be 1, 2, 4, or 8.")
    return out, dydx


def grid_encode_backward(grad, inputs, embeddings, offsets, per_level_scale, base_resolution,
                         dy_dx=None, gridtype=0, align_corners=False, interp=0):
    """grad: [L,B,C].  Returns (grad_embeddings, grad_inputs or None)."""
    g = _f32(grad)
    x = _f32(inputs)
    emb = _f32(embeddings)
    off = np.ascontiguousarray(offsets, dtype=np.int32)
    B, D = x.shape
    L = off.shape[0] - 1
    C = emb.shape[1]
    S = np.float32(np.log2(per_level_scale))
    gemb = np.zeros_like(emb)
    dd = _f32(dy_dx) if dy_dx is not None else None
    gin = np.zeros_like(x) if dy_dx is not None else None
    rc = lib().orc_grid_encode_backward(_p(g), _p(x), _p(emb), _p(off, _i32p), _p(gemb), B, D, C, L,
                                        ctypes.c_float(S), int(base_resolution), _p(dd), _p(gin),
                                        gridtype, int(align_corners), interp)
    if rc != 0:
        raise RuntimeError("GridEncoding: C must be 1, 2, 4, or 8.")
    return gemb, gin


# --------------------------------------------------------------------------
# SH encoder (shencoder.cu)
# --------------------------------------------------------------------------
def sh_encode_forward(inputs, degree=4, calc_dy_dx=False):
    x = _f32(inputs)
    B, D = x.shape
    out = np.empty((B, degree * degree), np.float32)
    dydx = np.empty((B, D * degree * degree), np.float32) if calc_dy_dx else None
    if lib().orc_sh_encode_forward(_p(x), _p(out), B, D, degree, _p(dydx)) != 0:
        raise RuntimeError("SH oracle supports input_dim 3, degree 1..8")
    return out, dydx


def sh_encode_backward(grad, inputs, degree, dy_dx):
    g = _f32(grad)
    x = _f32(inputs)
    B, D = x.shape
    gin = np.zeros_like(x)
    if lib().orc_sh_encode_backward(_p(g), _p(x), B, D, degree, _p(_f32(dy_dx)), _p(gin)) != 0:
        raise RuntimeError("SH oracle supports input_dim 3, degree 1..8")
    return gin


# --------------------------------------------------------------------------
# ray generation + sampling (sdf_model.py:207-222, 310-351, 363-378)
# --------------------------------------------------------------------------
def pixel_centres(res):
    """The renderer's i/j buffers (sdf_model.py:167-171): linspace(0.5, res-0.5, res)."""
    import torch
    return torch.linspace(0.5, res - 0.5, res).numpy().astype(np.float32)


def t_values(n_samples, offset_sampling=True):
    """sdf_model.py:174-177 (torch CPU linspace, float32)."""
    import torch
    if offset_sampling:
        return torch.linspace(0., 1. - 1 / n_samples, steps=n_samples).numpy().astype(np.float32)
    return torch.linspace(0., 1., steps=n_samples).numpy().astype(np.float32)


def sample_rays(cam, focal, near, far, H, W, N, t_rand=None, offset_sampling=True,
                static_viewdirs=False, z_normalize=True, bound=2.0, pix_x=None, pix_y=None):
    cam = _f32(cam).reshape(-1, 3, 4)
    B = cam.shape[0]
    focal = _f32(focal).reshape(B)
    near = _f32(near).reshape(B)
    far = _f32(far).reshape(B)
    px = _f32(pixel_centres(W) if pix_x is None else pix_x)
    py = _f32(pixel_centres(H) if pix_y is None else pix_y)
    tv = _f32(t_values(N, offset_sampling))
    tr = None
    per_sample = 0
    if t_rand is not None:
        tr = _f32(t_rand)
        per_sample = int(tr.size == B * H * W * N and N != 1)
    rays_d = np.empty((B, H, W, 3), np.float32)
    vd = np.empty((B, H, W, 3), np.float32)
    dn = np.empty((B, H, W), np.float32)
    z = np.empty((B, H, W, N), np.float32)
    pts = np.empty((B, H, W, N, 3), np.float32)
    u = np.empty((B, H, W, N, 3), np.float32)
    rc = lib().orc_sample_rays(_p(cam), _p(focal), _p(near), _p(far), _p(px), _p(py), _p(tv),
                               _p(tr), per_sample, int(offset_sampling), int(static_viewdirs),
                               int(z_normalize), ctypes.c_float(W * 0.5), ctypes.c_float(bound),
                               B, H, W, N, _p(rays_d), _p(vd), _p(dn), _p(z), _p(pts), _p(u))
    if rc != 0:
        raise RuntimeError("orc_sample_rays failed")
    return dict(rays_d=rays_d, viewdirs=vd, dnorm=dn, z_vals=z, pts=pts, grid_in=u)


# --------------------------------------------------------------------------
# full renderer restatement, PyTorch CPU fp32 (sdf_model.py:23-69, 143-423, 1534-1592)
# --------------------------------------------------------------------------
def _linear(x, w, b):
    import torch.nn.functional as F
    return F.linear(x, w, bias=b)


def render_ngp(sd, cam, focal, near, far, styles, *, N=24, res=64, t_rand=None,
               offset_sampling=True, static_viewdirs=False, z_normalize=True,
               force_background=False, output_features=True, with_sdf=True,
               return_intermediates=False, prefix="renderer."):
    """fp32 CPU restatement of VolumeFeatureRenderer(type='ngp').forward.

    ``sd``: a state dict with the reference's key names (``renderer.*``),
    ``styles``: the renderer latent [B,256] (after the mapping network).
    ``t_rand``: per-ray [B,H,W] uniform draws for offset sampling (None -> no perturb).
    Returns dict(rgb [B,3,H,W], features [B,256,H,W], sdf [B,H,W,N,1],
    mask [B,1,H,W], xyz [B,3,H,W]) (+ intermediates).
    """
    import torch

    def P(k):
        v = sd[prefix + k]
        return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))

    cam = torch.as_tensor(cam, dtype=torch.float32).reshape(-1, 3, 4)
    B = cam.shape[0]
    styles = torch.as_tensor(styles, dtype=torch.float32)
    ray = sample_rays(cam.numpy(), np.asarray(focal).reshape(B), np.asarray(near).reshape(B),
                      np.asarray(far).reshape(B), res, res, N, t_rand=t_rand,
                      offset_sampling=offset_sampling, static_viewdirs=static_viewdirs,
                      z_normalize=z_normalize)
    S = B * res * res * N
    net = "network."
    emb = P(net + "encoder.embeddings").numpy()
    offsets = P(net + "encoder.offsets").numpy()
    _, pls = grid_offsets()
    enc, _ = grid_encode_forward(ray["grid_in"].reshape(S, 3), emb, offsets, pls, 16)
    enc = torch.from_numpy(enc).permute(1, 0, 2).reshape(S, -1)           # grid.py:57
    vd = np.broadcast_to(ray["viewdirs"][:, :, :, None, :], (B, res, res, N, 3)).reshape(S, 3)
    sh, _ = sh_encode_forward(np.ascontiguousarray(vd), 4)
    sh = torch.from_numpy(sh)

    # NGPSIRENGenerator.forward, sdf_model.py:1566-1592 (per-face FiLM broadcast)
    h = _linear(enc, P(net + "input_linear.weight"), P(net + "input_linear.bias"))
    h = 1 * h + 0                                           # LinearLayer std/bias init
    h = h.view(B, res, res, N, -1)
    sty = styles

    def film(x, pre):
        out = _linear(x, P(pre + "weight"), P(pre + "bias"))
        gamma = 15 * _linear(sty, P(pre + "gamma.weight"), P(pre + "gamma.bias")) + 30
        beta = 0.25 * _linear(sty, P(pre + "beta.weight"), P(pre + "beta.bias")) + 0
        gamma = gamma.view(B, 1, 1, 1, -1)
        beta = beta.view(B, 1, 1, 1, -1)
        return torch.sin(gamma * out + beta)

    for i in range(3):
        h = film(h, f"{net}pts_linears.{i}.")
    sdf = 1 * _linear(h, P(net + "sigma_linear.weight"), P(net + "sigma_linear.bias")) + 0
    hv = torch.cat([h, sh.view(B, res, res, N, -1)], -1)
    feat = film(hv, net + "views_linears.")
    rgb_raw = 1 * _linear(feat, P(net + "rgb_linear.weight"), P(net + "rgb_linear.bias")) + 0

    out = _integrate(ray, sdf, rgb_raw, feat, P("sigmoid_beta"), with_sdf, force_background,
                     output_features)
    if return_intermediates:
        out.update(ray)
        out.update(enc=enc, sh=sh, rgb_raw=rgb_raw, feat_samples=feat)
    return out


def _integrate(ray, sdf, rgb_raw, feat, beta_s, with_sdf, force_background, output_features):
    """volume_integration, sdf_model.py:236-301 (torch CPU fp32)."""
    import torch
    z = torch.from_numpy(ray["z_vals"])
    dn = torch.from_numpy(ray["dnorm"])[..., None]
    dists = z[..., 1:] - z[..., :-1]
    dists = torch.cat([dists, torch.tensor([1e10]).expand(dn.shape)], -1)
    dists = dists * dn
    if with_sdf:
        sigma = torch.sigmoid(-sdf / beta_s) / beta_s
        sigma = 1 - torch.exp(-sigma * dists.unsqueeze(-1))
    else:
        sigma = 1 - torch.exp(-torch.nn.functional.softplus(sdf) * dists.unsqueeze(-1))
    vis = torch.cumprod(torch.cat([torch.ones_like(sigma[..., :1, :]), 1. - sigma + 1e-10], 3), 3)
    vis = vis[..., :-1, :]
    weights = sigma * vis
    if force_background:
        weights[..., -1, :] = 1 - weights[..., :-1, :].sum(3)
    rgb_map = -1 + 2 * torch.sum(weights * torch.sigmoid(rgb_raw), 3)
    feat_map = torch.sum(weights * feat, 3) if output_features else None
    pts = torch.from_numpy(ray["pts"])
    xyz = torch.sum(weights * pts, 3)
    mask = weights[..., -1, :]
    return dict(rgb=rgb_map.permute(0, 3, 1, 2).contiguous(),
                features=feat_map.permute(0, 3, 1, 2).contiguous() if feat_map is not None
                else None,
                sdf=sdf, mask=mask.permute(0, 3, 1, 2).contiguous(),
                xyz=xyz.permute(0, 3, 1, 2).contiguous(), weights=weights)


def render_siren(sd, cam, focal, near, far, styles, *, N=24, res=64, t_rand=None,
                 offset_sampling=True, static_viewdirs=False, z_normalize=True,
                 force_background=False, output_features=True, with_sdf=True, depth=8,
                 prefix="renderer."):
    """fp32 CPU restatement of VolumeFeatureRenderer(type='sdf').forward: the ray /
    sample chain of render_rays (sdf_model.py:310-351) feeding SirenGenerator
    (sdf_model.py:101-139) with the normalised points and unit view directions,
    then volume_integration.  Same arguments and outputs as render_ngp."""
    import torch

    def P(k):
        v = sd[prefix + k]
        return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))

    cam = torch.as_tensor(cam, dtype=torch.float32).reshape(-1, 3, 4)
    B = cam.shape[0]
    near = np.asarray(near, np.float32).reshape(B)
    far = np.asarray(far, np.float32).reshape(B)
    ray = sample_rays(cam.numpy(), np.asarray(focal).reshape(B), near, far, res, res, N,
                      t_rand=t_rand, offset_sampling=offset_sampling,
                      static_viewdirs=static_viewdirs, z_normalize=z_normalize)
    pts = torch.from_numpy(ray["pts"])
    if z_normalize:                                           # sdf_model.py:348-349
        span = torch.from_numpy(far - near).view(B, 1, 1, 1, 1)
        x = pts * 2 / span
    else:
        x = pts
    vd = torch.from_numpy(np.ascontiguousarray(
        np.broadcast_to(ray["viewdirs"][:, :, :, None, :], (B, res, res, N, 3))))
    sty = torch.as_tensor(styles, dtype=torch.float32)
    net = "network."

    def film(h, pre):
        out = _linear(h, P(pre + "weight"), P(pre + "bias"))
        gamma = 15 * _linear(sty, P(pre + "gamma.weight"), P(pre + "gamma.bias")) + 30
        beta = 0.25 * _linear(sty, P(pre + "beta.weight"), P(pre + "beta.bias")) + 0
        return torch.sin(gamma.view(B, 1, 1, 1, -1) * out + beta.view(B, 1, 1, 1, -1))

    h = x
    for i in range(depth):
        h = film(h, f"{net}pts_linears.{i}.")
    sdf = 1 * _linear(h, P(net + "sigma_linear.weight"), P(net + "sigma_linear.bias")) + 0
    feat = film(torch.cat([h, vd], -1), net + "views_linears.")
    rgb_raw = 1 * _linear(feat, P(net + "rgb_linear.weight"), P(net + "rgb_linear.bias")) + 0
    return _integrate(ray, sdf, rgb_raw, feat, P("sigmoid_beta"), with_sdf, force_background,
                      output_features)


def _posenc(p, L):
    """FCGenerator.transform_points (sdf_model.py:1628-1640): p / 2, then per frequency i
    sin and cos of (2^i pi) p, concatenated (torch CPU fp32, the reference's op order)."""
    import torch
    p = p / 2
    return torch.cat([torch.cat([torch.sin((2 ** i) * np.pi * p), torch.cos((2 ** i) * np.pi * p)],
                                dim=-1) for i in range(L)], dim=-1)


def render_fc(sd, cam, focal, near, far, styles, *, N=24, res=64, t_rand=None,
              offset_sampling=True, static_viewdirs=False, z_normalize=True,
              force_background=False, output_features=True, with_sdf=True, depth=8,
              prefix="renderer."):
    """fp32 CPU restatement of VolumeFeatureRenderer(fc=1).forward: render_rays'
    ray / sample chain (sdf_model.py:310-351) feeding FCGenerator (sdf_model.py:1599-1670:
    positional encodings, x_in + style_in, ReLU MLP, sigma, views_linears, rgb_linear),
    then volume_integration.  Same arguments and outputs as render_ngp."""
    import torch
    import torch.nn.functional as F

    def P(k):
        v = sd[prefix + k]
        return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))

    cam = torch.as_tensor(cam, dtype=torch.float32).reshape(-1, 3, 4)
    B = cam.shape[0]
    near = np.asarray(near, np.float32).reshape(B)
    far = np.asarray(far, np.float32).reshape(B)
    ray = sample_rays(cam.numpy(), np.asarray(focal).reshape(B), near, far, res, res, N,
                      t_rand=t_rand, offset_sampling=offset_sampling,
                      static_viewdirs=static_viewdirs, z_normalize=z_normalize)
    pts = torch.from_numpy(ray["pts"])
    if z_normalize:
        span = torch.from_numpy(far - near).view(B, 1, 1, 1, 1)
        x = pts * 2 / span
    else:
        x = pts
    vd = torch.from_numpy(np.ascontiguousarray(
        np.broadcast_to(ray["viewdirs"][:, :, :, None, :], (B, res, res, N, 3))))
    sty = torch.as_tensor(styles, dtype=torch.float32)
    net = "network."
    h = _linear(_posenc(x, 10), P(net + "x_in.weight"), P(net + "x_in.bias"))
    s = _linear(sty, P(net + "style_in.weight"), P(net + "style_in.bias")).view(B, 1, 1, 1, -1)
    h = F.relu(h + s)
    for i in range(depth - 1):
        h = F.relu(_linear(h, P(f"{net}pts_linears.{i}.weight"), P(f"{net}pts_linears.{i}.bias")))
    sdf = _linear(h, P(net + "sigma_linear.weight"), P(net + "sigma_linear.bias"))
    feat = _linear(torch.cat([h, _posenc(vd, 4)], -1), P(net + "views_linears.weight"),
                   P(net + "views_linears.bias"))
    rgb_raw = _linear(feat, P(net + "rgb_linear.weight"), P(net + "rgb_linear.bias"))
    return _integrate(ray, sdf, rgb_raw, feat, P("sigmoid_beta"), with_sdf, force_background,
                      output_features)


# --------------------------------------------------------------------------
# StyleGAN2 decoder ops (im2scene/sdf/models/sdf_op.py), numpy
# --------------------------------------------------------------------------
def fused_bias_act(x, bias, ref, act, grad, alpha, scale):
    """fused_bias_act_kernel.cu:18-47 in fp32: y = f(x + bias[dim 1]) * scale."""
    x = np.asarray(x, np.float32)
    if bias is not None and np.size(bias):
        x = (x + np.asarray(bias, np.float32).reshape([1, -1] + [1] * (x.ndim - 2))).astype(
            np.float32)
    mode = act * 10 + grad
    a = np.float32(alpha)
    if mode == 30:
        y = np.where(x > 0, x, x * a)
    elif mode == 31:
        y = np.where(np.asarray(ref, np.float32) > 0, x, x * a)
    elif mode in (12, 32):
        y = np.zeros_like(x)
    else:
        y = x
    return (y * np.float32(scale)).astype(np.float32)


def upfirdn2d(x, kernel, up_x, up_y, down_x, down_y, pad_x0, pad_x1, pad_y0, pad_y1):
    """upfirdn2d_native (sdf_op.py:273-316) on [major, h, w], accumulated in float64:
    zero-insertion upsample, pad / crop, true convolution with ``kernel``, decimate."""
    x = np.asarray(x, np.float64)
    k = np.asarray(kernel, np.float64)
    m, h, w = x.shape
    kh, kw = k.shape
    u = np.zeros((m, h * up_y, w * up_x))
    u[:, ::up_y, ::up_x] = x
    u = np.pad(u, ((0, 0), (max(pad_y0, 0), max(pad_y1, 0)), (max(pad_x0, 0), max(pad_x1, 0))))
    u = u[:, max(-pad_y0, 0):u.shape[1] - max(-pad_y1, 0),
          max(-pad_x0, 0):u.shape[2] - max(-pad_x1, 0)]
    oh, ow = u.shape[1] - kh + 1, u.shape[2] - kw + 1
    kf = k[::-1, ::-1]
    out = np.zeros((m, oh, ow))
    for i in range(kh):
        for j in range(kw):
            out += u[:, i:i + oh, j:j + ow] * kf[i, j]
    return out[:, ::down_y, ::down_x]


def styled_epilogue(conv, *, kernel2d, bias, noise_weight, noise=None, demod=None,
                    blur_up=False, s_next=None, rgb_w=None, rgb_b=None, skip=None,
                    slope=0.2, scale=2 ** 0.5):
    """What follows a decoder convolution in the reference, NCHW float64:
    ModulatedConv2d demod + blur (sdf_model.py:676-699), NoiseInjection
    (:704-792), FusedLeakyReLU (:818), ToRGB + Upsample of the skip (:821-843).
    Returns (y = act * s_next, rgb)."""
    c = np.asarray(conv, np.float64)
    B, C = c.shape[:2]
    if blur_up:   # Blur(pad=(1,1)) of the stride-2 transposed conv output
        c = upfirdn2d(c.reshape(B * C, *c.shape[2:]), kernel2d, 1, 1, 1, 1, 1, 1, 1, 1)
        c = c.reshape(B, C, *c.shape[1:])
    H, W = c.shape[2:]
    v = c * (1.0 if demod is None else np.asarray(demod, np.float64)[:, :, None, None])
    if noise is not None:
        v = v + float(noise_weight) * np.broadcast_to(np.asarray(noise, np.float64), (B, 1, H, W))
    v = v + np.asarray(bias, np.float64).reshape(1, C, 1, 1)
    v = np.where(v > 0, v, v * slope) * scale
    y = v if s_next is None else v * np.asarray(s_next, np.float64)[:, :, None, None]
    rgb = None
    if rgb_w is not None:
        rgb = np.einsum("bchw,boc->bohw", v, np.asarray(rgb_w, np.float64))
        rgb = rgb + np.asarray(rgb_b, np.float64).reshape(1, 3, 1, 1)
        if skip is not None:
            s = np.asarray(skip, np.float64)
            up = upfirdn2d(s.reshape(B * 3, *s.shape[2:]), kernel2d, 2, 2, 1, 1, 2, 1, 2, 1)
            rgb = rgb + up.reshape(B, 3, H, W)
    return y, rgb


# --------------------------------------------------------------------------
# deterministic, platform-independent weights (integer hash; no libm)
# --------------------------------------------------------------------------
def det_uniform(shape, lo, hi, seed):
    """splitmix64 over the flat index -> U[lo,hi) float32, bit-identical on any host."""
    n = int(np.prod(shape)) if len(shape) else 1
    with np.errstate(over="ignore"):
        x = np.arange(n, dtype=np.uint64) + np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    u = (x >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)
