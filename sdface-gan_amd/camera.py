"""Camera sampling for the renderer: generate_camera_params (sdf_utils.py:97-159).

Same argument meaning and the same random draws (torch.randn / torch.rand on
``device``, same order).  On the CPU the reference's torch ops, bit-identical to
it; on the GPU the draws then one HIP launch for everything after them
(``sdfr_camera_extrinsics``), equal to the reference to a few fp32 ulp.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def generate_camera_params(resolution, device, batch=1, locations=None, sweep=False,
                           uniform=False, azim_range=0.3, elev_range=0.15, fov_ang=6,
                           dist_radius=0.12):
    """Returns (extrinsics [B,3,4] = [R^T | T], focal [B,1,1], near [B,1,1],
    far [B,1,1], viewpoint [B,2] = (azim, elev))."""
    dev = torch.device(device)
    scalar = all(not isinstance(v, torch.Tensor) or v.numel() == 1
                 for v in (fov_ang, dist_radius))
    if dev.type == "cuda" and scalar:
        # per-view fov / radius tensors (sdf_mesh.py:46-55) take the torch ops below
        return _camera_cuda(resolution, dev, batch, locations, sweep, uniform, azim_range,
                            elev_range, fov_ang, dist_radius)
    if locations is not None:
        azim = locations[:, 0].view(-1, 1)
        elev = locations[:, 1].view(-1, 1)
        dist = torch.ones(azim.shape[0], 1, device=device)
        near, far = (dist - dist_radius).unsqueeze(-1), (dist + dist_radius).unsqueeze(-1)
        fov = fov_ang * torch.ones(azim.shape[0], 1, device=device).view(-1, 1) * np.pi / 180
        focal = 0.5 * resolution / torch.tan(fov).unsqueeze(-1)
    elif sweep:
        azim = (-azim_range + (2 * azim_range / 7) * torch.arange(8, device=device))
        azim = azim.view(-1, 1).repeat(batch, 1)
        elev = (-elev_range + 2 * elev_range *
                torch.rand(batch, 1, device=device).repeat(1, 8).view(-1, 1))
        dist = torch.ones(batch, 1, device=device).repeat(1, 8).view(-1, 1)
        near, far = (dist - dist_radius).unsqueeze(-1), (dist + dist_radius).unsqueeze(-1)
        fov = fov_ang * torch.ones(batch, 1, device=device).repeat(1, 8).view(-1, 1) * np.pi / 180
        focal = 0.5 * resolution / torch.tan(fov).unsqueeze(-1)
    else:
        if uniform:
            azim = -azim_range + 2 * azim_range * torch.rand(batch, 1, device=device)
            elev = -elev_range + 2 * elev_range * torch.rand(batch, 1, device=device)
        else:
            azim = azim_range * torch.randn(batch, 1, device=device)
            elev = elev_range * torch.randn(batch, 1, device=device)
        dist = torch.ones(batch, 1, device=device)
        near, far = (dist - dist_radius).unsqueeze(-1), (dist + dist_radius).unsqueeze(-1)
        fov = fov_ang * torch.ones(batch, 1, device=device) * np.pi / 180
        focal = 0.5 * resolution / torch.tan(fov).unsqueeze(-1)

    viewpoint = torch.cat([azim, elev], 1)
    x = torch.cos(elev) * torch.sin(azim)
    y = torch.sin(elev)
    z = torch.cos(elev) * torch.cos(azim)
    camera_dir = torch.stack([x, y, z], dim=1).view(-1, 3)
    camera_loc = dist * camera_dir

    up = torch.tensor([[0, 1, 0]]).float().to(device) * torch.ones_like(dist)
    z_axis = F.normalize(camera_dir, eps=1e-5)
    x_axis = F.normalize(torch.cross(up, z_axis, dim=1), eps=1e-5)
    y_axis = F.normalize(torch.cross(z_axis, x_axis, dim=1), eps=1e-5)
    is_close = torch.isclose(x_axis, torch.tensor(0.0), atol=5e-3).all(dim=1, keepdim=True)
    if is_close.any():
        repl = F.normalize(torch.cross(y_axis, z_axis, dim=1), eps=1e-5)
        x_axis = torch.where(is_close, repl, x_axis)
    R = torch.cat((x_axis[:, None, :], y_axis[:, None, :], z_axis[:, None, :]), dim=1)
    T = camera_loc[:, :, None]
    extrinsics = torch.cat((R.transpose(1, 2), T), -1)
    return extrinsics, focal, near, far, viewpoint


def _scaled_randn(n, scale, device):
    """scale * torch.randn(n, 1) as [n] in one launch: normal_(0, scale) makes the same
    draw (randn is normal_(0, 1)) and scales it in the sampling kernel by the same fp32
    product (x * scale + 0); tests/test_gpu_render.py pins the equality."""
    return torch.empty(n, device=device).normal_(0.0, scale)


def _camera_cuda(resolution, device, batch, locations, sweep, uniform, azim_range, elev_range,
                 fov_ang, dist_radius):
    """The GPU branch: the reference's random draws (same torch calls, same order, on
    the device), then every remaining op in one HIP launch (sdfr_camera_extrinsics) --
    ~25 elementwise / reduction kernels and the is_close.any() host sync of
    sdf_utils.py:151-154 replaced; capture-safe (no host sync, no host->device copy)."""
    from . import _lib
    if locations is not None:
        locations = locations.to(device, torch.float32)   # the kernel reads device memory
        azim = locations[:, 0].contiguous()
        elev = locations[:, 1].contiguous()
    elif sweep:
        azim = (-azim_range + (2 * azim_range / 7) * torch.arange(8, device=device))
        azim = azim.view(-1, 1).repeat(batch, 1).view(-1)
        elev = (-elev_range + 2 * elev_range *
                torch.rand(batch, 1, device=device).repeat(1, 8).view(-1))
    elif uniform:
        azim = (-azim_range + 2 * azim_range * torch.rand(batch, 1, device=device)).view(-1)
        elev = (-elev_range + 2 * elev_range * torch.rand(batch, 1, device=device)).view(-1)
    else:
        azim = _scaled_randn(batch, azim_range, device)
        elev = _scaled_randn(batch, elev_range, device)
    azim, elev = azim.float().contiguous(), elev.float().contiguous()
    n = azim.shape[0]
    ext = torch.empty(n, 3, 4, device=device)
    focal = torch.empty(n, 1, 1, device=device)
    near = torch.empty(n, 1, 1, device=device)
    far = torch.empty(n, 1, 1, device=device)
    vp = torch.empty(n, 2, device=device)
    _lib.check(_lib.lib().sdfr_camera_extrinsics(
        _lib.ptr(azim), _lib.ptr(elev), n, float(dist_radius), float(fov_ang),
        float(0.5 * resolution), _lib.ptr(ext), _lib.ptr(focal), _lib.ptr(near), _lib.ptr(far),
        _lib.ptr(vp), _lib.stream_of(azim)), "sdfr_camera_extrinsics")
    return ext, focal, near, far, vp
