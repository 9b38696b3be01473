"""Surface extraction helpers of sdf_mesh.py (im2scene/sdf/models/sdf_utils.py:164-223).

The SDF volume itself comes from the fused renderer: sdf_mesh.py builds a second
Generator at 128^2 rays x 128 samples with return_sdf / return_xyz
(sdf_mesh.py:244-252), whose forward runs ``sdfr_render_ngp_forward`` like any
other render and returns the per-sample SDF as a [B, H, W, N, 1] volume.
``align_volume`` resamples that frustum-shaped volume onto a cube (device-side
``grid_sample``, any device).  Marching cubes stays on the host: it needs
scikit-image (and trimesh for the .obj export), which this image does not ship,
so ``extract_mesh_with_marching_cubes`` raises ImportError naming them.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def align_volume(volume: torch.Tensor, near: float = 0.88, far: float = 1.12) -> torch.Tensor:
    """Frustum -> cube resampling of an SDF volume [1, H, W, D, C] (sdf_utils.py:164).

    The x/y sampling coordinates of depth slice k are scaled by
    linspace(far/near, 1, D)[k]; trilinear grid_sample with border padding and
    align_corners; cube cells whose scaled coordinate leaves [-1, 1] are set to 1
    so marching cubes sees "outside" there.  As in the reference the sampling grid
    has batch 1, so only single-volume batches are accepted (grid_sample raises
    otherwise).
    """
    b, h, w, d, c = volume.shape
    dev = volume.device
    # the 1-D linspaces come from the CPU (the reference's values, bit for bit);
    # the h*w*d grid is formed on the volume's device -- built on the host it
    # was a 200 MB copy per 256^3 volume (52 ms)
    lin = [torch.linspace(-1, 1, n).to(dev) for n in (h, w, d)]
    yy, xx, zz = torch.meshgrid(lin[0], lin[1], lin[2], indexing="ij")
    grid = torch.stack([xx, yy, zz], -1).unsqueeze(0)                     # [1,h,w,d,3]
    scale = torch.linspace(far / near, 1, d).view(1, 1, 1, -1, 1).to(dev)
    grid[..., :2] = grid[..., :2] * scale
    outside = torch.any(grid.lt(-1).logical_or(grid.gt(1)), -1, keepdim=True)
    sampled = F.grid_sample(volume.permute(0, 4, 3, 1, 2).contiguous(),
                            grid.permute(0, 3, 1, 2, 4).contiguous(),
                            padding_mode="border", align_corners=True)
    out = sampled.permute(0, 3, 4, 2, 1).contiguous()
    if out.shape[-1] != 1:
        out[outside] = 1            # the reference's boolean-index path (and its errors)
    else:
        out.masked_fill_(outside, 1.0)   # same cells, no host sync
    return out


def extract_mesh_with_marching_cubes(sdf: torch.Tensor):
    """Zero level set of an aligned SDF volume [1, H, W, D, 1] (sdf_utils.py:188).
    Returns a trimesh.Trimesh like the reference; needs scikit-image + trimesh."""
    try:
        from skimage.measure import marching_cubes
        import trimesh
    except ImportError as e:  # pragma: no cover - depends on the host image
        raise ImportError("extract_mesh_with_marching_cubes needs scikit-image and trimesh "
                          f"(host-side marching cubes): {e}") from e
    b, h, w, d, _ = sdf.shape
    vol = sdf[0, ..., 0].permute(1, 0, 2).cpu().numpy()
    verts, faces, _, _ = marching_cubes(vol, 0)
    verts[:, 0] = (verts[:, 0] / float(w) - 0.5) * 0.24
    verts[:, 1] = (verts[:, 1] / float(h) - 0.5) * 0.24
    verts[:, 2] = (verts[:, 2] / float(d) - 0.5) * 0.24
    verts[:, 2] *= -1
    verts[:, 1] *= -1
    return trimesh.Trimesh(verts, faces)


def xyz2mesh(xyz: torch.Tensor):
    """Mesh from an expected-surface xyz map [1, 3, H, W] (sdf_utils.py:209):
    Delaunay triangulation of the pixel grid, normals inverted.  Returns
    (vertices [H*W, 3], faces) or a trimesh.Trimesh when trimesh is present."""
    from scipy.spatial import Delaunay
    _, _, h, w = xyz.shape
    x, y = np.meshgrid(np.arange(h), np.arange(w))
    tri = Delaunay(np.concatenate((x.reshape(h * w, 1), y.reshape(h * w, 1)), 1))
    faces = tri.simplices
    faces[:, [0, 1]] = faces[:, [1, 0]]
    verts = xyz.squeeze(0).permute(1, 2, 0).reshape(h * w, 3).cpu().numpy()
    try:
        import trimesh
    except ImportError:
        return verts, faces
    return trimesh.Trimesh(verts, faces)
