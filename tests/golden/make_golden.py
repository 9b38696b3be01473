"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own code.

Run in the build container only (it reads /root/reference, which never reaches
the GPU box):

    python tests/golden/make_golden.py

What it does
------------
* Imports ``im2scene/sdf/models/sdf_model.py`` and ``sdf_utils.py`` from
  /root/reference under synthetic parent packages (their ``__init__`` files pull
  in torchvision-only encoder code), with inert stand-ins for the off-path
  third-party modules that are absent here (pytorch3d, torchvision, trimesh,
  lmdb, skimage, munch, configargparse) -- none of them is touched on the
  renderer / decoder code paths exercised below.
* ``sdf_op.py`` JIT-compiles CUDA at import; ``torch.utils.cpp_extension.load``
  is replaced by a no-op for the import so the file's own CPU branches
  (``sdf_op.py:106-117, 273-314``) run verbatim.
* The CUDA-only ``_gridencoder`` / ``_shencoder`` pybind modules are replaced by
  the C oracle (``oracle/csrc/sdfr_oracle.c``), so the reference's own
  ``grid.py`` / ``sphere_harmonics.py`` autograd wrappers run around it.
* Parameters come from ``oracle.det_uniform`` (integer-hash uniform), so the
  tests regenerate identical weights on any host without shipping them.

Everything written is data (inputs + expected outputs) in .npz files.
"""
from __future__ import annotations

import argparse
import importlib
import sys
import types
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
sys.dont_write_bytecode = True

from oracle import oracle  # noqa: E402
from tests.golden import weights as W  # noqa: E402


# ---------------------------------------------------------------- stubs
def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _Munch(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def copy(self):
        return _Munch(self)


class _CfgParser(argparse.ArgumentParser):
    def add_argument_group(self, *a, **k):
        g = super().add_argument_group(*a, **k)
        orig = g.add_argument

        def add(*aa, **kk):
            kk.pop("is_config_file", None)
            return orig(*aa, **kk)
        g.add_argument = add
        return g


def _install_stubs():
    noop = lambda *a, **k: None  # noqa: E731
    _stub("pytorch3d")
    _stub("pytorch3d.io")
    _stub("pytorch3d.structures", Meshes=object)
    _stub("pytorch3d.transforms", matrix_to_euler_angles=noop)
    _stub("pytorch3d.renderer", look_at_view_transform=noop, FoVPerspectiveCameras=object,
          PointLights=object, RasterizationSettings=object, MeshRenderer=object,
          MeshRasterizer=object, SoftPhongShader=object, TexturesVertex=object)
    _stub("torchvision")
    _stub("torchvision.transforms")
    _stub("torchvision.transforms.functional")
    _stub("trimesh")
    _stub("lmdb")
    _stub("skimage")
    _stub("skimage.measure", marching_cubes=noop)
    _stub("munch", Munch=_Munch, __all__=["Munch"])
    _stub("configargparse", ArgumentParser=_CfgParser)
    for pkg, path in [("im2scene", REF / "im2scene"), ("im2scene.sdf", REF / "im2scene/sdf"),
                      ("im2scene.sdf.models", REF / "im2scene/sdf/models")]:
        m = types.ModuleType(pkg)
        m.__path__ = [str(path)]
        sys.modules[pkg] = m


def _t2n(t):
    return t.detach().cpu().contiguous().numpy()


def _install_encoders():
    """The C oracle behind the reference's pybind names (gridencoder.h:11-16, shencoder.h:9-10)."""
    def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, dy_dx,
                            gridtype, align_corners, interp):
        per_level_scale = float(np.exp2(S))
        out, dd = oracle.grid_encode_forward(_t2n(inputs), _t2n(embeddings), _t2n(offsets),
                                             per_level_scale, H, dy_dx is not None, gridtype,
                                             align_corners, interp)
        outputs.copy_(torch.from_numpy(out))
        if dy_dx is not None:
            dy_dx.copy_(torch.from_numpy(dd))

    def grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L, S,
                             H, dy_dx, grad_inputs, gridtype, align_corners, interp):
        ge, gi = oracle.grid_encode_backward(_t2n(grad), _t2n(inputs), _t2n(embeddings),
                                             _t2n(offsets), float(np.exp2(S)), H,
                                             None if dy_dx is None else _t2n(dy_dx), gridtype,
                                             align_corners, interp)
        grad_embeddings.copy_(torch.from_numpy(ge))
        if grad_inputs is not None:
            grad_inputs.copy_(torch.from_numpy(gi))

    def sh_encode_forward(inputs, outputs, B, D, C, dy_dx):
        out, dd = oracle.sh_encode_forward(_t2n(inputs), C, dy_dx is not None)
        outputs.copy_(torch.from_numpy(out))
        if dy_dx is not None:
            dy_dx.copy_(torch.from_numpy(dd))

    def sh_encode_backward(grad, inputs, B, D, C, dy_dx, grad_inputs):
        gi = oracle.sh_encode_backward(_t2n(grad), _t2n(inputs), C, _t2n(dy_dx))
        grad_inputs.copy_(torch.from_numpy(gi))

    _stub("_gridencoder", grid_encode_forward=grid_encode_forward,
          grid_encode_backward=grid_encode_backward)
    _stub("_shencoder", sh_encode_forward=sh_encode_forward,
          sh_encode_backward=sh_encode_backward)


def import_reference():
    _install_stubs()
    _install_encoders()
    import torch.utils.cpp_extension as cx
    real_load = cx.load
    cx.load = lambda *a, **k: types.SimpleNamespace()
    try:
        sdf_model = importlib.import_module("im2scene.sdf.models.sdf_model")
        sdf_utils = importlib.import_module("im2scene.sdf.models.sdf_utils")
    finally:
        cx.load = real_load
    return sdf_model, sdf_utils


def make_opts(sdf_utils, size=256, n_samples=24, res=64, **render_kw):
    opt = sdf_utils.SDFOptions().parse(["--size", str(size), "--batch", "8", "--chunk", "2"])
    opt.model.freeze_renderer = True
    opt.model.psp = 0
    opt.model.renderer_spatial_output_dim = res
    opt.rendering.type = "ngp"
    opt.rendering.fc = 0
    opt.rendering.N_samples = n_samples
    for k, v in render_kw.items():
        opt.rendering[k] = v
    return opt


class _RandRecorder:
    """Records the CPU torch.rand draws the reference makes inside render_rays (sdf_model.py:331)."""

    def __init__(self):
        self.draws = []

    def __enter__(self):
        self.real = torch.rand

        def rand(*a, **k):
            t = self.real(*a, **k)
            self.draws.append(t.clone())
            return t
        torch.rand = rand
        return self

    def __exit__(self, *exc):
        torch.rand = self.real


# ---------------------------------------------------------------- cases
def case_encoders():
    offsets, pls = oracle.grid_offsets()
    emb = W.det_table(int(offsets[-1]), 2, seed=7)
    rng = np.random.default_rng(0)
    x = rng.uniform(0.0, 1.0, size=(4096, 3)).astype(np.float32)
    x[:8] = np.array([[0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.5], [-1e-7, 0.5, 0.5],
                      [0.5, 1.0000001, 0.5], [0.25, 0.75, 0.999999], [1e-30, 1e-30, 1e-30],
                      [0.3333333, 0.6666667, 0.1]], np.float32)
    import torch as T
    grid_mod = importlib.import_module("im2scene.sdf.models.gridencoder.grid")
    enc = grid_mod.GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                               log2_hashmap_size=19, desired_resolution=4096, gridtype="hash")
    enc.embeddings.data.copy_(T.from_numpy(emb))
    xin = T.from_numpy(x * 4 - 2)   # GridEncoder.forward maps (x+2)/4
    out = enc(xin, bound=2)
    xg = T.from_numpy(x).clone().requires_grad_(True)
    out_g = grid_mod.grid_encode(xg, enc.embeddings, enc.offsets, enc.per_level_scale, 16, True,
                                 0, False, 0)
    sh_mod = importlib.import_module("im2scene.sdf.models.shencoder.sphere_harmonics")
    dirs = rng.normal(size=(1024, 3)).astype(np.float32)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    dirs[0] = [0, 0, 1]
    shenc = sh_mod.SHEncoder(input_dim=3, degree=4)
    sh = shenc(T.from_numpy(dirs))
    np.savez_compressed(OUT / "encoders.npz", offsets=_t2n(enc.offsets),
                        per_level_scale=np.float64(enc.per_level_scale), grid_x=x,
                        grid_out_via_bound=_t2n(out), grid_out=_t2n(out_g), sh_dirs=dirs,
                        sh_out=_t2n(sh), table_seed=np.int64(7))
    print("encoders.npz", out.shape, sh.shape)


def case_sh_deg8():
    """SH encoder at degree 8 (shencoder.cu:27-355: outputs[0..63] and the dy_dx lambdas
    write_sh_dx / _dy / _dz).  The CUDA kernel cannot run here, so its formulas are read
    from the reference source and evaluated in float32 (numpy, one rounding per
    operation; nvcc may contract a*b+c, so the kernel itself can differ by an ulp).
    Stored: unit directions (plus the poles and axis points), outputs [B, 64] and
    dy_dx [B, 3, 64]."""
    import re
    src = (REF / "im2scene/sdf/models/shencoder/src/shencoder.cu").read_text()
    rx = re.compile(r"^\s*(outputs|dx|dy|dz)\[(\d+)\]\s*=\s*(.*?)\s*;", re.M)
    exprs = {"outputs": {}, "dx": {}, "dy": {}, "dz": {}}
    for name, idx, e in rx.findall(src):
        exprs[name][int(idx)] = re.sub(r"(\d+\.\d*(?:e[-+]?\d+)?)f", r"F(\1)", e)
    assert all(len(v) == 64 for v in exprs.values()), {k: len(v) for k, v in exprs.items()}
    rng = np.random.default_rng(8)
    d = rng.normal(size=(2048, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[:6] = np.array([[0, 0, 1], [0, 0, -1], [1, 0, 0], [0, 1, 0], [-1, 0, 0],
                      [0.6, 0.0, 0.8]], np.float32)
    F = np.float32
    x, y, z = (d[:, i].copy() for i in range(3))
    env = dict(F=F, pow=lambda a, n: np.power(a, np.float32(n)), x=x, y=y, z=z, xy=x * y, xz=x * z, yz=y * z, x2=x * x, y2=y * y, z2=z * z)
    env.update(xyz=env["xy"] * z, x4=env["x2"] * env["x2"], y4=env["y2"] * env["y2"],
               z4=env["z2"] * env["z2"])
    env.update(x6=env["x4"] * env["x2"], y6=env["y4"] * env["y2"], z6=env["z4"] * env["z2"])

    def ev(e):
        v = eval(e, {"__builtins__": {}}, env)       # reference arithmetic on float32 arrays
        return np.broadcast_to(np.asarray(v, np.float32), x.shape)
    out = np.stack([ev(exprs["outputs"][i]) for i in range(64)], 1)
    dydx = np.stack([np.stack([ev(exprs[k][i]) for i in range(64)], 1)
                     for k in ("dx", "dy", "dz")], 1)
    assert out.dtype == np.float32 and dydx.dtype == np.float32
    np.savez_compressed(OUT / "sh_deg8.npz", dirs=d, sh_out=out, dy_dx=dydx)
    print("sh_deg8.npz", out.shape, dydx.shape)


def case_camera(sdf_utils):
    res = {}
    for name, kw in [("gauss", {}), ("uniform", {"uniform": True}), ("sweep", {"sweep": True})]:
        torch.manual_seed(123)
        ext, focal, near, far, vp = sdf_utils.generate_camera_params(64, "cpu", batch=5, **kw)
        for k, v in zip(["ext", "focal", "near", "far", "vp"], [ext, focal, near, far, vp]):
            res[f"{name}_{k}"] = _t2n(v)
    # the last two rows look straight down / up: the degenerate-axis fix (:151-154)
    locs = torch.tensor([[0., 0.], [0.3, -0.1], [-0.45, 0.2], [0.2, np.pi / 2],
                         [-0.1, -np.pi / 2]])
    ext, focal, near, far, vp = sdf_utils.generate_camera_params(128, "cpu", batch=5, locations=locs)
    for k, v in zip(["ext", "focal", "near", "far", "vp"], [ext, focal, near, far, vp]):
        res[f"loc_{k}"] = _t2n(v)
    res["loc_locations"] = _t2n(locs)
    np.savez_compressed(OUT / "camera.npz", **res)
    print("camera.npz")


def _generator(sdf_model, sdf_utils, size=256, res=64, n_samples=24, full_pipeline=True,
               table_amp=1.0, train_renderer=False, **rk):
    opt = make_opts(sdf_utils, size=size, n_samples=n_samples, res=res, **rk)
    opt.model.freeze_renderer = not train_renderer
    g = sdf_model.Generator(opt.model, opt.rendering, full_pipeline=full_pipeline)
    W.det_init_(g, table_amp=table_amp)
    g.eval()
    return g, opt


def _cams(sdf_utils, B, res, seed):
    torch.manual_seed(seed)
    return sdf_utils.generate_camera_params(res, "cpu", batch=B)


def case_render(sdf_model, sdf_utils, name, B, res, n_samples, intermediates, seed, table_amp=1.0,
                **rk):
    g, opt = _generator(sdf_model, sdf_utils, res=res, n_samples=n_samples, full_pipeline=False,
                        table_amp=table_amp, **rk)
    ext, focal, near, far, vp = _cams(sdf_utils, B, res, seed)
    torch.manual_seed(seed + 1)
    z = torch.randn(B, 256)
    with torch.no_grad():
        latent = g.style(z)
        torch.manual_seed(seed + 2)
        with _RandRecorder() as rr:
            rgb, feat, sdf, mask, xyz, _ = g.renderer(ext, focal, near, far, styles=latent)
    t_rand = _t2n(rr.draws[0]) if rr.draws else np.zeros((0,), np.float32)
    d = dict(z=_t2n(z), ext=_t2n(ext), focal=_t2n(focal), near=_t2n(near), far=_t2n(far),
             latent=_t2n(latent), t_rand=t_rand, rgb=_t2n(rgb),
             render_opts=np.array(repr(dict(opt.rendering))), res=np.int64(res),
             n_samples=np.int64(n_samples), table_amp=np.float64(table_amp))
    if feat is not None:
        d["features"] = _t2n(feat)
    if sdf is not None:
        d["sdf"] = _t2n(sdf)
    if xyz is not None:
        d["xyz"] = _t2n(xyz)
        d["mask"] = _t2n(mask)
    if intermediates:
        # re-run the reference's building blocks for the intermediate tensors
        r = g.renderer
        with torch.no_grad():
            rays_o, rays_d, viewdirs = r.get_rays(focal, ext)
            viewdirs = viewdirs / torch.norm(viewdirs, dim=-1, keepdim=True)
            nr = near.unsqueeze(-1) * torch.ones_like(rays_d[..., :1])
            fr = far.unsqueeze(-1) * torch.ones_like(rays_d[..., :1])
            zv = nr * (1. - r.t_vals) + fr * r.t_vals
            if r.perturb > 0:
                upper = torch.cat([zv[..., 1:], fr], -1)
                zv = zv + (upper - zv) * torch.from_numpy(t_rand).unsqueeze(-1)
            pts = rays_o.unsqueeze(3) + rays_d.unsqueeze(3) * zv.unsqueeze(-1)
            npts = pts * 2 / ((fr - nr).unsqueeze(3))
            gin = (npts + 2) / 4
            raw = r.run_network(npts, viewdirs, styles=latent)
        d.update(rays_d=_t2n(rays_d), viewdirs=_t2n(viewdirs), z_vals=_t2n(zv), pts=_t2n(pts),
                 grid_in=_t2n(gin), raw=_t2n(raw))
    np.savez_compressed(OUT / f"{name}.npz", **d)
    print(f"{name}.npz", rgb.shape)


def case_mesh(sdf_model, sdf_utils):
    """sdf_mesh.py's surface extractor (sdf_mesh.py:244-252: renderer at 128^2 rays x
    128 samples, return_sdf/xyz, full_pipeline=False) on one face, plus
    sdf_utils.align_volume (:164-184) on its SDF volume and on a small random one.
    The 128^3 SDF is stored on every 8th pixel row/column (all samples)."""
    g, opt = _generator(sdf_model, sdf_utils, res=128, n_samples=128, full_pipeline=False,
                        return_sdf=True, return_xyz=True)
    ext, focal, near, far, vp = _cams(sdf_utils, 1, 128, 51)
    torch.manual_seed(52)
    z = torch.randn(1, 256)
    with torch.no_grad():
        torch.manual_seed(53)
        with _RandRecorder() as rr:
            out = g([z], ext, focal, near, far, return_sdf=True, return_xyz=True)
        _, thumb, xyz, sdf, mask = out
        aligned = sdf_utils.align_volume(sdf)
        torch.manual_seed(54)
        vol = torch.randn(1, 12, 10, 16, 1)   # align_volume supports batch 1 only
        vol_aligned = sdf_utils.align_volume(vol)
    sub = slice(0, None, 8)
    np.savez_compressed(OUT / "mesh128.npz", z=_t2n(z), ext=_t2n(ext), focal=_t2n(focal),
                        near=_t2n(near), far=_t2n(far), t_rand=_t2n(rr.draws[0]),
                        thumb=_t2n(thumb), xyz=_t2n(xyz), mask=_t2n(mask),
                        sdf_sub=_t2n(sdf[:, sub, sub]), aligned_sub=_t2n(aligned[:, sub, sub]),
                        vol=_t2n(vol), vol_aligned=_t2n(vol_aligned), res=np.int64(128),
                        n_samples=np.int64(128))
    print("mesh128.npz", sdf.shape, aligned.shape)


def case_mesh256(sdf_model, sdf_utils):
    """BASELINE configs[3]: sdf_mesh.py's surface query at 256^2 rays x 256 samples
    (sdf_mesh.py:243-252 with 256 for its 128; the options of :211-214: static
    viewdirs, force_background, perturb 0) on every 16th pixel row and column.  The
    reference's own get_rays runs at the full 256^2 resolution; its rays are then
    subsampled before render_rays, which treats every ray independently -- so the
    stored 16 x 16 x 256 SDF values are exactly those of the full 256^3 volume."""
    g, opt = _generator(sdf_model, sdf_utils, res=256, n_samples=256, full_pipeline=False,
                        return_sdf=True, return_xyz=True, static_viewdirs=True,
                        force_background=True, perturb=0)
    r = g.renderer
    full_get_rays = r.get_rays
    sub = slice(0, None, 16)
    r.get_rays = lambda focal, c2w: tuple(t[:, sub, sub] for t in full_get_rays(focal, c2w))
    ext, focal, near, far, vp = _cams(sdf_utils, 1, 256, 61)
    torch.manual_seed(62)
    z = torch.randn(1, 256)
    with torch.no_grad():
        _, thumb, xyz, sdf, mask = g([z], ext, focal, near, far, return_sdf=True,
                                     return_xyz=True)
    np.savez_compressed(OUT / "mesh256_sub.npz", z=_t2n(z), ext=_t2n(ext), focal=_t2n(focal),
                        near=_t2n(near), far=_t2n(far), thumb_sub=_t2n(thumb),
                        xyz_sub=_t2n(xyz), mask_sub=_t2n(mask), sdf_sub=_t2n(sdf),
                        stride=np.int64(16), res=np.int64(256), n_samples=np.int64(256))
    print("mesh256_sub.npz", tuple(sdf.shape))


def case_siren(sdf_model, sdf_utils):
    """rendering.type == 'sdf' (SirenGenerator, 100 % reference code on CPU)."""
    case_render(sdf_model, sdf_utils, "render_siren_small", B=2, res=8, n_samples=24,
                intermediates=False, seed=61, type="sdf")
    case_render(sdf_model, sdf_utils, "render_siren_mesh_opts", B=1, res=8, n_samples=32,
                intermediates=False, seed=71, type="sdf", static_viewdirs=True,
                force_background=True, perturb=0, return_sdf=True, return_xyz=True)
    case_render(sdf_model, sdf_utils, "render_siren_face32", B=1, res=32, n_samples=24,
                intermediates=False, seed=81, type="sdf", return_sdf=True, return_xyz=True)
    g, _ = _generator(sdf_model, sdf_utils, res=8, n_samples=24, full_pipeline=False, type="sdf")
    sd = g.state_dict()
    shapes = np.array([repr((k, tuple(sd[k].shape))) for k in sorted(sd)])
    np.savez_compressed(OUT / "state_dict_keys_siren.npz", entries=shapes)
    print("state_dict_keys_siren.npz", len(shapes), "keys")


def case_table_scales(sdf_model, sdf_utils):
    """The hash table at the reference's own init scale U(-1e-4, 1e-4) (grid.py:138-140)
    and at a trained-like U(-0.05, 0.05): the operand scales the split-fp16 field
    kernel meets in practice (the other fixtures use U(-1, 1) to expose index errors)."""
    for tag, amp in (("tab1e4", 1e-4), ("tab05", 0.05)):
        case_render(sdf_model, sdf_utils, f"render_small_{tag}", B=2, res=8, n_samples=24,
                    intermediates=False, seed=111, table_amp=amp)
        case_render(sdf_model, sdf_utils, f"render_face64_{tag}", B=1, res=64, n_samples=24,
                    intermediates=False, seed=141, table_amp=amp)


def _stage1_generator(sdf_model, sdf_utils, res, n_samples, table_amp=1.0, **rk):
    """Stage-1 configuration (training_utils.py:150-161): renderer trained, sdf returned
    (min_surf_lambda > 0), no feature output, Generator(full_pipeline=False)."""
    return _generator(sdf_model, sdf_utils, res=res, n_samples=n_samples, full_pipeline=False,
                      table_amp=table_amp, train_renderer=True, no_features_output=True,
                      return_sdf=True, **rk)


def case_eikonal(sdf_model, sdf_utils):
    """Stage-1 forward with return_sdf / return_eikonal (training_utils.py:411-413): the
    eikonal term d sdf / d pts (sdf_model.py:224-229) through the grid encoder's
    dy_dx (grid.py:44-52), plus the gradients a stage-1 style loss sends into the
    network.  Reference semantics: the custom backward writes grad_inputs through the
    CUDA op, outside autograd, so the eikonal term is a constant (requires_grad False)
    and the eikonal loss reaches no parameter."""
    res, N, B = 8, 24, 2
    g, opt = _stage1_generator(sdf_model, sdf_utils, res, N, table_amp=0.05)
    ext, focal, near, far, vp = _cams(sdf_utils, B, res, 91)
    torch.manual_seed(92)
    z = torch.randn(B, 256)
    torch.manual_seed(93)
    with _RandRecorder() as rr:
        _, thumb, sdf, eik = g([z], ext, focal, near, far, return_sdf=True,
                               return_eikonal=True)
    eik_loss = ((eik.norm(dim=-1) - 1) ** 2).mean()
    surf = torch.exp(-100 * torch.abs(sdf)).mean()
    loss = thumb.mean() + surf + (eik_loss if eik_loss.requires_grad else 0)
    loss.backward()
    net = g.renderer.network
    n_dense = int(net.encoder.offsets[2])                  # levels 0-1: dense rows
    # the hashed levels (5-15, grid.py:117-128): every 4th row that received gradient
    gt = net.encoder.embeddings.grad
    first_hashed = int(net.encoder.offsets[5])
    hit = torch.nonzero(gt[first_hashed:].abs().sum(1) > 0).flatten() + first_hashed
    hashed_rows = hit[::4].numpy().astype(np.int64)
    np.savez_compressed(
        OUT / "eikonal.npz", z=_t2n(z), ext=_t2n(ext), focal=_t2n(focal), near=_t2n(near),
        far=_t2n(far), t_rand=_t2n(rr.draws[0]), thumb=_t2n(thumb), sdf=_t2n(sdf),
        eikonal=_t2n(eik), eik_requires_grad=np.bool_(eik.requires_grad),
        eik_loss=np.float64(eik_loss.item()),
        grad_sigma_w=_t2n(net.sigma_linear.weight.grad),
        grad_input_w=_t2n(net.input_linear.weight.grad),
        grad_beta=_t2n(g.renderer.sigmoid_beta.grad),
        grad_table_dense=_t2n(net.encoder.embeddings.grad[:n_dense]),
        grad_table_hashed_rows=hashed_rows, grad_table_hashed=_t2n(gt[hashed_rows]),
        res=np.int64(res), n_samples=np.int64(N), table_amp=np.float64(0.05))
    print("eikonal.npz", tuple(eik.shape), "eik requires_grad:", eik.requires_grad)


def case_eikonal_siren(sdf_model, sdf_utils):
    """Stage-1 forward of the SIREN network (rendering.type 'sdf', configs[4]) with
    return_eikonal: here the eikonal term d sdf / d pts (sdf_model.py:224-229) is an
    autograd.grad(create_graph=True) through the FiLM MLP itself (:101-139), so the
    eikonal loss reaches every pts_linears parameter through a double backward.  The
    gradients of thumb + surface + eikonal loss (training_utils.py:396-451) are kept
    for layers on every path: first, middle and last FiLM layers (weight, bias and
    the gamma / beta style layers), the views layer and both heads."""
    res, N, B = 8, 24, 2
    g, opt = _stage1_generator(sdf_model, sdf_utils, res, N, type="sdf")
    ext, focal, near, far, vp = _cams(sdf_utils, B, res, 191)
    torch.manual_seed(192)
    z = torch.randn(B, 256)
    torch.manual_seed(193)
    with _RandRecorder() as rr:
        _, thumb, sdf, eik = g([z], ext, focal, near, far, return_sdf=True,
                               return_eikonal=True)
    eik_loss = ((eik.norm(dim=-1) - 1) ** 2).mean()
    surf = torch.exp(-100 * torch.abs(sdf)).mean()
    loss = thumb.mean() + surf + 0.1 * eik_loss
    loss.backward()
    net = g.renderer.network
    grads = {}
    for name, prm in net.named_parameters():
        if any(name.startswith(p) for p in ("pts_linears.0.", "pts_linears.3.", "pts_linears.7.",
                                            "views_linears.", "sigma_linear.", "rgb_linear.")):
            grads["grad__" + name.replace(".", "__")] = _t2n(prm.grad)
    np.savez_compressed(
        OUT / "eikonal_siren.npz", z=_t2n(z), ext=_t2n(ext), focal=_t2n(focal), near=_t2n(near),
        far=_t2n(far), t_rand=_t2n(rr.draws[0]), thumb=_t2n(thumb), sdf=_t2n(sdf),
        eikonal=_t2n(eik), eik_requires_grad=np.bool_(eik.requires_grad),
        eik_loss=np.float64(eik_loss.item()), grad_beta=_t2n(g.renderer.sigmoid_beta.grad),
        res=np.int64(res), n_samples=np.int64(N), **grads)
    print("eikonal_siren.npz", tuple(eik.shape), "eik requires_grad:", eik.requires_grad,
          len(grads), "gradients")


def case_init_pass(sdf_model, sdf_utils):
    """Sphere initialisation (training_utils.py:287-317): Generator.init_forward ->
    mlp_init_pass (sdf_model.py:380-409, 1156-1161) with its stratified torch.rand
    draw captured, and the L1 loss's gradients."""
    res, N, B = 8, 24, 3
    g, opt = _stage1_generator(sdf_model, sdf_utils, res, N, table_amp=0.05)
    ext, focal, near, far, vp = _cams(sdf_utils, B, res, 95)
    torch.manual_seed(96)
    z = torch.randn(B, 256)
    torch.manual_seed(97)
    with _RandRecorder() as rr:
        sdf, target = g.init_forward([z], ext, focal, near, far)
    loss = torch.nn.functional.l1_loss(sdf, target)
    loss.backward()
    net = g.renderer.network
    np.savez_compressed(
        OUT / "init_pass.npz", z=_t2n(z), ext=_t2n(ext), focal=_t2n(focal), near=_t2n(near),
        far=_t2n(far), t_rand=_t2n(rr.draws[0]), sdf=_t2n(sdf), target=_t2n(target),
        loss=np.float64(loss.item()), grad_sigma_w=_t2n(net.sigma_linear.weight.grad),
        grad_input_w=_t2n(net.input_linear.weight.grad),
        res=np.int64(res), n_samples=np.int64(N), table_amp=np.float64(0.05))
    print("init_pass.npz", tuple(sdf.shape), f"loss {loss.item():.5f}")


def case_fc(sdf_model, sdf_utils):
    """rendering.fc = 1 with type 'sdf': the positional-encoding ReLU MLP FCGenerator
    (sdf_model.py:197-200, 1599-1670), 100 % reference code on CPU."""
    case_render(sdf_model, sdf_utils, "render_fc_small", B=2, res=8, n_samples=24,
                intermediates=False, seed=151, type="sdf", fc=1, return_sdf=True,
                return_xyz=True)
    g, _ = _generator(sdf_model, sdf_utils, res=8, n_samples=24, full_pipeline=False, type="sdf",
                      fc=1)
    sd = g.state_dict()
    shapes = np.array([repr((k, tuple(sd[k].shape))) for k in sorted(sd)])
    np.savez_compressed(OUT / "state_dict_keys_fc.npz", entries=shapes)
    print("state_dict_keys_fc.npz", len(shapes), "keys")


def case_generator(sdf_model, sdf_utils):
    g, opt = _generator(sdf_model, sdf_utils, size=256, res=64, n_samples=24)
    ext, focal, near, far, vp = _cams(sdf_utils, 1, 64, 31)
    torch.manual_seed(32)
    z = torch.randn(1, 256)
    with torch.no_grad():
        torch.manual_seed(33)
        with _RandRecorder() as rr:
            rgb, thumb = g([z], ext, focal, near, far, randomize_noise=False)
        # decoder alone on fixed features (isolates the StyleGAN2 part)
        latent = g.style(z)
        torch.manual_seed(34)
        feats = torch.randn(1, 256, 64, 64) * 0.3
        img, _ = g.decoder(feats, [latent], randomize_noise=False)
        # mean_latent(n, device, z=...) raises UnboundLocalError in the reference
        # (sdf_model.py:1127-1130); the z=None branch draws z from the CPU RNG.
        torch.manual_seed(99)
        mean_z = torch.randn(64, 256)
        torch.manual_seed(99)
        mean = g.mean_latent(64, "cpu")
    np.savez_compressed(OUT / "generator.npz", z=_t2n(z), ext=_t2n(ext), focal=_t2n(focal),
                        near=_t2n(near), far=_t2n(far), t_rand=_t2n(rr.draws[0]),
                        rgb=_t2n(rgb), thumb=_t2n(thumb), dec_feats=_t2n(feats),
                        dec_latent=_t2n(latent), dec_img=_t2n(img),
                        mean_z=_t2n(mean_z),
                        mean_renderer=_t2n(mean[0]), mean_decoder=_t2n(mean[1]))
    keys = sorted(g.state_dict().keys())
    shapes = np.array([repr((k, tuple(g.state_dict()[k].shape))) for k in keys])
    np.savez_compressed(OUT / "state_dict_keys.npz", entries=shapes)
    print("generator.npz", rgb.shape, thumb.shape, len(keys), "keys")


def case_init_stats(sdf_model, sdf_utils):
    """Parameter statistics of a seeded random-init reference Generator (the
    drop-in must consume the CPU RNG identically)."""
    opt = make_opts(sdf_utils, size=256, n_samples=24, res=64)
    torch.manual_seed(0)
    g = sdf_model.Generator(opt.model, opt.rendering)
    names, stats = [], []
    for k, v in g.state_dict().items():
        if not torch.is_floating_point(v):
            continue
        v64 = v.double().reshape(-1)
        names.append(k)
        stats.append([v64.sum().item(), (v64 * v64).sum().item(), v64[0].item(), v64[-1].item()])
    np.savez_compressed(OUT / "init_stats.npz", names=np.array(names), stats=np.array(stats),
                        param_order=np.array([k for k, _ in g.named_parameters()]))
    print("init_stats.npz", len(names))


def main():
    sdf_model, sdf_utils = import_reference()
    if len(sys.argv) > 1:                       # selected cases only, e.g. `mesh`
        import inspect
        for name in sys.argv[1:]:
            fn = globals()[f"case_{name}"]
            args = (sdf_model, sdf_utils)
            n = len(inspect.signature(fn).parameters)
            fn(*args[2 - n:] if n else ())
        return
    case_init_stats(sdf_model, sdf_utils)
    case_encoders()
    case_sh_deg8()
    case_camera(sdf_utils)
    case_render(sdf_model, sdf_utils, "render_small", B=2, res=8, n_samples=24,
                intermediates=True, seed=11)
    case_render(sdf_model, sdf_utils, "render_mesh_opts", B=1, res=8, n_samples=32,
                intermediates=False, seed=21, static_viewdirs=True, force_background=True,
                perturb=0, return_sdf=True, return_xyz=True)
    case_render(sdf_model, sdf_utils, "render_face64", B=1, res=64, n_samples=24,
                intermediates=False, seed=41, return_sdf=True, return_xyz=True)
    case_generator(sdf_model, sdf_utils)
    case_mesh(sdf_model, sdf_utils)
    case_mesh256(sdf_model, sdf_utils)
    case_siren(sdf_model, sdf_utils)
    case_table_scales(sdf_model, sdf_utils)
    case_eikonal(sdf_model, sdf_utils)
    case_eikonal_siren(sdf_model, sdf_utils)
    case_init_pass(sdf_model, sdf_utils)
    case_fc(sdf_model, sdf_utils)


if __name__ == "__main__":
    main()
