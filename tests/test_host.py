"""CPU: the C-ABI library, the drop-in module surface and the PyTorch parts."""
import ast
import ctypes
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from tests.golden import weights as W

REPO = Path(__file__).resolve().parents[1]


def header_symbols(ablation=False):
    """Functions include/sdfr.h declares: the product ones, or (ablation=True) only
    those of its `#ifdef SDFR_ABLATION` block (profiling builds)."""
    txt = (REPO / "include" / "sdfr.h").read_text()
    blocks = re.findall(r"#ifdef SDFR_ABLATION\n(.*?)#endif", txt, re.S)
    if ablation:
        txt = "\n".join(blocks)
    else:
        txt = re.sub(r"#ifdef SDFR_ABLATION\n.*?#endif", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char \*)\s*(sdfr_\w+)\s*\(", txt, re.M)))


def library_symbols(path):
    """Global text symbols with the sdfr_ prefix that a shared library exports."""
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], capture_output=True,
                         text=True, check=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines()
                   if ln.split()[-2:-1] == ["T"] and ln.split()[-1].startswith("sdfr_")})


def test_library_exports_every_header_symbol(sdfr):
    lib = sdfr._lib.lib()
    syms = header_symbols()
    assert len(syms) >= 9
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(sdfr._lib.EXPORTS)
    assert lib.sdfr_abi_version() == sdfr._lib.ABI_VERSION
    # the product library exports exactly the documented entry points: no profiling
    # hooks (process-global state) outside `make ABLATION=1` builds
    assert library_symbols(sdfr._lib.LIB_PATH) == syms
    assert header_symbols(ablation=True) == sorted(sdfr._lib.ABLATION_EXPORTS)
    for s in sdfr._lib.ABLATION_EXPORTS:
        assert not hasattr(lib, s), s


def test_argument_errors_mirror_reference(sdfr):
    """Rejections happen before any launch, so they are checkable without a GPU."""
    lib = sdfr._lib.lib()
    nul = None
    rc = lib.sdfr_grid_encode_forward(nul, nul, nul, nul, 4, 3, 3, 16, 0.5, 16, nul, 0, 0, 0, nul)
    assert rc == sdfr._lib.SDFR_EINVAL
    assert b"C must be 1, 2, 4, or 8" in lib.sdfr_last_error()
    rc = lib.sdfr_grid_encode_forward(nul, nul, nul, nul, 4, 6, 2, 16, 0.5, 16, nul, 0, 0, 0, nul)
    assert rc == sdfr._lib.SDFR_EINVAL
    rc = lib.sdfr_sh_encode_forward(nul, nul, 4, 2, 4, nul, nul)
    assert rc == sdfr._lib.SDFR_EINVAL and b"input dim == 3" in lib.sdfr_last_error()
    rc = lib.sdfr_sh_encode_forward(nul, nul, 4, 3, 9, nul, nul)
    assert rc == sdfr._lib.SDFR_EINVAL
    rc = lib.sdfr_sh_encode_forward(nul, nul, 4, 3, 6, nul, nul)   # degrees 5..8 exist:
    assert rc == sdfr._lib.SDFR_EINVAL and b"null tensor" in lib.sdfr_last_error()
    w, a = sdfr._lib.NgpWeights(), sdfr._lib.NgpRenderArgs()
    rc = lib.sdfr_render_ngp_forward(ctypes.byref(w), ctypes.byref(a), nul)
    assert rc in (sdfr._lib.SDFR_EINVAL, sdfr._lib.SDFR_EUNSUPPORTED)
    with pytest.raises(RuntimeError, match="sdfr_render_ngp_forward"):
        sdfr._lib.check(rc, "sdfr_render_ngp_forward")


def test_workspace_size(sdfr):
    lib = sdfr._lib.lib()
    n = lib.sdfr_render_ngp_workspace_bytes(2, 64, 64, 24, 16)
    enc = 2 * 4096 * 24 * 16 * 2 * 4
    fixed = 67 * 1024 * 16 + 2 * 8 * 256 * 4          # fp32 fragments + FiLM vectors
    # split-fp16 fragments (51 slices of one 16-K k-step: layer 0 = input_linear o
    # pts_linears.0), su, bias_s, the composed layer 0 (W [256][32] | b [256])
    xfixed = 51 * 1024 * 16 + 2 * 4 * 256 * 4 + 33 * 256 * 4
    zd = 2 * 4096 * 24 * (2 + 4) * 4                   # per-sample (z, segment length), (u, inside)
    # 2 faces = 128 workgroups of 4 tiles: rays split in 2 sample segments, partials of
    # (256 features + rgb, xyz, T, w_last) per segment and ray
    part2 = 2 * (256 + 8) * 2 * 4096 * 4
    assert enc + fixed + xfixed + zd + part2 <= n <= enc + fixed + xfixed + zd + part2 + 1536
    # 1 face = 64 workgroups: 4 sample segments
    n1 = lib.sdfr_render_ngp_workspace_bytes(1, 64, 64, 24, 16)
    part = 4 * (256 + 8) * 4096 * 4
    base1 = enc // 2 + 67 * 1024 * 16 + 8 * 256 * 4 + xfixed + zd // 2
    assert base1 + part <= n1 <= base1 + part + 1536
    n32 = lib.sdfr_render_ngp_workspace_bytes(32, 64, 64, 24, 16)   # >= 256 workgroups: no split
    assert n32 <= 16 * (enc + zd) + fixed + 32 * 8 * 256 * 4 + xfixed + 1536
    # the per-call sample-split bound is validated before anything is launched
    w, a = sdfr._lib.NgpWeights(), sdfr._lib.NgpRenderArgs()
    w.num_levels, a.B, a.H, a.W, a.N = 16, 1, 8, 8, 24
    for bad in (3, 5, 8):
        a.max_field_segments = bad
        assert lib.sdfr_render_ngp_forward(ctypes.byref(w), ctypes.byref(a), None) == \
            sdfr._lib.SDFR_EINVAL
        assert b"max_field_segments" in lib.sdfr_last_error()


def test_conv_split_k_workspace(sdfr):
    """Split-K decisions of the decoder convolutions (host arithmetic, no launch):
    a workspace only when the unsplit grid leaves CUs idle, sized ksplit x slots x one
    128 x 256 fp32 partial tile; the factor is the largest of 4, 3, 2 whose split grid
    stays within 320 workgroups (1.25 rounds of the 256 CUs)."""
    lib = sdfr._lib.lib()
    tile = 16 * 512 * 16
    assert lib.sdfr_conv_ws_bytes(32, 64, 64, 512, 0) == 0            # 2048 workgroups
    assert lib.sdfr_conv_ws_bytes(1, 64, 64, 512, 0) == 4 * 64 * tile  # 64 -> 4 x 64
    assert lib.sdfr_conv_ws_bytes(1, 128, 128, 256, 0) == 2 * 128 * tile
    assert lib.sdfr_conv_ws_bytes(5, 64, 64, 128, 0) == 4 * 80 * tile  # 80 slots: 4-way split
    assert lib.sdfr_conv_ws_bytes(6, 64, 64, 128, 0) == 3 * 96 * tile  # 96 slots: 3-way split
    assert lib.sdfr_conv_act_ws_bytes(1, 64, 64, 512) == lib.sdfr_conv_ws_bytes(1, 64, 64, 512, 0)
    # transposed: four parity classes (17x17, 17x16, 16x17, 16x16 at 16^2), 8-padded
    assert lib.sdfr_conv_ws_bytes(1, 16, 16, 128, 1) == 4 * 32 * tile
    assert lib.sdfr_conv_ws_bytes(1, 64, 64, 256, 1) == 2 * 152 * tile  # 152 slots: 2-way
    assert lib.sdfr_conv_ws_bytes(1, 128, 128, 128, 1) == 0           # 280 slots: no split
    # 32 faces: conv_t_kernel (its edge classes unsplit: SDFR_EDGE_SPLIT off)
    assert lib.sdfr_conv_ws_bytes(32, 64, 64, 256, 1) == 0
    assert lib.sdfr_conv_ws_bytes(1, 64, 64, 100, 1) == 0             # Cout % 128


def test_fused_decoder_batch_chunk(sdfr):
    """Faces per fused decoder call (host arithmetic): the largest per-face activation
    of the 64^2 -> 256^2 decoder is the 257^2 x 128 raw output of the last transposed
    convolution, so 63 faces stay under the kernels' 2^31-byte offsets; the split-NHWC
    features the renderer hands over give the same bound."""
    opt = sdfr.vol_render_opt()
    opt.model.feature_encoder_in_channels = opt.rendering.width
    dec = sdfr.Decoder(opt.model)
    seq = [dec.conv1] + list(dec.convs)
    assert dec._fused_chunk(torch.empty(1, 256, 64, 64, device="meta"), seq) == 63
    assert dec._fused_chunk(torch.empty(1, 64, 64, 32, 2, 8, device="meta"), seq) == 63
    assert (2 ** 31 - 1) // (257 * 257 * 128 * 4) == 63


def test_state_dict_matches_reference(sdfr, golden_dir):
    opt = sdfr.vol_render_opt()
    g = sdfr.Generator(opt.model, opt.rendering)
    mine = {k: tuple(v.shape) for k, v in g.state_dict().items()}
    ref = dict(W.golden_entries(golden_dir))
    assert mine == ref


def test_siren_state_dict_matches_reference(sdfr, golden_dir):
    opt = sdfr.vol_render_opt(ngp=False)
    g = sdfr.Generator(opt.model, opt.rendering, full_pipeline=False)
    mine = {k: tuple(v.shape) for k, v in g.state_dict().items()}
    assert mine == dict(W.golden_entries(golden_dir, siren=True))


def test_seeded_init_identical_to_reference(sdfr, golden_dir):
    z = np.load(golden_dir / "init_stats.npz")
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering)
    sd = g.state_dict()
    for k, st in zip(z["names"], z["stats"]):
        v = sd[str(k)].double().reshape(-1)
        mine = [v.sum().item(), (v * v).sum().item(), v[0].item(), v[-1].item()]
        np.testing.assert_allclose(mine, st, rtol=1e-12, atol=1e-12, err_msg=str(k))
    assert [k for k, _ in g.named_parameters()] == list(z["param_order"])


def test_camera_matches_reference(sdfr, golden_dir):
    g = np.load(golden_dir / "camera.npz")
    for name, kw in [("gauss", {}), ("uniform", {"uniform": True}), ("sweep", {"sweep": True})]:
        torch.manual_seed(123)
        out = sdfr.generate_camera_params(64, "cpu", batch=5, **kw)
        for k, v in zip(["ext", "focal", "near", "far", "vp"], out):
            np.testing.assert_array_equal(v.numpy(), g[f"{name}_{k}"], err_msg=f"{name}_{k}")
    locs = torch.from_numpy(g["loc_locations"])
    out = sdfr.generate_camera_params(128, "cpu", batch=locs.shape[0], locations=locs)
    for k, v in zip(["ext", "focal", "near", "far", "vp"], out):
        np.testing.assert_array_equal(v.numpy(), g[f"loc_{k}"])


@pytest.fixture(scope="module")
def det_generator(sdfr):
    opt = sdfr.vol_render_opt()
    g = sdfr.Generator(opt.model, opt.rendering)
    W.det_init_(g)
    return g.eval()


def test_decoder_matches_reference(det_generator, golden_dir):
    z = np.load(golden_dir / "generator.npz")
    with torch.no_grad():
        img, _ = det_generator.decoder(torch.from_numpy(z["dec_feats"]),
                                       [torch.from_numpy(z["dec_latent"])],
                                       randomize_noise=False)
    # batched modulation conv(x*s, W)*demod vs the reference's per-face weights
    np.testing.assert_allclose(img.numpy(), z["dec_img"], rtol=0, atol=2e-5)


def test_mapping_and_mean_latent(det_generator, golden_dir):
    z = np.load(golden_dir / "generator.npz")
    with torch.no_grad():
        lat = det_generator.style(torch.from_numpy(z["z"]))
        np.testing.assert_array_equal(lat.numpy(), z["dec_latent"])
        mean = det_generator.mean_latent(64, "cpu", z=torch.from_numpy(z["mean_z"]))
    np.testing.assert_array_equal(mean[0].numpy(), z["mean_renderer"])
    np.testing.assert_array_equal(mean[1].numpy(), z["mean_decoder"])


def test_cpu_tensors_rejected_like_reference(sdfr):
    enc = sdfr.GridEncoder(desired_resolution=4096)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        enc(torch.zeros(4, 3), bound=2)
    sh = sdfr.SHEncoder()
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        sh(torch.zeros(4, 3))


def test_options_defaults(sdfr):
    opt = sdfr.vol_render_opt()
    assert opt.rendering.N_samples == 24 and opt.rendering.perturb == 1.0
    assert opt.model.renderer_spatial_output_dim == 64 and opt.model.size == 256
    assert opt.camera.fov == 6 and opt.camera.dist_radius == 0.12
    assert opt.rendering.type == "ngp" and opt.model.freeze_renderer
    o1 = sdfr.vol_render_opt(train_renderer=True)
    assert "no_features_output" in o1.rendering and o1.rendering.return_sdf


def test_fused_path_selection(sdfr):
    opt = sdfr.vol_render_opt()
    r = sdfr.VolumeFeatureRenderer(opt.rendering, style_dim=256, out_im_res=8)
    cam = torch.zeros(1, 3, 4)
    st = torch.zeros(1, 256)
    with torch.no_grad():
        assert not r._fused_ok(cam, st, False)      # CPU tensors never take the HIP path
    opt2 = sdfr.vol_render_opt(ngp=False)
    r2 = sdfr.VolumeFeatureRenderer(opt2.rendering, style_dim=256, out_im_res=8)
    assert isinstance(r2.network, sdfr.SirenGenerator)


def test_align_volume_matches_reference(sdfr, golden_dir):
    """sdf_utils.align_volume on a random volume: same grid_sample, bit for bit."""
    g = np.load(golden_dir / "mesh128.npz")
    out = sdfr.align_volume(torch.from_numpy(g["vol"]))
    np.testing.assert_array_equal(out.numpy(), g["vol_aligned"])


def test_xyz2mesh_faces(sdfr):
    xyz = torch.arange(3 * 4 * 5, dtype=torch.float32).reshape(1, 3, 4, 5)
    res = sdfr.xyz2mesh(xyz)
    verts, faces = res if isinstance(res, tuple) else (res.vertices, res.faces)
    assert verts.shape == (20, 3) and faces.shape[1] == 3 and faces.max() < 20


def test_graphed_generator_rejects_cpu(sdfr):
    opt = sdfr.vol_render_opt()
    g = sdfr.Generator(opt.model, opt.rendering).eval()
    with pytest.raises(RuntimeError, match="on a GPU"):
        sdfr.GraphedGenerator(g)


def test_get_rays_bit_exact_vs_reference(sdfr, golden_dir):
    """get_rays' rays_d as the explicit left-to-right sum equals the reference's
    torch.sum (sdf_model.py:213) on CPU, bit for bit (the GPU test repeats it on cuda)."""
    g = np.load(golden_dir / "render_small.npz")
    opt = sdfr.vol_render_opt()
    ren = sdfr.VolumeFeatureRenderer(opt.rendering, style_dim=256, out_im_res=int(g["res"]))
    _, rays_d, viewdirs = ren.get_rays(torch.from_numpy(g["focal"]), torch.from_numpy(g["ext"]))
    np.testing.assert_array_equal(rays_d.numpy(), g["rays_d"])
    vd = viewdirs / torch.norm(viewdirs, dim=-1, keepdim=True)
    np.testing.assert_array_equal(vd.numpy(), g["viewdirs"])


def _golden_renderer(sdfr, golden_dir, name, kind):
    g = np.load(golden_dir / f"{name}.npz")
    opt = sdfr.vol_render_opt(ngp=kind == "ngp", fc=kind == "fc")
    r = opt.rendering
    r.N_samples = int(g["n_samples"])
    for k, v in ast.literal_eval(str(g["render_opts"])).items():   # the fixture's options
        if k in ("return_sdf", "return_xyz", "static_viewdirs", "force_background", "perturb"):
            r[k] = v
    ren = sdfr.VolumeFeatureRenderer(r, style_dim=256, out_im_res=int(g["res"]))
    amp = float(g["table_amp"]) if "table_amp" in g.files else 1.0
    sd = W.det_state_dict(W.golden_entries(golden_dir, kind=kind), "renderer.", table_amp=amp)
    ren.load_state_dict({k[len("renderer."):]: v for k, v in sd.items()}, strict=True)
    return g, ren.eval()


def test_fc_state_dict_matches_reference(sdfr, golden_dir):
    opt = sdfr.vol_render_opt(ngp=False, fc=True)
    g = sdfr.Generator(opt.model, opt.rendering, full_pipeline=False)
    mine = {k: tuple(v.shape) for k, v in g.state_dict().items()}
    assert mine == dict(W.golden_entries(golden_dir, kind="fc"))


def test_fc_renderer_matches_reference_cpu(sdfr, golden_dir):
    """rendering.fc = 1 (FCGenerator, sdf_model.py:1599-1670): the drop-in renderer on
    CPU runs the reference's torch ops in the reference's order."""
    g, ren = _golden_renderer(sdfr, golden_dir, "render_fc_small", "fc")
    assert isinstance(ren.network, sdfr.FCGenerator)
    t = lambda k: torch.from_numpy(g[k])  # noqa: E731
    with torch.no_grad():
        rgb, feat, sdf, mask, xyz, _ = ren(t("ext"), t("focal"), t("near"), t("far"),
                                           styles=t("latent"), t_rand=t("t_rand"))
    for k, v in dict(rgb=rgb, features=feat, sdf=sdf, xyz=xyz, mask=mask).items():
        np.testing.assert_allclose(v.numpy(), g[k], rtol=0, atol=1e-6, err_msg=k)
