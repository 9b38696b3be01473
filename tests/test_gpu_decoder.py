"""GPU parity: the decoder HIP ops against the oracle (oracle/oracle.py, decoder ops).

fused_bias_act and modulate_to_nhwc are element-wise in the reference's
operation order: BIT-EXACT.  upfirdn2d and the styled epilogue sum filter taps
/ channels in a different order than the float64 oracle: bounded by 1e-5
absolute on O(1) data; measured on MI355X: epilogue <= 1.7e-6, upfirdn2d
<= 7.2e-7, whole decoder fused vs op-by-op 8.6e-6 on outputs of magnitude 7
(all recorded in the parity JSON).
"""
import json
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
_record = {}


def teardown_module(module):
    out = os.environ.get("SDFR_PARITY_JSON")
    if out:
        with open(out.replace(".json", "_decoder.json"), "w") as f:
            json.dump(_record, f, indent=1, sort_keys=True)


def _close(name, got, ref, atol, mean_tol=None):
    got = np.asarray(got, np.float64)
    err = np.abs(got - np.asarray(ref, np.float64))
    _record[name] = [float(err.max()), float(err.mean())]
    assert err.max() <= atol, f"{name}: max err {err.max():.3e} > {atol:.1e}"
    if mean_tol is not None:
        assert err.mean() <= mean_tol, f"{name}: mean err {err.mean():.3e} > {mean_tol:.1e}"


@pytest.fixture(scope="module")
def ops(sdfr):
    return sdfr.decoder_ops


@pytest.mark.parametrize("shape", [(4, 37, 5, 7), (8, 64, 16, 16), (32, 512)])
def test_fused_bias_act_bit_exact(ops, oracle_mod, shape):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(*shape, generator=g)
    b = torch.randn(shape[1], generator=g)
    ref_out = oracle_mod.fused_bias_act(x.numpy(), b.numpy(), None, 3, 0, 0.2, math.sqrt(2))
    out = ops.fused_bias_act(x.to(DEV), b.to(DEV), None, 3, 0, 0.2, math.sqrt(2))
    np.testing.assert_array_equal(out.cpu().numpy(), ref_out)
    gr = torch.randn(*shape, generator=g)
    ref_g = oracle_mod.fused_bias_act(gr.numpy(), None, ref_out, 3, 1, 0.2, math.sqrt(2))
    got_g = ops.fused_bias_act(gr.to(DEV), torch.empty(0, device=DEV), out, 3, 1, 0.2,
                               math.sqrt(2))
    np.testing.assert_array_equal(got_g.cpu().numpy(), ref_g)
    lin = ops.fused_bias_act(x.to(DEV), b.to(DEV), None, 1, 0, 0.2, 1.0)
    np.testing.assert_array_equal(lin.cpu().numpy(),
                                  oracle_mod.fused_bias_act(x.numpy(), b.numpy(), None, 1, 0,
                                                            0.2, 1.0))


def test_fused_leaky_relu_autograd(ops):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(3, 16, 9, 9, generator=g)
    b = torch.randn(16, generator=g)
    go = torch.randn(3, 16, 9, 9, generator=g)
    xc, bc = x.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yc = ops.fused_leaky_relu(xc, bc)
    yc.backward(go)
    xg, bg = x.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    yg = ops.fused_leaky_relu(xg, bg)
    yg.backward(go.to(DEV))
    np.testing.assert_array_equal(yg.detach().cpu().numpy(), yc.detach().numpy())
    _close("flrelu_grad_x", xg.grad.cpu(), xc.grad, 1e-6)
    _close("flrelu_grad_b", bg.grad.cpu(), bc.grad, 1e-4)


UFD = [(2, 1, (2, 1), (4, 4), 3), (1, 1, (1, 1), (4, 4), 5), (1, 2, (2, 2), (4, 4), 3),
       (2, 2, (-1, 3), (3, 5), 2), (3, 1, (0, 0), (2, 2), 1)]


@pytest.mark.parametrize("up,down,pad,kshape,ch", UFD)
def test_upfirdn2d_vs_oracle(ops, oracle_mod, up, down, pad, kshape, ch):
    g = torch.Generator().manual_seed(up * 10 + down)
    x = torch.randn(2, ch, 13, 17, generator=g)
    k = torch.randn(*kshape, generator=g) / 4
    xg = x.to(DEV).requires_grad_(True)
    out = ops.upfirdn2d(xg, k.to(DEV), up=up, down=down, pad=pad)
    ref = oracle_mod.upfirdn2d(x.reshape(-1, 13, 17).numpy(), k.numpy(), up, up, down, down,
                               pad[0], pad[1], pad[0], pad[1])
    _close(f"upfirdn2d_{up}{down}{pad}", out.detach().cpu().reshape(ref.shape), ref, 1e-5)
    # backward against autograd of the reference formula on the CPU
    go = torch.randn(out.shape, generator=g)
    out.backward(go.to(DEV))
    xc = x.clone().requires_grad_(True)
    oc = ops.upfirdn2d_native(xc, k, up, up, down, down, pad[0], pad[1], pad[0], pad[1])
    oc.backward(go)
    _close(f"upfirdn2d_bwd_{up}{down}{pad}", xg.grad.cpu(), xc.grad, 1e-5)


# the tiled 4x4 kernel (upfirdn2d_tile_kernel) at the discriminator / decoder-training
# shapes, across tile edges (64-wide, 16- or 32-tall output tiles), negative pads
UFD_TILE = [(1, 1, (2, 2), (2, 128, 64, 64)), (1, 1, (1, 1), (2, 64, 129, 131)),
            (2, 1, (2, 1), (2, 3, 128, 128)), (1, 2, (2, 2), (2, 3, 259, 257)),
            (1, 1, (-1, 3), (1, 4, 33, 95)), (2, 1, (0, 3), (1, 5, 40, 70)),
            (1, 2, (1, -1), (1, 6, 70, 150))]


@pytest.mark.parametrize("up,down,pad,shape", UFD_TILE)
def test_upfirdn2d_tiled_vs_reference_formula(ops, up, down, pad, shape):
    """Forward and backward against the reference's own formulation (upfirdn2d_native,
    sdf_op.py:273-316: zero-insert, pad, F.conv2d with the flipped kernel, stride) and
    its autograd, on the CPU in fp32, with the StyleGAN blur taps."""
    g = torch.Generator(device=DEV).manual_seed(sum(shape) + up + 3 * down)
    x = torch.randn(*shape, device=DEV, generator=g)
    f = torch.tensor([1.0, 3.0, 3.0, 1.0], device=DEV)
    k = torch.outer(f, f)
    k = k / k.sum() * (up * up)
    xg = x.clone().requires_grad_(True)
    out = ops.upfirdn2d(xg, k, up=up, down=down, pad=pad)
    xr = x.cpu().requires_grad_(True)
    ref = ops.upfirdn2d_native(xr, k.cpu(), up, up, down, down, pad[0], pad[1], pad[0], pad[1])
    assert out.shape == ref.shape
    _close(f"upfirdn2d_tile_{up}{down}{pad}{shape}", out.detach().cpu(), ref.detach().cpu(), 1e-5)
    go = torch.randn(out.shape, device=DEV, generator=g)
    out.backward(go)
    ref.backward(go.cpu())
    _close(f"upfirdn2d_tile_bwd_{up}{down}{pad}{shape}", xg.grad.cpu(), xr.grad.cpu(), 1e-5)


def test_upfirdn2d_empty_and_errors(ops, sdfr):
    k = torch.ones(4, 4, device=DEV) / 16
    assert ops.upfirdn2d(torch.zeros(0, 3, 8, 8, device=DEV), k, pad=(1, 2)).shape == (0, 3, 8, 8)
    with pytest.raises(RuntimeError, match="up and down factors"):
        ops._upfirdn2d_op(torch.zeros(1, 4, 4, device=DEV), k, 0, 1, 1, 1, 0, 0, 0, 0)
    lib = sdfr._lib
    x = torch.zeros(1, 4, 4, device=DEV)
    rc = lib.lib().sdfr_upfirdn2d(lib.ptr(x), lib.ptr(x), lib.ptr(k), 1, 4, 4, 4, 4, 1, 1, 1, 1,
                                  -3, -3, 0, 0, lib.stream_of(x))
    assert rc == lib.SDFR_EINVAL and b"not positive" in lib.lib().sdfr_last_error()


EPI = [  # name, C, H, blur, rgb, skip, s_next, store_y, noise, demod
    ("conv1_like", 512, 8, False, True, False, True, True, True, True),
    ("conv128_like", 256, 16, False, True, True, True, True, True, True),
    ("last_layer", 128, 16, False, True, True, False, False, True, True),
    ("up_256", 256, 8, True, False, False, True, True, True, True),
    ("up_128_nonoise", 128, 12, True, False, False, True, True, False, False),
    ("plain_64_no_rgb", 64, 10, False, False, False, False, True, True, True),
    ("c1024_rgb", 1024, 4, False, True, True, True, True, True, True),
    ("c16_rgb", 16, 6, False, True, True, True, True, False, True),
]


@pytest.mark.parametrize("name,C,H,blur,rgb,skip,s_next,store_y,noise,demod", EPI)
def test_styled_epilogue_vs_oracle(ops, oracle_mod, name, C, H, blur, rgb, skip, s_next,
                                   store_y, noise, demod):
    B = 3
    g = torch.Generator().manual_seed(C + H)
    Hc, Ho = (2 * H + 1, 2 * H) if blur else (H, H)
    conv = torch.randn(B, C, Hc, Hc, generator=g)
    bias = torch.randn(C, generator=g)
    nw = torch.tensor([0.7])
    nz = torch.randn(B, 1, Ho, Ho, generator=g) if noise else None
    dm = torch.rand(B, C, generator=g) + 0.5 if demod else None
    sn = torch.rand(B, C, generator=g) + 0.5 if s_next else None
    rw = torch.randn(B, 3, C, generator=g) / math.sqrt(C) if rgb else None
    rb = torch.randn(3, generator=g) if rgb else None
    sk = torch.randn(B, 3, H // 2, H // 2, generator=g) if skip else None
    k2 = torch.outer(torch.tensor([1., 3, 3, 1]), torch.tensor([1., 3, 3, 1])) / 16
    fir = ops.separable_taps(k2)
    assert fir == [0.25, 0.75, 0.75, 0.25]
    d = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    y, out_rgb = ops.styled_epilogue(
        conv.to(DEV).contiguous(memory_format=torch.channels_last), fir=fir, bias=d(bias),
        noise_weight=d(nw), noise=d(nz), demod=d(dm), blur_up=blur, s_next=d(sn),
        store_y=store_y, rgb_w=d(rw), rgb_b=d(rb), skip=d(sk))
    npf = lambda t: None if t is None else t.numpy()  # noqa: E731
    ry, rrgb = oracle_mod.styled_epilogue(
        conv.numpy(), kernel2d=k2.numpy(), bias=bias.numpy(), noise_weight=0.7, noise=npf(nz),
        demod=npf(dm), blur_up=blur, s_next=npf(sn), rgb_w=npf(rw), rgb_b=npf(rb), skip=npf(sk))
    if store_y:
        assert y.is_contiguous(memory_format=torch.channels_last)
        _close(f"epilogue_{name}_y", y.cpu(), ry, 1e-5, 2e-7)
    else:
        assert y is None
    if rgb:
        _close(f"epilogue_{name}_rgb", out_rgb.cpu(), rrgb, 1e-5, 5e-7)


def test_styled_epilogue_rejects_bad_channels(ops):
    conv = torch.zeros(1, 12, 4, 4, device=DEV)
    with pytest.raises(RuntimeError, match="power of two"):
        ops.styled_epilogue(conv, fir=[0.25, 0.75, 0.75, 0.25], bias=torch.zeros(12, device=DEV),
                            noise_weight=None, rgb_w=torch.zeros(1, 3, 12, device=DEV),
                            rgb_b=torch.zeros(3, device=DEV), store_y=False)


def test_split_planes_bit_exact(ops):
    """modulate_to_nhwc_split and the epilogue's split y write exactly the
    round-to-nearest (hi, lo) fp16 split of their fp32 result, in the split-NHWC
    layout [B,H,W,C/8,2,8] (also split_nhwc's, which the conv tests feed)."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 8, 12, generator=g)
    s = torch.rand(2, 64, generator=g) + 0.5
    xs = ops.modulate_to_nhwc_split(x.to(DEV), s.to(DEV))
    assert xs.shape == (2, 8, 12, 8, 2, 8) and xs.dtype == torch.float16
    np.testing.assert_array_equal(xs.cpu().numpy(),
                                  ops.split_nhwc(x * s[:, :, None, None]).numpy())
    hi, lo = ops.unsplit_nhwc(xs)
    ref = (x * s[:, :, None, None]).permute(0, 2, 3, 1).contiguous()
    rh = ref.half()
    np.testing.assert_array_equal(hi.cpu().numpy(), rh.numpy())
    np.testing.assert_array_equal(lo.cpu().numpy(), (ref - rh.float()).half().numpy())
    conv = torch.randn(2, 64, 8, 12, generator=g).to(DEV).contiguous(
        memory_format=torch.channels_last)
    kw = dict(fir=[0.125, 0.375, 0.375, 0.125], bias=torch.randn(64, device=DEV),
              noise_weight=torch.full((1,), 0.1, device=DEV),
              noise=torch.randn(2, 1, 8, 12, device=DEV), demod=torch.rand(2, 64, device=DEV),
              s_next=torch.rand(2, 64, device=DEV))
    y, _ = ops.styled_epilogue(conv, **kw)
    ys, _ = ops.styled_epilogue(conv, split_y=True, **kw)
    yh, yl = ops.unsplit_nhwc(ys)
    ref = y.permute(0, 2, 3, 1).contiguous().cpu()
    np.testing.assert_array_equal(yh.cpu().numpy(), ref.half().numpy())
    np.testing.assert_array_equal(yl.cpu().numpy(), (ref - ref.half().float()).half().numpy())


@pytest.mark.parametrize("C,H", [(256, 64), (36, 5), (128, 20)])
def test_modulate_to_nhwc_bit_exact(ops, C, H):
    g = torch.Generator().manual_seed(C)
    x = torch.randn(2, C, H, H + (H % 4 == 1) * 3, generator=g)
    s = torch.randn(2, C, generator=g)
    y = ops.modulate_to_nhwc(x.to(DEV), s.to(DEV))
    assert y.is_contiguous(memory_format=torch.channels_last)
    np.testing.assert_array_equal(y.cpu().numpy(), (x * s[:, :, None, None]).numpy())


@pytest.mark.parametrize("B,Cin,Cout,H,W,transposed", [
    (2, 32, 128, 5, 7, False),        # ragged pixel tiles, border taps
    (1, 256, 256, 16, 16, False),
    (3, 64, 128, 6, 5, True),         # all four parity classes, ragged
    (1, 512, 256, 8, 8, True),
])
def test_conv3x3_f16x3_vs_fp64(ops, B, Cin, Cout, H, W, transposed):
    """Split-fp16 implicit-GEMM conv against float64; its error must be of the same
    order as PyTorch-ROCm's own fp32 convolution of the same inputs."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(B * 7 + Cin + H)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(1, Cout, Cin, 3, 3, generator=g)
    scale = 1 / math.sqrt(Cin * 9)
    w32 = (scale * w[0]).float()
    packed, su = ops.conv_pack_weights(w[0].to(DEV), scale)
    out = ops.conv3x3_f16x3(ops.split_nhwc(x.to(DEV)), packed, Cout, transposed=transposed)
    got = (out / su.view(1, -1, 1, 1)).cpu().double()
    if transposed:
        ref = F.conv_transpose2d(x.double(), w32.double().transpose(0, 1), stride=2)
        r32 = F.conv_transpose2d(x.to(DEV), w32.to(DEV).transpose(0, 1).contiguous(), stride=2)
    else:
        ref = F.conv2d(x.double(), w32.double(), padding=1)
        r32 = F.conv2d(x.to(DEV), w32.to(DEV), padding=1)
    assert got.shape == ref.shape
    assert torch.all(su == torch.exp2(torch.round(torch.log2(su))))      # powers of two
    e16 = float((got - ref).abs().max())
    e32 = float((r32.cpu().double() - ref).abs().max())
    name = f"conv_f16x3_B{B}_{Cin}x{Cout}_{H}x{W}_{'T' if transposed else 'N'}"
    _record[name] = [e16, e32]
    assert e16 <= 4 * e32 + 1e-6, (e16, e32)
    # split-K (small grids: K shared by 2-4 workgroups, partials summed in a fixed
    # order): the unsplit result to fp32 summation-order rounding, deterministic
    xs = ops.split_nhwc(x.to(DEV))
    o1 = ops.conv3x3_f16x3(xs, packed, Cout, transposed=transposed, split_k=False)
    o2 = ops.conv3x3_f16x3(xs, packed, Cout, transposed=transposed)
    o3 = ops.conv3x3_f16x3(xs, packed, Cout, transposed=transposed)
    assert torch.equal(o2, o3)
    scale = float(o1.abs().max())
    _close(f"{name}_splitk", o2.cpu(), o1.cpu(), 2e-6 * scale, 2e-7 * scale)


@pytest.mark.parametrize("B,Cin,Cout,H,W", [
    (1, 64, 128, 16, 16),        # one tile per 64-channel block, the four edge classes
    (2, 96, 256, 32, 48),        # odd channel-group count, non-square, 4 channel blocks
    (1, 512, 256, 64, 64),       # the decoder's 64 -> 128 layer at one face
    (1, 256, 128, 128, 128),     # ... and its 128 -> 256 layer
])
def test_conv_t_kernel_vs_fp64_and_strip_kernel(ops, sdfr, B, Cin, Cout, H, W):
    """The transposed conv on conv_t_kernel (all four parity classes of a 16 x 16 input
    block per workgroup, one halo per channel group; the last output row / column as
    thin conv_x_kernel classes), forced at any tile count (sdfr_set_conv_t_mode(2)):
    against float64 (the same bound as the strip kernel's, PyTorch-ROCm fp32 for scale)
    and against conv_x_kernel (mode 0) to fp32 summation-order rounding;
    deterministic."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(B * 11 + Cin + H)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g)
    scale = 1 / math.sqrt(Cin * 9)
    w32 = (scale * w).float()
    packed, su = ops.conv_pack_weights(w.to(DEV), scale)
    xs = ops.split_nhwc(x.to(DEV))
    L = sdfr._lib.lib()
    L.sdfr_set_conv_t_mode(2)
    out = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True, split_k=False)
    out2 = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True, split_k=False)
    L.sdfr_set_conv_t_mode(3)
    # with a workspace and SDFR_CONV_T=3: at one face (64 / 128 tiles) each tile's
    # channel groups split 4 / 2 ways, partials summed in split order
    sk = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True)
    sk2 = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True)
    L.sdfr_set_conv_t_mode(0)
    strip = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True, split_k=False)
    assert L.sdfr_set_conv_t_mode(-1) == 0             # back to the load-time default
    torch.cuda.synchronize()
    assert torch.equal(out, out2) and torch.equal(sk, sk2)
    got = (out / su.view(1, -1, 1, 1)).cpu().double()
    ref = F.conv_transpose2d(x.double(), w32.double().transpose(0, 1), stride=2)
    r32 = F.conv_transpose2d(x.to(DEV), w32.to(DEV).transpose(0, 1).contiguous(), stride=2)
    assert got.shape == ref.shape == (B, Cout, 2 * H + 1, 2 * W + 1)
    e16 = float((got - ref).abs().max())
    e32 = float((r32.cpu().double() - ref).abs().max())
    name = f"conv_t_B{B}_{Cin}x{Cout}_{H}x{W}"
    _record[name] = [e16, e32]
    assert e16 <= 4 * e32 + 1e-6, (e16, e32)
    s = float(strip.abs().max())
    _close(f"{name}_vs_strip", out.cpu(), strip.cpu(), 2e-6 * s, 2e-7 * s)
    _close(f"{name}_ksplit", sk.cpu(), out.cpu(), 2e-6 * s, 2e-7 * s)


@pytest.mark.parametrize("B,Cin,Cout,H,W,noise,s_next,mode", [
    (1, 64, 128, 16, 16, True, True, 2),     # one block per 64 channels: every pixel
                                             # is a block border or next to one
    (2, 96, 256, 32, 48, True, True, 2),     # odd channel-group count, 2 x 3 blocks
    (1, 32, 128, 32, 32, False, False, 2),   # no noise, no next modulation
    (4, 512, 256, 64, 64, True, True, 1),    # the decoder's 64 -> 128 layer at 4 faces
    (4, 256, 128, 128, 128, True, True, 1),  # ... and its 128 -> 256 layer (512 tiles)
])
def test_conv_t_act_equals_conv_then_blur_epilogue(ops, sdfr, B, Cin, Cout, H, W, noise,
                                                     s_next, mode):
    """sdfr_conv_t_act (blur + styled epilogue inside conv_t_kernel for each block's
    interior, conv_t_border_kernel for the block borders from the raw band rows and
    columns) against sdfr_conv3x3_f16x3 (transposed) + sdfr_styled_epilogue (blur_up):
    the same fp32 operations in the same order -- y bit-exact."""
    g = torch.Generator().manual_seed(B + Cin + Cout + H + W)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g)
    packed, su = ops.conv_pack_weights(w.to(DEV), 1 / math.sqrt(Cin * 9))
    xs = ops.split_nhwc(x.to(DEV))
    demod = (torch.rand(B, Cout, generator=g) + 0.5).to(DEV) / su
    bias = (torch.randn(Cout, generator=g) * 0.1).to(DEV)
    nw = torch.tensor([0.3]).to(DEV)
    nz = torch.randn(B, 1, 2 * H, 2 * W, generator=g).to(DEV) if noise else None
    sn = (torch.rand(B, Cout, generator=g) + 0.5).to(DEV) if s_next else None
    fir = ops.separable_taps(torch.outer(torch.tensor([1., 3., 3., 1.]),
                                         torch.tensor([1., 3., 3., 1.])) / 64 * 4)
    L = sdfr._lib.lib()
    prev = L.sdfr_set_conv_t_mode(mode)
    try:
        assert ops.conv_t_act_supported(xs, Cout)
        y = ops.conv_t_act(xs, packed, Cout, fir=fir, demod=demod, bias=bias, noise_weight=nw,
                           noise=nz, s_next=sn)
        raw = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True, split_k=False)
        ref, _ = ops.styled_epilogue(raw, fir=fir, bias=bias, noise_weight=nw, noise=nz,
                                     demod=demod, blur_up=True, s_next=sn, store_y=True,
                                     split_y=True)
    finally:
        L.sdfr_set_conv_t_mode(prev)
    torch.cuda.synchronize()
    assert y.shape == ref.shape == (B, 2 * H, 2 * W, Cout // 8, 2, 8)
    bad = (y != ref).reshape(B, 2 * H, 2 * W, -1).any(-1)
    assert not bad.any(), f"{int(bad.sum())} pixels differ, first {bad.nonzero()[:5].tolist()}"


def test_conv_t_act_unsupported_shape(ops, sdfr):
    """Below conv_t_kernel's range (default mode, one face at 64^2: 64 tiles) the entry
    point refuses; the decoder then takes the two-launch path."""
    xs = torch.zeros(1, 64, 64, 64, 2, 8, device=DEV, dtype=torch.float16)
    assert not ops.conv_t_act_supported(xs, 256)
    assert ops.conv_t_act_supported(torch.zeros(4, 64, 64, 64, 2, 8, device=DEV,
                                                dtype=torch.float16), 256)


@pytest.mark.parametrize("B,Cin,Cout,H,W,rgb,skip,store_y", [
    (2, 64, 128, 16, 16, True, True, True),     # one Cout block, ToRGB with skip
    (1, 256, 512, 16, 32, True, False, True),   # four Cout blocks (partials), no skip
    (2, 128, 256, 32, 8, True, True, False),    # last layer: rgb only
    (1, 32, 256, 16, 16, False, False, True),   # y only
    (2, 96, 128, 32, 48, True, True, True),     # halo kernel: odd channel-group count, 2x3 blocks
    (1, 256, 256, 64, 64, True, False, True),   # halo kernel: decoder-sized layer
    (1, 256, 512, 64, 64, True, False, True),   # batch-1 conv1: halo kernel, 4-way K split
    (3, 32, 256, 128, 128, True, False, True),  # persistent halo kernel: 384 tiles (2 per
                                                # workgroup on half the CUs), one group
    (2, 64, 128, 256, 256, True, True, False),  # ... 512 tiles (2 per workgroup), rgb only
])
def test_conv_act_equals_conv_then_epilogue(ops, B, Cin, Cout, H, W, rgb, skip, store_y):
    """sdfr_conv3x3_f16x3_act (+ sdfr_rgb_finish) against sdfr_conv3x3_f16x3 followed by
    sdfr_styled_epilogue on the same inputs: y (split-NHWC) bit-exact -- same fp32
    operations in the same order -- and rgb to fp32 summation-order rounding."""
    g = torch.Generator().manual_seed(B + Cin + Cout + H)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g)
    packed, su = ops.conv_pack_weights(w.to(DEV), 1 / math.sqrt(Cin * 9))
    xs = ops.split_nhwc(x.to(DEV))
    fir = [0.125, 0.375, 0.375, 0.125]
    demod = (torch.rand(B, Cout, generator=g) + 0.5).to(DEV) / su
    kw = dict(bias=torch.randn(Cout, generator=g).to(DEV),
              noise_weight=torch.full((1,), 0.1, device=DEV),
              noise=torch.randn(B, 1, H, W, generator=g).to(DEV),
              s_next=(torch.rand(B, Cout, generator=g) + 0.5).to(DEV) if store_y else None,
              store_y=store_y)
    # ToRGB's weight as the generator forms it: scaled base [3, Cout] x style [B, Cout]
    rgb_base = torch.randn(3, Cout, generator=g).to(DEV)
    rgb_s = (torch.rand(B, Cout, generator=g) + 0.5).to(DEV)
    rgb_w = rgb_base[None] * rgb_s[:, None, :] if rgb else None
    rgb_b = torch.randn(3, generator=g).to(DEV)
    sk = torch.randn(B, 3, H // 2, W // 2, generator=g).to(DEV) if skip else None
    ys, part = ops.conv3x3_f16x3_act(xs, packed, Cout, demod=demod, rgb_w=rgb_w, split_k=False,
                                     **kw)
    out = ops.conv3x3_f16x3(xs, packed, Cout, split_k=False)
    y_ref, rgb_ref = ops.styled_epilogue(out, fir=fir, demod=demod, rgb_w=rgb_w,
                                         rgb_b=rgb_b if rgb else None, skip=sk,
                                         split_y=store_y, **kw)
    if store_y:
        np.testing.assert_array_equal(ys.cpu().numpy(), y_ref.cpu().numpy())
    else:
        assert ys is None
    if rgb:
        assert part.shape == (Cout // 128, B, 3, H, W)
        # the product formed inside the kernel (rgb_base x rgb_s): bit-identical
        ysb, partb = ops.conv3x3_f16x3_act(xs, packed, Cout, demod=demod, rgb_base=rgb_base,
                                           rgb_s=rgb_s, split_k=False, **kw)
        assert torch.equal(part, partb)
        if store_y:
            assert torch.equal(ys, ysb)
        got = ops.rgb_finish(part, rgb_b, skip=sk, fir=fir)
        scale = float(rgb_ref.abs().max())
        _close(f"conv_act_rgb_{Cin}x{Cout}_{H}x{W}", got.cpu(), rgb_ref.cpu(), 1e-5 * scale,
               1e-6 * scale)
    else:
        assert part is None
    # split-K (small grids: K over 2 or 4 workgroups -- conv_h_kernel's channel-group
    # split + conv_h_finish_kernel, or conv_x_kernel's -- partial tiles summed in a fixed
    # order, then the same epilogue): fp32 summation-order rounding of the conv
    ys2, part2 = ops.conv3x3_f16x3_act(xs, packed, Cout, demod=demod, rgb_w=rgb_w, **kw)
    ys3, _ = ops.conv3x3_f16x3_act(xs, packed, Cout, demod=demod, rgb_w=rgb_w, **kw)
    if store_y:
        hi, lo = ops.unsplit_nhwc(ys2)
        hr, lr = ops.unsplit_nhwc(y_ref)
        y2, yr = hi.float() + lo.float(), hr.float() + lr.float()
        scale = float(yr.abs().max())
        _close(f"conv_act_splitk_y_{Cin}x{Cout}_{H}x{W}", y2.cpu(), yr.cpu(), 2e-6 * scale,
               2e-7 * scale)
        assert torch.equal(ys2, ys3)                      # deterministic
    if rgb:
        _, part2b = ops.conv3x3_f16x3_act(xs, packed, Cout, demod=demod, rgb_base=rgb_base,
                                          rgb_s=rgb_s, **kw)
        assert torch.equal(part2, part2b)
        got2 = ops.rgb_finish(part2, rgb_b, skip=sk, fir=fir)
        scale = float(rgb_ref.abs().max())
        _close(f"conv_act_splitk_rgb_{Cin}x{Cout}_{H}x{W}", got2.cpu(), rgb_ref.cpu(),
               1e-5 * scale, 1e-6 * scale)


@pytest.mark.parametrize("B,H,W,nparts", [(2, 16, 16, 1), (3, 32, 24, 2), (1, 64, 64, 4)])
def test_rgb_finish_skip_bit_exact(ops, B, H, W, nparts):
    """sdfr_rgb_finish's closed-form 2x upsampled skip equals skip_up's tap loop (the
    one sdfr_styled_epilogue runs) bit for bit: with ToRGB weights of zero the epilogue's
    rgb is bias + skip_up exactly, and rgb_finish of zero partials the same sum."""
    g = torch.Generator().manual_seed(B * H + W)
    C = 128
    conv = torch.randn(B, C, H, W, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    fir = [0.125, 0.375, 0.375, 0.125]
    rgb_b = torch.randn(3, generator=g).to(DEV)
    skip = torch.randn(B, 3, H // 2, W // 2, generator=g).to(DEV)
    _, rgb_ref = ops.styled_epilogue(conv, fir=fir, bias=torch.zeros(C, device=DEV),
                                     noise_weight=torch.zeros(1, device=DEV), store_y=False,
                                     rgb_w=torch.zeros(B, 3, C, device=DEV), rgb_b=rgb_b, skip=skip)
    part = torch.zeros(nparts, B, 3, H, W, device=DEV)
    got = ops.rgb_finish(part, rgb_b, skip=skip, fir=fir)
    assert torch.equal(got, rgb_ref)
    # and the partial sums add in order before the bias
    part = torch.randn(nparts, B, 3, H, W, generator=g).to(DEV)
    got = ops.rgb_finish(part, rgb_b, skip=skip, fir=fir)
    want = part[0]
    for k in range(1, nparts):
        want = want + part[k]
    want = (want + rgb_b[None, :, None, None]) + (rgb_ref - rgb_b[None, :, None, None])
    torch.testing.assert_close(got, want, rtol=0, atol=2e-6)


def test_prepared_fallback_draws_nothing_twice(sdfr):
    """Decoder.forward(prepared=...) falling back to the module path (features that
    require grad) runs on the prep's latent and noise maps: no second draw of the
    injection index or of the noise, so the RNG streams stay where the reference
    leaves them."""
    import random
    opt = sdfr.vol_render_opt()
    torch.manual_seed(3)
    dec = sdfr.Generator(opt.model, opt.rendering).to(DEV).decoder.eval()
    feats = (torch.randn(2, 256, 64, 64, device=DEV) * 0.3).requires_grad_()
    styles = [torch.randn(2, 256, device=DEV), torch.randn(2, 256, device=DEV)]  # mixing
    random.seed(5)
    torch.manual_seed(7)
    with torch.no_grad():
        prep = dec.prepare_fused(styles, 2, torch.device(DEV))
    py_state, t_state = random.getstate(), torch.cuda.get_rng_state()
    img, lat = dec(feats, styles, prepared=prep, return_latents=True)
    assert img.requires_grad                                  # the autograd path ran
    assert random.getstate() == py_state                      # no second inject_index
    assert torch.equal(torch.cuda.get_rng_state(), t_state)   # no second noise draw
    ref, _ = dec(feats, [prep[0]], input_is_latent=True, noise=prep[1])
    assert torch.equal(lat, prep[0])
    torch.testing.assert_close(img, ref, rtol=0, atol=1e-6)


def test_decoder_fused_batch_chunks(sdfr):
    """64 faces exceed the fused kernels' 32-bit activation offsets (the 256^2 layers'
    (257^2 x 128) fp32 per face: 63 faces per call): the fused decoder runs them as two
    chunks of 32 on the same styles and noise maps -- bit-identical to two 32-face calls
    (conv_launch rejected the whole batch before)."""
    opt = sdfr.vol_render_opt()
    opt.model.feature_encoder_in_channels = opt.rendering.width
    torch.manual_seed(0)
    dec = sdfr.Decoder(opt.model).to(DEV).eval()
    B = 64
    feats = torch.randn(B, 256, 64, 64, device=DEV) * 0.3
    z = torch.randn(B, 256, device=DEV)
    noise = [torch.randn(B, 1, 2 ** r, 2 ** r, device=DEV) for r in (6, 7, 7, 8, 8)]
    with torch.no_grad():
        assert dec._fused_ok(feats, None, None)
        assert dec._fused_chunk(feats, [dec.conv1] + list(dec.convs)) == 63
        whole, _ = dec(feats, [z], noise=noise)
        halves = [dec(feats[s], [z[s]], noise=[n[s] for n in noise])[0]
                  for s in (slice(0, 32), slice(32, 64))]
    assert whole.shape == (B, 3, 256, 256)
    assert torch.equal(whole, torch.cat(halves, 0))


@pytest.mark.parametrize("conv_impl,fuse", [("f16x3", True), ("f16x3", False), ("miopen", False)])
def test_decoder_fused_equals_module_path(sdfr, conv_impl, fuse):
    """Same weights, latents and noise: HIP-epilogue decoder == op-by-op decoder."""
    opt = sdfr.vol_render_opt()
    opt.model.feature_encoder_in_channels = opt.rendering.width   # as Generator.__init__ sets it
    torch.manual_seed(0)
    dec = sdfr.Decoder(opt.model).to(DEV).eval()
    dec.conv_impl = conv_impl
    dec.fuse_conv_act = fuse
    with torch.no_grad():
        for m in dec.modules():
            if isinstance(m, sdfr.NoiseInjection):
                m.weight.fill_(0.1)
            if isinstance(m, sdfr.FusedLeakyReLU):
                m.bias.normal_(0, 0.1)
    B = 2
    feats = torch.randn(B, 256, 64, 64, device=DEV)
    z = [torch.randn(B, 256, device=DEV)]
    noise = [torch.randn(B, 1, 2 ** r, 2 ** r, device=DEV) for r in (6, 7, 7, 8, 8)]
    with torch.no_grad():
        assert dec._fused_ok(feats, None, None)
        fused, _ = dec(feats, z, noise=noise)
        dec.use_fused = False
        mod, _ = dec(feats, z, noise=noise)
        dec.use_fused = True
    assert fused.shape == mod.shape == (B, 3, 256, 256)
    scale = float(mod.abs().max())
    tag = conv_impl + ("_act" if fuse else "")
    _record[f"decoder_fused_vs_module_scale_{tag}"] = scale
    _close(f"decoder_fused_vs_module_{tag}", fused.cpu(), mod.cpu(), 1e-4 * max(1.0, scale),
           1e-5 * max(1.0, scale))


def test_decoder_conv_t_blur_fusion_bit_exact(sdfr):
    """The fused decoder at 4 faces (both upsampling layers on sdfr_conv_t_act) gives the
    image of the two-launch path (conv_t_kernel raw output + epi_blur_kernel) bit for bit."""
    opt = sdfr.vol_render_opt()
    opt.model.feature_encoder_in_channels = opt.rendering.width
    torch.manual_seed(0)
    dec = sdfr.Decoder(opt.model).to(DEV).eval()
    with torch.no_grad():
        for m in dec.modules():
            if isinstance(m, sdfr.NoiseInjection):
                m.weight.fill_(0.1)
            if isinstance(m, sdfr.FusedLeakyReLU):
                m.bias.normal_(0, 0.1)
    B = 4
    feats = torch.randn(B, 256, 64, 64, device=DEV)
    z = [torch.randn(B, 256, device=DEV)]
    noise = [torch.randn(B, 1, 2 ** r, 2 ** r, device=DEV) for r in (6, 7, 7, 8, 8)]
    outs = []
    with torch.no_grad():
        for fuse in (True, False):
            dec.fuse_conv_t_blur = fuse
            outs.append(dec(feats, z, noise=noise)[0])
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_ema_accumulate_invalidates_fused_caches(sdfr):
    """training.accumulate (the EMA step, sdf_utils.py:64-69) bumps the parameters'
    versions, so the fused decoder's packed-weight / modulation / demodulation
    caches are rebuilt: after an EMA step the fused image equals the module path's
    on the NEW weights (not the first call's)."""
    from importlib import import_module
    training = import_module(sdfr.Generator.__module__.rsplit(".", 1)[0] + ".training")
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g_ema = sdfr.Generator(opt.model, opt.rendering, ema=True).to(DEV).eval()
    torch.manual_seed(1)
    g = sdfr.Generator(opt.model, opt.rendering).to(DEV)
    B = 2
    feats = torch.randn(B, 256, 64, 64, device=DEV)
    z = [torch.randn(B, 256, device=DEV)]
    noise = [torch.randn(B, 1, 2 ** r, 2 ** r, device=DEV) for r in (6, 7, 7, 8, 8)]
    dec = g_ema.decoder
    with torch.no_grad():
        first, _ = dec(feats, z, noise=noise)                  # fills the caches
        training.accumulate(g_ema, g, 0.5)
        fused, _ = dec(feats, z, noise=noise)
        dec.use_fused = False
        mod, _ = dec(feats, z, noise=noise)
        dec.use_fused = True
    assert not torch.equal(first, fused)
    scale = float(mod.abs().max())
    _close("ema_fused_vs_module", fused.cpu(), mod.cpu(), 1e-4 * max(1.0, scale))


def test_graphed_generator_recaptures_after_weight_update(sdfr):
    """GraphedGenerator keys its graphs on every tensor's (data_ptr, version): after an
    in-place weight update the replay equals the eager forward on the new weights."""
    dev = torch.device("cuda", 0)
    opt = sdfr.vol_render_opt()
    torch.manual_seed(5)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    g.renderer.rng_device = "device"
    gg = sdfr.GraphedGenerator(g)
    z = torch.randn(2, 256, device=dev)
    cam, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=2)
    gg(z, cam, focal, near, far)
    with torch.no_grad():
        for p in g.decoder.parameters():
            p.mul_(0.9)
        g.renderer.network.views_linears.weight.mul_(1.1)
    gg(z, cam, focal, near, far)                      # re-captures (warm-up draws)
    torch.cuda.manual_seed(7)
    got, _ = gg(z, cam, focal, near, far)
    torch.cuda.manual_seed(7)
    with torch.no_grad():
        ref, _ = g([z], cam, focal, near, far)
    assert torch.equal(got, ref)
    with pytest.raises(TypeError, match="tensor"):
        gg.random_faces(1, 64, locations=torch.zeros(1, 2, device=dev))


@pytest.mark.parametrize("B", [1, 5, 37])
def test_mapping_linear_matches_module_path(sdfr, B):
    """sdfr_mapping_linear (one launch per layer, PixelNorm folded in) against the
    module path's GEMM + fused_leaky_relu, for both mapping networks of the Generator
    (3 MappingLinear, sdf_model.py:1084) and of the Decoder (PixelNorm + 5 EqualLinear,
    sdf_model.py:893-902).  fp32, summation order differs: bounded relative to the
    output scale."""
    from sdface_gan_amd.generator import mapping_forward
    opt = sdfr.vol_render_opt()
    torch.manual_seed(B)
    g = sdfr.Generator(opt.model, opt.rendering).to("cuda")
    z = torch.randn(B, 256, device="cuda")
    for seq, x in ((g.style, z), (g.decoder.style, g.style(z).detach())):
        with torch.no_grad():
            got = mapping_forward(seq, x)
        with torch.enable_grad():
            ref = seq(x).detach()
        assert got.shape == ref.shape
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-6, err
