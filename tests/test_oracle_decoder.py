"""CPU: the decoder-op oracle (oracle.fused_bias_act / upfirdn2d / styled_epilogue).

Pinned by known answers and against the drop-in modules' CPU path, which is the
reference's own PyTorch formulation (sdf_op.py:106-114, :273-316) and whose
whole Decoder matches the reference golden (test_host.py::test_decoder_matches_reference).
"""
import math

import numpy as np
import torch


def test_fused_bias_act_kat(oracle_mod):
    x = np.array([[-2.0, 3.0], [0.5, -0.25]], np.float32).reshape(2, 2, 1)
    b = np.array([1.0, -1.0], np.float32)
    y = oracle_mod.fused_bias_act(x, b, None, 3, 0, 0.2, 2.0)
    # (x + b) -> lrelu(0.2) -> * 2, bias along dim 1
    np.testing.assert_array_equal(y.ravel(), np.float32([(-1.0 * 0.2) * 2, 2.0 * 2,
                                                         1.5 * 2, (-1.25 * 0.2) * 2]))
    g = oracle_mod.fused_bias_act(np.ones_like(x), None, y, 3, 1, 0.2, 2.0)
    np.testing.assert_array_equal(g.ravel(), np.float32([0.4, 2, 2, 0.4]))


def test_upfirdn2d_kat(oracle_mod):
    k = np.outer([1, 3, 3, 1], [1, 3, 3, 1]).astype(np.float32) / 64
    delta = np.zeros((1, 7, 7), np.float32)
    delta[0, 3, 3] = 1
    # true convolution of a delta reproduces the kernel: out[y] = sum_i in[y+i-1] k[3-i]
    out = oracle_mod.upfirdn2d(delta, k, 1, 1, 1, 1, 1, 2, 1, 2)
    np.testing.assert_array_equal(out[0, 1:5, 1:5], k)
    assert out.sum() == 1.0
    # Upsample (x2, pad (2,1), kernel*4) keeps a constant image constant
    ones = np.ones((2, 5, 6), np.float32)
    up = oracle_mod.upfirdn2d(ones, k * 4, 2, 2, 1, 1, 2, 1, 2, 1)
    assert up.shape == (2, 10, 12)
    np.testing.assert_allclose(up[:, 2:-2, 2:-2], 1.0, atol=1e-12)
    # down=2 keeps every other sample of the filtered image
    full = oracle_mod.upfirdn2d(ones, k, 1, 1, 1, 1, 1, 1, 1, 1)
    dn = oracle_mod.upfirdn2d(ones, k, 1, 1, 2, 2, 1, 1, 1, 1)
    np.testing.assert_array_equal(dn, full[:, ::2, ::2])


def test_upfirdn2d_matches_reference_formula(sdfr, oracle_mod):
    from importlib import import_module
    ops = import_module(sdfr.__name__ + ".decoder_ops")
    rng = np.random.default_rng(0)
    for (up, down, pad, kshape) in [(2, 1, (2, 1), (4, 4)), (1, 1, (1, 1), (4, 4)),
                                    (1, 2, (2, 2), (4, 4)), (2, 2, (-1, 3), (3, 5)),
                                    (3, 1, (0, 0), (2, 2))]:
        x = rng.normal(size=(2, 3, 9, 11)).astype(np.float32)
        k = rng.normal(size=kshape).astype(np.float32)
        ref = ops.upfirdn2d_native(torch.from_numpy(x), torch.from_numpy(k), up, up, down, down,
                                   pad[0], pad[1], pad[0], pad[1]).numpy()
        got = oracle_mod.upfirdn2d(x.reshape(6, 9, 11), k, up, up, down, down, pad[0], pad[1],
                                   pad[0], pad[1])
        np.testing.assert_allclose(got.reshape(ref.shape), ref, rtol=1e-5, atol=1e-5)


def test_styled_epilogue_matches_modules(sdfr, oracle_mod):
    """oracle.styled_epilogue == StyledConv's post-conv chain + ToRGB (CPU modules)."""
    torch.manual_seed(0)
    B, C, H = 2, 8, 6
    sc = sdfr.StyledConv(C, C, 3, 16, upsample=True)
    trgb = sdfr.ToRGB(C, 16)
    with torch.no_grad():
        sc.noise.weight.fill_(0.3)
        sc.activate.bias.normal_()
        trgb.bias.normal_()
    conv = torch.randn(B, C, 2 * H + 1, 2 * H + 1)
    demod = torch.rand(B, C) + 0.5
    noise = torch.randn(B, 1, 2 * H, 2 * H)
    skip = torch.randn(B, 3, H, H)
    style = torch.randn(B, 16)
    with torch.no_grad():
        ref = sc.conv.blur(conv * demod[:, :, None, None])
        ref = sc.activate(sc.noise(ref, noise=noise))
        ref_rgb = trgb(ref, style, skip=skip)
        s = trgb.conv.modulation(style)
        rgb_w = (trgb.conv.scale * trgb.conv.weight[0, :, :, 0, 0])[None] * s[:, None, :]
    y, _ = oracle_mod.styled_epilogue(conv.numpy(), kernel2d=sc.conv.blur.kernel.numpy(),
                                      bias=sc.activate.bias.detach().numpy(), noise_weight=0.3,
                                      noise=noise.numpy(), demod=demod.numpy(), blur_up=True)
    np.testing.assert_allclose(y, ref.numpy(), rtol=1e-5, atol=1e-5)
    _, rgb = oracle_mod.styled_epilogue(ref.numpy() / math.sqrt(2), kernel2d=trgb.upsample.kernel.numpy(),
                                        bias=np.zeros(C), noise_weight=0.0, rgb_w=rgb_w.numpy(),
                                        rgb_b=trgb.bias.detach().numpy(), skip=skip.numpy(),
                                        slope=1.0, scale=math.sqrt(2))
    np.testing.assert_allclose(rgb, ref_rgb.numpy(), rtol=1e-5, atol=1e-5)
