"""StyleGAN2 decoder ops on libsdfr (drop-in for im2scene/sdf/models/sdf_op.py).

``fused_leaky_relu`` / ``FusedLeakyReLU`` (sdf_op.py:21-118) and ``upfirdn2d``
(sdf_op.py:133-271) keep the reference's split: CPU tensors take the
reference's own PyTorch formulas (sdf_op.py:106-114 and upfirdn2d_native
:273-316), GPU tensors take the HIP kernels (``sdfr_fused_bias_act``,
``sdfr_upfirdn2d``) through autograd Functions with the reference's backward
and double-backward structure.  A missing libsdfr.so raises; there is no
silent PyTorch substitute on the GPU.

``styled_epilogue`` / ``modulate_to_nhwc`` are the fused decoder pieces used
by ``Decoder`` on its inference path (see generator.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.autograd import Function

from . import _lib


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f"{tuple(t.shape)} must be a CUDA tensor")


# ---------------------------------------------------------------------------
# fused_bias_act (fused_bias_act.cpp:11 / fused_bias_act_kernel.cu:50-95)
# ---------------------------------------------------------------------------
def fused_bias_act(input, bias, refer, act, grad, alpha, scale):
    """Same contract as the reference's ``fused.fused_bias_act``: bias indexed
    along dim 1, ``refer``/``bias`` may be empty tensors."""
    _require_cuda(input, bias)
    x = input.contiguous()
    b = bias.contiguous() if bias is not None and bias.numel() else None
    r = refer.contiguous() if refer is not None and refer.numel() else None
    out = torch.empty_like(x)
    step_b = 1
    for d in range(2, x.dim()):
        step_b *= x.shape[d]
    L = _lib.lib()
    _lib.check(L.sdfr_fused_bias_act(_lib.ptr(out), _lib.ptr(x), _lib.ptr(b), _lib.ptr(r),
                                     x.numel(), step_b, 0 if b is None else b.numel(), act, grad,
                                     float(alpha), float(scale), _lib.stream_of(x)),
               "fused_bias_act")
    return out


class FusedLeakyReLUFunctionBackward(Function):
    """sdf_op.py:21-54."""

    @staticmethod
    def forward(ctx, grad_output, out, bias, negative_slope, scale):
        ctx.save_for_backward(out)
        ctx.negative_slope = negative_slope
        ctx.scale = scale
        empty = grad_output.new_empty(0)
        grad_input = fused_bias_act(grad_output, empty, out, 3, 1, negative_slope, scale)
        dim = [0] + list(range(2, grad_input.ndim))
        grad_bias = grad_input.sum(dim).detach() if bias else empty
        return grad_input, grad_bias

    @staticmethod
    def backward(ctx, gradgrad_input, gradgrad_bias):
        out, = ctx.saved_tensors
        gradgrad_out = fused_bias_act(gradgrad_input, gradgrad_bias, out, 3, 1,
                                      ctx.negative_slope, ctx.scale)
        return gradgrad_out, None, None, None, None


class FusedLeakyReLUFunction(Function):
    """sdf_op.py:57-85."""

    @staticmethod
    def forward(ctx, input, bias, negative_slope, scale):
        empty = input.new_empty(0)
        ctx.bias = bias is not None
        out = fused_bias_act(input, empty if bias is None else bias, empty, 3, 0,
                             negative_slope, scale)
        ctx.save_for_backward(out)
        ctx.negative_slope = negative_slope
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, grad_output):
        out, = ctx.saved_tensors
        grad_input, grad_bias = FusedLeakyReLUFunctionBackward.apply(
            grad_output, out, ctx.bias, ctx.negative_slope, ctx.scale)
        return grad_input, (grad_bias if ctx.bias else None), None, None


def fused_leaky_relu(input, bias=None, negative_slope=0.2, scale=2 ** 0.5):
    """sdf_op.py:105-118 (CPU: the reference's PyTorch formula, slope fixed at 0.2)."""
    if input.device.type == "cpu":
        if bias is not None:
            rest = [1] * (input.ndim - bias.ndim - 1)
            return F.leaky_relu(input + bias.view(1, bias.shape[0], *rest),
                                negative_slope=0.2) * scale
        return F.leaky_relu(input, negative_slope=0.2) * scale
    return FusedLeakyReLUFunction.apply(input, bias, negative_slope, scale)


class FusedLeakyReLU(nn.Module):
    """sdf_op.py:88-102 (same parameter name ``bias``)."""

    def __init__(self, channel, bias=True, negative_slope=0.2, scale=2 ** 0.5):
        super().__init__()
        if bias:
            self.bias = nn.Parameter(torch.zeros(channel))
        else:
            self.bias = None
        self.negative_slope = negative_slope
        self.scale = scale

    def forward(self, input):
        return fused_leaky_relu(input, self.bias, self.negative_slope, self.scale)


# ---------------------------------------------------------------------------
# upfirdn2d (upfirdn2d.cpp:12; autograd structure of sdf_op.py:133-256)
# ---------------------------------------------------------------------------
def _upfirdn2d_op(x, kernel, up_x, up_y, down_x, down_y, px0, px1, py0, py1):
    """x [major, in_h, in_w] -> [major, out_h, out_w] on the GPU."""
    _require_cuda(x, kernel)
    x = x.contiguous()
    k = kernel.to(device=x.device, dtype=torch.float32).contiguous()
    major, in_h, in_w = x.shape
    kh, kw = k.shape
    if min(up_x, up_y, down_x, down_y) < 1:
        raise RuntimeError("upfirdn2d: up and down factors must be >= 1")
    out_h = (in_h * up_y + py0 + py1 - kh) // down_y + 1
    out_w = (in_w * up_x + px0 + px1 - kw) // down_x + 1
    out = torch.empty(major, out_h, out_w, device=x.device, dtype=torch.float32)
    _lib.check(_lib.lib().sdfr_upfirdn2d(_lib.ptr(out), _lib.ptr(x), _lib.ptr(k), major, in_h,
                                         in_w, kh, kw, up_x, up_y, down_x, down_y, px0, px1,
                                         py0, py1, _lib.stream_of(x)), "upfirdn2d")
    return out


class UpFirDn2dBackward(Function):
    @staticmethod
    def forward(ctx, grad_output, kernel, grad_kernel, up, down, pad, g_pad, in_size, out_size):
        up_x, up_y = up
        down_x, down_y = down
        gx0, gx1, gy0, gy1 = g_pad
        g = grad_output.reshape(-1, out_size[0], out_size[1])
        grad_input = _upfirdn2d_op(g, grad_kernel, down_x, down_y, up_x, up_y, gx0, gx1, gy0, gy1)
        grad_input = grad_input.view(in_size[0], in_size[1], in_size[2], in_size[3])
        ctx.save_for_backward(kernel)
        ctx.up, ctx.down, ctx.pad = up, down, pad
        ctx.in_size, ctx.out_size = in_size, out_size
        return grad_input

    @staticmethod
    def backward(ctx, gradgrad_input):
        kernel, = ctx.saved_tensors
        gg = gradgrad_input.reshape(-1, ctx.in_size[2], ctx.in_size[3])
        px0, px1, py0, py1 = ctx.pad
        out = _upfirdn2d_op(gg, kernel, ctx.up[0], ctx.up[1], ctx.down[0], ctx.down[1],
                            px0, px1, py0, py1)
        out = out.view(ctx.in_size[0], ctx.in_size[1], ctx.out_size[0], ctx.out_size[1])
        return out, None, None, None, None, None, None, None, None


class UpFirDn2d(Function):
    @staticmethod
    def forward(ctx, input, kernel, up, down, pad):
        up_x, up_y = up
        down_x, down_y = down
        px0, px1, py0, py1 = pad
        kh, kw = kernel.shape
        batch, channel, in_h, in_w = input.shape
        ctx.in_size = input.shape
        ctx.save_for_backward(kernel, torch.flip(kernel, [0, 1]))
        out_h = (in_h * up_y + py0 + py1 - kh) // down_y + 1
        out_w = (in_w * up_x + px0 + px1 - kw) // down_x + 1
        ctx.out_size = (out_h, out_w)
        ctx.up, ctx.down, ctx.pad = (up_x, up_y), (down_x, down_y), (px0, px1, py0, py1)
        ctx.g_pad = (kw - px0 - 1, in_w * up_x - out_w * down_x + px0 - up_x + 1,
                     kh - py0 - 1, in_h * up_y - out_h * down_y + py0 - up_y + 1)
        out = _upfirdn2d_op(input.reshape(-1, in_h, in_w), kernel, up_x, up_y, down_x, down_y,
                            px0, px1, py0, py1)
        return out.view(-1, channel, out_h, out_w)

    @staticmethod
    def backward(ctx, grad_output):
        kernel, grad_kernel = ctx.saved_tensors
        grad_input = UpFirDn2dBackward.apply(grad_output, kernel, grad_kernel, ctx.up, ctx.down,
                                             ctx.pad, ctx.g_pad, ctx.in_size, ctx.out_size)
        return grad_input, None, None, None, None


def upfirdn2d_native(input, kernel, up_x, up_y, down_x, down_y, pad_x0, pad_x1, pad_y0, pad_y1):
    """The reference's PyTorch formulation (sdf_op.py:273-316), used for CPU tensors."""
    _, channel, in_h, in_w = input.shape
    kh, kw = kernel.shape
    x = input.reshape(-1, 1, in_h, in_w)
    if up_x > 1 or up_y > 1:
        z = x.new_zeros(x.shape[0], 1, in_h, up_y, in_w, up_x)
        z[:, :, :, 0, :, 0] = x.view(-1, 1, in_h, in_w)
        x = z.view(-1, 1, in_h * up_y, in_w * up_x)
    x = F.pad(x, [max(pad_x0, 0), max(pad_x1, 0), max(pad_y0, 0), max(pad_y1, 0)])
    x = x[:, :, max(-pad_y0, 0):x.shape[2] - max(-pad_y1, 0),
          max(-pad_x0, 0):x.shape[3] - max(-pad_x1, 0)]
    w = torch.flip(kernel, [0, 1]).to(x.dtype).view(1, 1, kh, kw)
    x = F.conv2d(x, w)
    x = x[:, :, ::down_y, ::down_x]
    out_h = (in_h * up_y + pad_y0 + pad_y1 - kh) // down_y + 1
    out_w = (in_w * up_x + pad_x0 + pad_x1 - kw) // down_x + 1
    return x.reshape(-1, channel, out_h, out_w)


def upfirdn2d(input, kernel, up=1, down=1, pad=(0, 0)):
    """sdf_op.py:259-270."""
    if input.device.type == "cpu":
        return upfirdn2d_native(input, kernel, up, up, down, down, pad[0], pad[1], pad[0], pad[1])
    return UpFirDn2d.apply(input, kernel, (up, up), (down, down), (pad[0], pad[1], pad[0], pad[1]))


# ---------------------------------------------------------------------------
# fused decoder pieces (no reference counterpart; include/sdfr.h)
# ---------------------------------------------------------------------------
def separable_taps(kernel_2d):
    """1-D taps f with outer(f, f) == kernel_2d exactly (4x4), else None."""
    k = kernel_2d.detach().float().cpu()
    if k.shape != (4, 4):
        return None
    f = k.diagonal().sqrt()
    if torch.equal(torch.outer(f, f), k):
        return [float(v) for v in f]
    return None


def modulate_to_nhwc(x, s):
    """x [B,C,H,W] (NCHW) * s[b,c] -> channels_last [B,C,H,W]."""
    _require_cuda(x, s)
    B, C, H, W = x.shape
    x = x.contiguous()
    s = s.contiguous()
    y = torch.empty(B, C, H, W, device=x.device, memory_format=torch.channels_last)
    _lib.check(_lib.lib().sdfr_modulate_to_nhwc(_lib.ptr(y), _lib.ptr(x), _lib.ptr(s), B, C,
                                                H * W, _lib.stream_of(x)), "modulate_to_nhwc")
    return y


def styled_epilogue(conv, *, fir, bias, noise_weight, noise=None, demod=None, blur_up=False,
                    s_next=None, store_y=True, rgb_w=None, rgb_b=None, skip=None,
                    negative_slope=0.2, act_scale=math.sqrt(2), split_y=False):
    """One pass after a decoder convolution (sdfr_styled_epilogue).

    conv: channels_last [B,C,Hc,Wc] (Hc = 2H+1 when blur_up).  Returns
    (y, rgb [B,3,H,W] or None) with y channels_last [B,C,H,W], or with split_y the
    split-NHWC fp16 tensor [B,H,W,C/8,2,8] that conv3x3_f16x3 reads, or None."""
    _require_cuda(conv)
    B, C, Hc, Wc = conv.shape
    H, W = (Hc - 1, Wc - 1) if blur_up else (Hc, Wc)
    conv = conv.contiguous(memory_format=torch.channels_last)
    y = (torch.empty(B, C, H, W, device=conv.device, memory_format=torch.channels_last)
         if store_y and not split_y else None)
    ys = None
    if store_y and split_y:
        ys = torch.empty(B, H, W, C // 8, 2, 8, device=conv.device, dtype=torch.float16)
    rgb = torch.empty(B, 3, H, W, device=conv.device) if rgb_w is not None else None
    if noise is not None:
        noise = noise.expand(B, 1, H, W).contiguous()
    a = _lib.StyledEpilogueArgs()
    a.B, a.C, a.H, a.W = B, C, H, W
    a.conv = _lib.ptr(conv)
    a.blur_up = int(blur_up)
    for i in range(4):
        a.fir[i] = fir[i]
    keep = []

    def cptr(t):
        if t is None:
            return None
        t = t.contiguous()
        keep.append(t)
        return _lib.ptr(t)

    a.demod = cptr(demod)
    a.noise = cptr(noise)
    a.noise_weight = cptr(noise_weight)
    a.bias = cptr(bias.reshape(-1))
    a.negative_slope = negative_slope
    a.act_scale = act_scale
    a.s_next = cptr(s_next)
    a.y = _lib.ptr(y)
    a.rgb_w = cptr(rgb_w)
    a.rgb_b = cptr(None if rgb_b is None else rgb_b.reshape(-1))
    a.skip = cptr(skip)
    a.rgb = _lib.ptr(rgb)
    a.y_split = _lib.ptr(ys)
    _lib.check(_lib.lib().sdfr_styled_epilogue(a, _lib.stream_of(conv)), "styled_epilogue")
    return (ys if split_y and store_y else y), rgb


# ---------------------------------------------------------------------------
# decoder convolutions on split-fp16 MFMA (csrc/conv_f16x3.hip)
# ---------------------------------------------------------------------------
def conv_pack_weights(weight, scale):
    """ModulatedConv2d weight [Cout, Cin, 3, 3] * scale -> (packed fragments, su [Cout]).
    The convolution result comes out multiplied by su (fold 1/su into demod)."""
    _require_cuda(weight)
    w = weight.detach().float().contiguous()
    Cout, Cin = w.shape[0], w.shape[1]
    nbytes = _lib.lib().sdfr_conv_pack_bytes(Cout, Cin) - 4 * Cout
    packed = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    su = torch.empty(Cout, dtype=torch.float32, device=w.device)
    _lib.check(_lib.lib().sdfr_conv_pack_weights(_lib.ptr(w), float(scale), Cout, Cin,
                                                 _lib.ptr(packed), _lib.ptr(su),
                                                 _lib.stream_of(w)), "conv_pack_weights")
    return packed, su


def split_nhwc(x):
    """fp32 tensor (any layout, logically [B,C,H,W], C % 8 == 0) -> the round-to-nearest
    fp16 split x = hi + lo (to ~2^-22) in the split-NHWC layout [B,H,W,C/8,2,8]: per
    pixel and group of 8 channels, 8 hi then 8 lo halves (include/sdfr.h)."""
    B, C, H, W = x.shape
    xh = x.permute(0, 2, 3, 1).reshape(B, H, W, C // 8, 1, 8)
    hi = xh.half()
    lo = (xh - hi.float()).half()
    return torch.cat([hi, lo], dim=4).contiguous()


def unsplit_nhwc(xs):
    """split-NHWC [B,H,W,C/8,2,8] fp16 -> (hi, lo) NHWC fp16 planes [B,H,W,C]."""
    B, H, W = xs.shape[:3]
    return xs[:, :, :, :, 0].reshape(B, H, W, -1), xs[:, :, :, :, 1].reshape(B, H, W, -1)


def conv3x3_f16x3(x_split, packed, Cout, transposed=False, split_k=True):
    """x_split = split-NHWC fp16 [B, H, W, Cin/8, 2, 8] (split_nhwc) -> channels_last
    fp32 [B, Cout, H, W] (conv2d, pad 1) or [B, Cout, 2H+1, 2W+1] (conv_transpose2d
    stride 2), scaled by su (conv_pack_weights).  ``split_k``: give the kernel a
    workspace so that small batches split K over 2-4 workgroups
    (sdfr_conv3x3_f16x3_ws)."""
    _require_cuda(x_split)
    if x_split.dtype != torch.float16 or x_split.dim() != 6 or x_split.shape[4:] != (2, 8) \
            or not x_split.is_contiguous():
        raise RuntimeError("conv3x3_f16x3: x_split must be a contiguous split-NHWC fp16 "
                           "tensor [B,H,W,Cin/8,2,8]")
    B, H, W, Cin = x_split.shape[0], x_split.shape[1], x_split.shape[2], 8 * x_split.shape[3]
    Ho, Wo = (2 * H + 1, 2 * W + 1) if transposed else (H, W)
    out = torch.empty(B, Cout, Ho, Wo, device=x_split.device, memory_format=torch.channels_last)
    wsb = _lib.lib().sdfr_conv_ws_bytes(B, H, W, Cout, int(bool(transposed))) if split_k else 0
    ws = torch.empty(wsb, dtype=torch.uint8, device=x_split.device) if wsb else None
    _lib.check(_lib.lib().sdfr_conv3x3_f16x3_ws(_lib.ptr(out), _lib.ptr(x_split),
                                                _lib.ptr(packed), B, H, W, Cin, Cout,
                                                int(bool(transposed)), _lib.ptr(ws), wsb,
                                                _lib.stream_of(x_split)),
               "conv3x3_f16x3")
    return out


def conv3x3_f16x3_act(x_split, packed, Cout, *, demod, bias, noise_weight, noise=None,
                      s_next=None, store_y=True, rgb_w=None, negative_slope=0.2,
                      act_scale=math.sqrt(2), split_k=True, rgb_base=None, rgb_s=None):
    """Regular conv with the plain styled epilogue fused (sdfr_conv3x3_f16x3_act):
    returns (y split-NHWC [B,H,W,Cout/8,2,8] or None, ToRGB partial sums
    [Cout/128,B,3,H,W] or None).  demod must already carry 1/su.  ``split_k``: give
    the kernel a workspace so that small batches split K over 2 or 4 workgroups.
    The ToRGB weight is ``rgb_w`` [B,3,Cout], or ``rgb_base`` [3,Cout] x ``rgb_s``
    [B,Cout] multiplied in the kernel (the same fp32 products, one launch less)."""
    if rgb_w is not None and rgb_base is not None:
        raise RuntimeError("conv3x3_f16x3_act: rgb_w and rgb_base are exclusive")
    _require_cuda(x_split)
    if x_split.dtype != torch.float16 or x_split.dim() != 6 or x_split.shape[4:] != (2, 8) \
            or not x_split.is_contiguous():
        raise RuntimeError("conv3x3_f16x3_act: x_split must be a contiguous split-NHWC fp16 "
                           "tensor [B,H,W,Cin/8,2,8]")
    B, H, W, Cin = x_split.shape[0], x_split.shape[1], x_split.shape[2], 8 * x_split.shape[3]
    dev = x_split.device
    ys = (torch.empty(B, H, W, Cout // 8, 2, 8, device=dev, dtype=torch.float16)
          if store_y else None)
    rgb = rgb_w is not None or rgb_base is not None
    part = torch.empty(Cout // 128, B, 3, H, W, device=dev) if rgb else None
    if noise is not None:
        noise = noise.expand(B, 1, H, W).contiguous()
    keep = []

    def cptr(t):
        if t is None:
            return None
        t = t.contiguous()
        keep.append(t)
        return _lib.ptr(t)

    a = _lib.ConvActArgs()
    a.x_split, a.packed = _lib.ptr(x_split), _lib.ptr(packed)
    a.B, a.H, a.W, a.Cin, a.Cout = B, H, W, Cin, Cout
    a.demod = cptr(demod)
    a.noise = cptr(noise)
    a.noise_weight = cptr(noise_weight)
    a.bias = cptr(bias.reshape(-1))
    a.negative_slope, a.act_scale = negative_slope, act_scale
    a.s_next = cptr(s_next)
    a.y_split = _lib.ptr(ys)
    a.rgb_w = cptr(rgb_w)
    a.rgb_base = cptr(rgb_base)
    a.rgb_s = cptr(rgb_s)
    a.rgb_partial = _lib.ptr(part)
    wsb = _lib.lib().sdfr_conv_act_ws_bytes(B, H, W, Cout) if split_k else 0
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev) if wsb else None
    a.ws, a.ws_bytes = _lib.ptr(ws), wsb
    _lib.check(_lib.lib().sdfr_conv3x3_f16x3_act(a, _lib.stream_of(x_split)), "conv3x3_f16x3_act")
    return ys, part


def conv_t_act_supported(x_split, Cout):
    """Does sdfr_conv_t_act take this upsampling layer (enough 64-channel x 16 x 16
    tiles to fill the chip: the batch sizes of the 32-face bench and above)?"""
    B, H, W, Cin = x_split.shape[0], x_split.shape[1], x_split.shape[2], 8 * x_split.shape[3]
    return bool(_lib.lib().sdfr_conv_t_act_supported(B, H, W, Cin, Cout))


def conv_t_act(x_split, packed, Cout, *, fir, demod, bias, noise_weight, noise=None,
               s_next=None, negative_slope=0.2, act_scale=math.sqrt(2)):
    """The upsampling StyledConv with its blur and styled epilogue in the conv kernel
    (sdfr_conv_t_act): returns y split-NHWC [B,2H,2W,Cout/8,2,8] fp16 -- the same bits
    as conv3x3_f16x3(transposed=True) followed by styled_epilogue(blur_up=True,
    split_y=True).  demod must already carry 1/su."""
    _require_cuda(x_split)
    if x_split.dtype != torch.float16 or x_split.dim() != 6 or x_split.shape[4:] != (2, 8) \
            or not x_split.is_contiguous():
        raise RuntimeError("conv_t_act: x_split must be a contiguous split-NHWC fp16 "
                           "tensor [B,H,W,Cin/8,2,8]")
    B, H, W, Cin = x_split.shape[0], x_split.shape[1], x_split.shape[2], 8 * x_split.shape[3]
    dev = x_split.device
    ys = torch.empty(B, 2 * H, 2 * W, Cout // 8, 2, 8, device=dev, dtype=torch.float16)
    raw = torch.empty(B, 2 * H + 1, 2 * W + 1, Cout, device=dev)
    if noise is not None:
        noise = noise.expand(B, 1, 2 * H, 2 * W).contiguous()
    keep = []

    def cptr(t):
        if t is None:
            return None
        t = t.contiguous()
        keep.append(t)
        return _lib.ptr(t)

    a = _lib.ConvTActArgs()
    a.x_split, a.packed = _lib.ptr(x_split), _lib.ptr(packed)
    a.B, a.H, a.W, a.Cin, a.Cout = B, H, W, Cin, Cout
    for i in range(4):
        a.fir[i] = fir[i]
    a.demod = cptr(demod)
    a.noise = cptr(noise)
    a.noise_weight = cptr(noise_weight)
    a.bias = cptr(bias.reshape(-1))
    a.negative_slope, a.act_scale = negative_slope, act_scale
    a.s_next = cptr(s_next)
    a.y_split = _lib.ptr(ys)
    a.raw = _lib.ptr(raw)
    _lib.check(_lib.lib().sdfr_conv_t_act(a, _lib.stream_of(x_split)), "conv_t_act")
    return ys


def rgb_finish(partial, rgb_b, skip=None, fir=None):
    """ToRGB output [B,3,H,W] = partial.sum(0) + rgb_b + upsampled skip (sdfr_rgb_finish)."""
    _require_cuda(partial)
    n, B, _, H, W = partial.shape
    partial = partial.contiguous()
    rgb = torch.empty(B, 3, H, W, device=partial.device)
    rgb_b = rgb_b.reshape(-1).contiguous()
    skip = skip.contiguous() if skip is not None else None
    f = (_lib._f32 * 4)(*(fir if fir is not None else [0.0] * 4))
    _lib.check(_lib.lib().sdfr_rgb_finish(_lib.ptr(rgb), _lib.ptr(partial), n, _lib.ptr(rgb_b),
                                          _lib.ptr(skip), f, B, H, W,
                                          _lib.stream_of(partial)), "rgb_finish")
    return rgb


def modulate_to_nhwc_split(x, s):
    """(x * s[:, :, None, None]) in the split-NHWC fp16 layout [B,H,W,C/8,2,8], from
    NCHW fp32 x."""
    _require_cuda(x, s)
    B, C, H, W = x.shape
    x = x.contiguous()
    s = s.contiguous()
    ys = torch.empty(B, H, W, C // 8, 2, 8, device=x.device, dtype=torch.float16)
    _lib.check(_lib.lib().sdfr_modulate_to_nhwc_split(_lib.ptr(ys), _lib.ptr(x), _lib.ptr(s),
                                                      B, C, H * W, _lib.stream_of(x)),
               "modulate_to_nhwc_split")
    return ys
