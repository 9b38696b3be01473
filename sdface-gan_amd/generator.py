"""Generator (mapping + fused renderer + StyleGAN2 decoder), drop-in API.

Follows im2scene/sdf/models/sdf_model.py:
  MappingLinear :437-466   Upsample/Blur :480-538    EqualLinear :579-611
  ModulatedConv2d :614-701 NoiseInjection :704-792   StyledConv :795-818
  ToRGB :821-843           Decoder :883-1056         Generator :1059-1216
and the device-agnostic forms of the fused ops of sdf_op.py:105-120 / 259-314.

The decoder's convolutions stay on MIOpen.  Its modulated
convolution runs as ``conv(x * s, W) * demod`` -- one batched convolution
instead of the reference's per-face grouped convolution (same algebra, fp32).
On the GPU, the bias/leaky-ReLU and upfirdn2d ops are the HIP kernels of
decoder_ops.py; at inference (no grad) everything between two convolutions is
one HIP epilogue over channels_last activations (``Decoder._fused_forward``).
Geometry-aware noise projection (``project_noise``, pytorch3d) is not
supported and raises.
"""
from __future__ import annotations

import math
import random

import torch
import torch.nn as nn
import torch.nn.functional as F

from .decoder_ops import (conv3x3_f16x3, conv3x3_f16x3_act, conv_pack_weights,  # noqa: E402
                          conv_t_act, conv_t_act_supported, modulate_to_nhwc_split, rgb_finish)
from .decoder_ops import (FusedLeakyReLU, fused_leaky_relu, modulate_to_nhwc,  # noqa: F401
                          separable_taps, styled_epilogue, upfirdn2d)
from .renderer import VolumeFeatureRenderer


def make_kernel(k):
    k = torch.tensor(k, dtype=torch.float32)
    if k.ndim == 1:
        k = k[None, :] * k[:, None]
    return k / k.sum()


_EMPTY = {}                      # device -> a 0-element tensor (fused_ready's probe)

class Upsample(nn.Module):
    def __init__(self, kernel, factor=2):
        super().__init__()
        self.factor = factor
        self.register_buffer("kernel", make_kernel(kernel) * (factor ** 2))
        p = self.kernel.shape[0] - factor
        self.pad = ((p + 1) // 2 + factor - 1, p // 2)

    def forward(self, input):
        return upfirdn2d(input, self.kernel, up=self.factor, down=1, pad=self.pad)


class Blur(nn.Module):
    def __init__(self, kernel, pad, upsample_factor=1):
        super().__init__()
        k = make_kernel(kernel)
        if upsample_factor > 1:
            k = k * (upsample_factor ** 2)
        self.register_buffer("kernel", k)
        self.pad = pad

    def forward(self, input):
        return upfirdn2d(input, self.kernel, pad=self.pad)


class PixelNorm(nn.Module):
    def forward(self, input):
        return input * torch.rsqrt(torch.mean(input ** 2, dim=1, keepdim=True) + 1e-8)


class MappingLinear(nn.Module):
    """Renderer mapping layer (sdf_model.py:437-466)."""

    def __init__(self, in_dim, out_dim, bias=True, activation=None, is_last=False):
        super().__init__()
        std = 0.25 if is_last else 1
        self.weight = nn.Parameter(std * nn.init.kaiming_normal_(
            torch.empty(out_dim, in_dim), a=0.2, mode="fan_in", nonlinearity="leaky_relu"))
        if bias:
            lim = math.sqrt(1 / in_dim)
            self.bias = nn.Parameter(nn.init.uniform_(torch.empty(out_dim), a=-lim, b=lim))
        else:
            self.bias = None
        self.activation = activation

    def forward(self, input):
        if self.activation is not None:
            return fused_leaky_relu(F.linear(input, self.weight), self.bias, scale=1)
        return F.linear(input, self.weight, bias=self.bias)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.weight.shape[1]}, {self.weight.shape[0]})"


class EqualLinear(nn.Module):
    def __init__(self, in_dim, out_dim, bias=True, bias_init=0, lr_mul=1, activation=None):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(out_dim, in_dim).div_(lr_mul))
        self.bias = nn.Parameter(torch.zeros(out_dim).fill_(bias_init)) if bias else None
        self.activation = activation
        self.scale = (1 / math.sqrt(in_dim)) * lr_mul
        self.lr_mul = lr_mul

    def forward(self, input):
        if self.activation:
            return fused_leaky_relu(F.linear(input, self.weight * self.scale),
                                    self.bias * self.lr_mul)
        return F.linear(input, self.weight * self.scale, bias=self.bias * self.lr_mul)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.weight.shape[1]}, {self.weight.shape[0]})"


def mapping_forward(seq, x):
    """A mapping network (nn.Sequential of PixelNorm / EqualLinear / MappingLinear) on
    the inference path: one HIP launch per linear layer (``sdfr_mapping_linear``,
    PixelNorm folded into the next layer) when ``x`` is on the GPU and no gradient
    is recorded; the modules themselves otherwise.  Same per-element arithmetic
    (W * scale, b * lr_mul, x + b, leaky ReLU, * scale); the dot products are
    summed in a different order than the GEMM's (fp32 rounding level)."""
    if not (x.is_cuda and not torch.is_grad_enabled() and x.dtype == torch.float32
            and x.dim() == 2):
        return seq(x)
    from . import _lib
    L = _lib.lib()
    pixelnorm = 0
    for m in seq:
        if isinstance(m, PixelNorm):
            pixelnorm = 1
            continue
        if isinstance(m, EqualLinear):
            wscale, bscale, act_scale = m.scale, m.lr_mul, 2 ** 0.5
        elif isinstance(m, MappingLinear):
            wscale, bscale, act_scale = 1.0, 1.0, 1.0
        else:
            return seq(x)                          # unknown layer: module path
        w = m.weight.detach()
        if w.shape[1] not in (256, 512) or not w.is_contiguous():
            return seq(x)
        x = x.contiguous()
        out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=torch.float32)
        _lib.check(L.sdfr_mapping_linear(
            _lib.ptr(out), _lib.ptr(x), _lib.ptr(w),
            _lib.ptr(m.bias.detach()) if m.bias is not None else None, x.shape[0], w.shape[1],
            w.shape[0], float(wscale), float(bscale), int(m.activation is not None), 0.2,
            float(act_scale), pixelnorm, _lib.stream_of(x)), "sdfr_mapping_linear")
        x, pixelnorm = out, 0
    if pixelnorm:
        return seq[-1](x)
    return x


class ModulatedConv2d(nn.Module):
    def __init__(self, in_channel, out_channel, kernel_size, style_dim, demodulate=True,
                 upsample=False, downsample=False, blur_kernel=(1, 3, 3, 1)):
        super().__init__()
        self.eps = 1e-8
        self.kernel_size = kernel_size
        self.in_channel = in_channel
        self.out_channel = out_channel
        self.upsample = upsample
        self.downsample = downsample
        if upsample:
            factor = 2
            p = (len(blur_kernel) - factor) - (kernel_size - 1)
            self.blur = Blur(blur_kernel, pad=((p + 1) // 2 + factor - 1, p // 2 + 1),
                             upsample_factor=factor)
        if downsample:
            factor = 2
            p = (len(blur_kernel) - factor) + (kernel_size - 1)
            self.blur = Blur(blur_kernel, pad=((p + 1) // 2, p // 2))
        self.scale = 1 / math.sqrt(in_channel * kernel_size ** 2)
        self.padding = kernel_size // 2
        self.weight = nn.Parameter(torch.randn(1, out_channel, in_channel, kernel_size,
                                               kernel_size))
        self.modulation = EqualLinear(style_dim, in_channel, bias_init=1)
        self.demodulate = demodulate

    def __repr__(self):
        return (f"{self.__class__.__name__}({self.in_channel}, {self.out_channel}, "
                f"{self.kernel_size}, upsample={self.upsample}, downsample={self.downsample})")

    def forward(self, input, style):
        batch = input.shape[0]
        s = self.modulation(style)                                   # [B, in]
        w = self.scale * self.weight[0]                              # [out, in, k, k]
        x = input * s.view(batch, -1, 1, 1)
        if self.upsample:
            out = F.conv_transpose2d(x, w.transpose(0, 1), padding=0, stride=2)
        elif self.downsample:
            out = F.conv2d(self.blur(x), w, padding=0, stride=2)
        else:
            out = F.conv2d(x, w, padding=self.padding)
        if self.demodulate:
            wsq = (w * w).sum([2, 3])                                # [out, in]
            demod = torch.rsqrt((s * s) @ wsq.t() + 1e-8)            # [B, out]
            out = out * demod.view(batch, -1, 1, 1)
        if self.upsample:
            out = self.blur(out)
        return out


class NoiseInjection(nn.Module):
    def __init__(self, project=False):
        super().__init__()
        self.project = project
        self.weight = nn.Parameter(torch.zeros(1))
        self.prev_noise = None
        self.mesh_fn = None
        self.vert_noise = None

    def forward(self, image, noise=None, transform=None, mesh_path=None):
        batch, _, height, width = image.shape
        if noise is None:
            noise = image.new_empty(batch, 1, height, width).normal_()
        elif self.project:
            raise NotImplementedError("geometry-aware noise projection (pytorch3d) is not "
                                      "part of this framework")
        return image + self.weight * noise


class StyledConv(nn.Module):
    def __init__(self, in_channel, out_channel, kernel_size, style_dim, upsample=False,
                 blur_kernel=(1, 3, 3, 1), project_noise=False):
        super().__init__()
        self.conv = ModulatedConv2d(in_channel, out_channel, kernel_size, style_dim,
                                    upsample=upsample, blur_kernel=blur_kernel)
        self.noise = NoiseInjection(project=project_noise)
        self.bias = nn.Parameter(torch.zeros(1, out_channel, 1, 1))
        self.activate = FusedLeakyReLU(out_channel)

    def forward(self, input, style, noise=None, transform=None, mesh_path=None):
        out = self.conv(input, style)
        out = self.noise(out, noise=noise, transform=transform, mesh_path=mesh_path)
        return self.activate(out)


class ToRGB(nn.Module):
    def __init__(self, in_channel, style_dim, upsample=True, blur_kernel=(1, 3, 3, 1)):
        super().__init__()
        self.upsample = Upsample(blur_kernel) if upsample else upsample
        self.conv = ModulatedConv2d(in_channel, 3, 1, style_dim, demodulate=False)
        self.bias = nn.Parameter(torch.zeros(1, 3, 1, 1))

    def forward(self, input, style, skip=None):
        out = self.conv(input, style) + self.bias
        if skip is not None:
            if self.upsample:
                skip = self.upsample(skip)
            out = out + skip
        return out


class Decoder(nn.Module):
    """StyleGAN2 2D decoder, 64^2 x 256 features -> size^2 RGB (sdf_model.py:883-1056)."""

    def __init__(self, model_opt, blur_kernel=(1, 3, 3, 1)):
        super().__init__()
        o = model_opt
        self.size = o.size
        self.style_dim = o.style_dim * 2
        in_dim = self.style_dim if o.psp else self.style_dim // 2
        layers = [PixelNorm(), EqualLinear(in_dim, self.style_dim, lr_mul=o.lr_mapping,
                                           activation="fused_lrelu")]
        for _ in range(4):
            layers.append(EqualLinear(self.style_dim, self.style_dim, lr_mul=o.lr_mapping,
                                      activation="fused_lrelu"))
        self.style = nn.Sequential(*layers)
        cm = o.channel_multiplier
        self.channels = {4: 512, 8: 512, 16: 512, 32: 512, 64: 256 * cm, 128: 128 * cm,
                         256: 64 * cm, 512: 32 * cm, 1024: 16 * cm}
        dec_in = o.renderer_spatial_output_dim
        self.log_size = int(math.log(self.size, 2))
        self.log_in_size = int(math.log(dec_in, 2))
        in_feat = o.feature_encoder_in_channels if not o.psp else self.style_dim
        self.conv1 = StyledConv(in_feat, self.channels[dec_in], 3, self.style_dim,
                                blur_kernel=blur_kernel, project_noise=o.project_noise)
        self.to_rgb1 = ToRGB(self.channels[dec_in], self.style_dim, upsample=False)
        self.num_layers = (self.log_size - self.log_in_size) * 2 + 1
        self.convs = nn.ModuleList()
        self.upsamples = nn.ModuleList()
        self.to_rgbs = nn.ModuleList()
        self.noises = nn.Module()
        in_ch = self.channels[dec_in]
        for idx in range(self.num_layers):
            res = (idx + 2 * self.log_in_size + 1) // 2
            self.noises.register_buffer(f"noise_{idx}", torch.randn(1, 1, 2 ** res, 2 ** res))
        for i in range(self.log_in_size + 1, self.log_size + 1):
            out_ch = self.channels[2 ** i]
            self.convs.append(StyledConv(in_ch, out_ch, 3, self.style_dim, upsample=True,
                                         blur_kernel=blur_kernel,
                                         project_noise=o.project_noise))
            self.convs.append(StyledConv(out_ch, out_ch, 3, self.style_dim,
                                         blur_kernel=blur_kernel,
                                         project_noise=o.project_noise))
            self.to_rgbs.append(ToRGB(out_ch, self.style_dim))
            in_ch = out_ch
        self.n_latent = (self.log_size - self.log_in_size) * 2 + 2
        self.use_fused = True      # HIP epilogues on the inference path (GPU, no grad)
        # convolutions of the fused path: "f16x3" (split-fp16 MFMA implicit GEMM,
        # csrc/conv_f16x3.hip) or "miopen" (F.conv2d / conv_transpose2d, fp32)
        self.conv_impl = "f16x3"
        # regular f16x3 convs with the styled epilogue fused into the conv kernel
        # (sdfr_conv3x3_f16x3_act + sdfr_rgb_finish) instead of a separate pass
        self.fuse_conv_act = True
        # upsampling convs with the blur + styled epilogue inside conv_t_kernel
        # (sdfr_conv_t_act) wherever that kernel runs (>= 256 tiles: batches of 4+)
        self.fuse_conv_t_blur = True
        # profiling: (start, end) HIP event pairs recorded on the current stream around
        # the fused regular convolutions (conv_h_kernel) of the next forward, in order,
        # and their fp32-equivalent FLOPs (bench.py's decoder roofline)
        self.conv_events = None
        self.conv_flops = 0
        self._conv_ev = 0
        self._fir = None
        self._packs = {}
        self._mod_stack = None
        self._demod_stack = None

    def mean_latent(self, renderer_latent):
        return self.style(renderer_latent).mean(0, keepdim=True)

    def get_latent(self, input):
        return self.style(input)

    def styles_and_noise_forward(self, styles, noise, inject_index=None, truncation=1,
                                 truncation_latent=None, input_is_latent=False,
                                 randomize_noise=True):
        if not input_is_latent:
            styles = [mapping_forward(self.style, s) for s in styles]
        if noise is None:
            noise = ([None] * self.num_layers if randomize_noise else
                     [getattr(self.noises, f"noise_{i}") for i in range(self.num_layers)])
        if truncation < 1:
            styles = [truncation_latent[1] + truncation * (s - truncation_latent[1])
                      for s in styles]
        if len(styles) < 2:
            inject_index = self.n_latent
            latent = (styles[0].unsqueeze(1).repeat(1, inject_index, 1)
                      if styles[0].ndim < 3 else styles[0])
        else:
            if inject_index is None:
                inject_index = random.randint(1, self.n_latent - 1)
            latent = torch.cat([styles[0].unsqueeze(1).repeat(1, inject_index, 1),
                                styles[1].unsqueeze(1).repeat(1, self.n_latent - inject_index, 1)],
                               1)
        return latent, noise

    def forward(self, features, styles, rgbd_in=None, transform=None, return_latents=False,
                inject_index=None, truncation=1, truncation_latent=None, input_is_latent=False,
                noise=None, randomize_noise=True, mesh_path=None, prepared=None):
        if prepared is not None:         # prepare_fused() ran earlier (Generator.forward)
            latent, noise, sty = prepared
            if self._fused_ok(features, rgbd_in, transform):
                return (self._fused_forward(features, latent, noise, sty),
                        (latent if return_latents else None))
            # the features turned out to need the autograd path (they require grad):
            # run the module path below on the prep's latent and noise maps -- drawing
            # them again would shift the RNG streams against the reference's order
        else:
            latent, noise = self.styles_and_noise_forward(styles, noise, inject_index,
                                                          truncation, truncation_latent,
                                                          input_is_latent, randomize_noise)
            if self._fused_ok(features, rgbd_in, transform):
                return (self._fused_forward(features, latent, noise),
                        (latent if return_latents else None))
        out = self.conv1(features, latent[:, 0], noise=noise[0], transform=transform,
                         mesh_path=mesh_path)
        skip = self.to_rgb1(out, latent[:, 1], skip=rgbd_in)
        i = 1
        for c1, c2, n1, n2, to_rgb in zip(self.convs[::2], self.convs[1::2], noise[1::2],
                                          noise[2::2], self.to_rgbs):
            out = c1(out, latent[:, i], noise=n1, transform=transform, mesh_path=mesh_path)
            out = c2(out, latent[:, i + 1], noise=n2, transform=transform, mesh_path=mesh_path)
            skip = to_rgb(out, latent[:, i + 2], skip=skip)
            i += 2
        return skip, (latent if return_latents else None)

    # -- fused inference path ------------------------------------------------
    def _fused_ok(self, features, rgbd_in, transform):
        if not (self.use_fused and features.is_cuda and rgbd_in is None and transform is None):
            return False
        if torch.is_grad_enabled() and (features.requires_grad or
                                        any(p.requires_grad for p in self.parameters())):
            return False
        if self._fir is None:
            fir = separable_taps(self.convs[0].conv.blur.kernel) if len(self.convs) else [0.0] * 4
            ok = fir is not None and all(
                torch.equal(t.upsample.kernel.cpu(), self.convs[0].conv.blur.kernel.cpu())
                for t in self.to_rgbs)
            self._fir = fir if ok else False
        return self._fir is not False

    def fused_ready(self, device, transform=None, rgbd_in=None):
        """Will forward() take the fused path for features on ``device``?  (Checked
        before the features exist, so that prepare_fused can run beside the renderer.)"""
        if device.type != "cuda":
            return False
        probe = _EMPTY.get(device)
        if probe is None:
            probe = _EMPTY[device] = torch.empty(0, device=device)
        return self._fused_ok(probe, rgbd_in, transform)

    def prepare_fused(self, styles, B, device, noise=None, inject_index=None, truncation=1,
                      truncation_latent=None, input_is_latent=False, randomize_noise=True):
        """Everything of the fused forward that does not depend on the features: the
        mapping network, the noise maps and every layer's modulation / demodulation;
        forward(..., prepared=<this>) then runs the convolutions.  The same work, in
        the same order, as forward() does it."""
        latent, noise = self.styles_and_noise_forward(styles, noise, inject_index, truncation,
                                                      truncation_latent, input_is_latent,
                                                      randomize_noise)
        seq = [self.conv1] + list(self.convs)
        noise = self._fused_noise(noise, B, device, torch.float32)
        split = [self._conv_x(sc.conv) for sc in seq]
        return latent, noise, self._fused_styles(latent, seq, split)

    def _fused_styles(self, latent, seq, split):
        if latent.is_cuda and latent.dtype == torch.float32 and self.style_dim in (256, 512):
            return self._styles_fused(latent, seq, split)
        mods, rgb_mods, mods_raw = self._modulations(latent)
        return mods, rgb_mods, self._demods(seq, split, mods_raw)

    def _conv_x(self, mc):
        """Does this ModulatedConv2d run on the split-fp16 implicit GEMM?"""
        _, cout, cin, k, _ = mc.weight.shape
        return (self.conv_impl == "f16x3" and k == 3 and mc.demodulate and not mc.downsample
                and cout % 128 == 0 and cin % 32 == 0)

    def _pack(self, i, mc):
        """Per weight version of layer i: the packed split-fp16 weights, their row
        scales su and, for the demodulation, su^2 * sum_{ky,kx} w^2 as [Cin, Cout]
        plus su^2 * 1e-8: rsqrt(s^2 @ that + that) is demod / su exactly (powers
        of two commute with rounding), in one GEMM + one rsqrt per call."""
        key = (mc.weight.data_ptr(), mc.weight._version, mc.weight.device)
        hit = self._packs.get(i)
        if hit is None or hit[0] != key:
            packed, su = conv_pack_weights(mc.weight[0], mc.scale)
            with torch.no_grad():
                w = mc.scale * mc.weight[0]
                s2 = su * su
                wsq = ((w * w).sum([2, 3]) * s2[:, None]).t().contiguous()
                eps = s2 * 1e-8
            hit = (key, packed, su, wsq, eps)
            self._packs[i] = hit
        return hit[1:]

    def _modulations(self, latent):
        """Every conv and ToRGB modulation of the fused path (EqualLinear,
        sdf_model.py:676-699) as ONE batched GEMM: the 11 weight matrices
        (x scale, zero-padded to the widest) and biases (x lr_mul) are stacked once
        per weight version, latent rows gathered per layer; one baddbmm instead of
        three small kernels per layer.  fp32, summation order of the batched GEMM."""
        seq = [self.conv1] + list(self.convs)
        rgbs = [self.to_rgb1] + list(self.to_rgbs)
        lins = [sc.conv.modulation for sc in seq] + [t.conv.modulation for t in rgbs]
        key = tuple((m.weight.data_ptr(), m.weight._version, m.bias._version) for m in lins)
        if self._mod_stack is None or self._mod_stack[0] != key:
            cmax = max(m.weight.shape[0] for m in lins)
            w0 = lins[0].weight
            wt = w0.new_zeros(len(lins), w0.shape[1], cmax)
            bs = w0.new_zeros(len(lins), 1, cmax)
            with torch.no_grad():
                for k, m in enumerate(lins):
                    c = m.weight.shape[0]
                    wt[k, :, :c] = (m.weight * m.scale).t()
                    bs[k, 0, :c] = m.bias * m.lr_mul
            # latent index per stacked layer: conv i -> i, ToRGB k -> 2k + 1
            idx = torch.tensor(list(range(len(seq))) + [2 * k + 1 for k in range(len(rgbs))],
                               device=w0.device)
            self._mod_stack = (key, wt, bs, idx, [m.weight.shape[0] for m in lins], len(seq))
        _, wt, bs, idx, cins, nconv = self._mod_stack
        out = torch.baddbmm(bs, latent.index_select(1, idx).transpose(0, 1), wt)
        mods = [out[k, :, :c].contiguous() for k, c in enumerate(cins)]
        return mods[:nconv], mods[nconv:], out[:nconv]

    def _demods(self, seq, split, mods_raw):
        """demod / su of every split-fp16 layer (see _pack) in one batched GEMM +
        one rsqrt: the layers' [Cin, Cout] weight sums and eps rows are stacked
        (zero-padded) once per weight version; mods_raw is _modulations' padded
        [layers, B, Cmax] output (its padding is exactly 0)."""
        layers = [i for i, sc in enumerate(seq) if split[i] and sc.conv.demodulate]
        if not layers:
            return {}
        packs = {i: self._pack(i, seq[i].conv) for i in layers}
        key = tuple(self._packs[i][0] for i in layers)
        if getattr(self, "_demod_stack", None) is None or self._demod_stack[0] != key:
            cmax = mods_raw.shape[-1]
            omax = max(packs[i][2].shape[1] for i in layers)
            w0 = packs[layers[0]][2]
            wsq = w0.new_zeros(len(layers), cmax, omax)
            eps = w0.new_zeros(len(layers), 1, omax)
            for j, i in enumerate(layers):
                cin, cout = packs[i][2].shape
                wsq[j, :cin, :cout] = packs[i][2]
                eps[j, 0, :cout] = packs[i][3]
            sel = torch.tensor(layers, device=w0.device)
            self._demod_stack = (key, wsq, eps, sel)
        _, wsq, eps, sel = self._demod_stack
        m = mods_raw.index_select(0, sel)
        d = torch.rsqrt(torch.baddbmm(eps, m * m, wsq))
        return {i: d[j, :, :packs[i][2].shape[1]].contiguous() for j, i in enumerate(layers)}

    def _styles_fused(self, latent, seq, split):
        """_modulations + _demods in two HIP launches (sdfr_decoder_styles): the
        stacked, scaled weights are built once per weight version; the per-layer
        modulations and demodulations come back as contiguous slices of two flat
        buffers.  fp32, fixed summation order (not the batched GEMM's)."""
        from . import _lib
        rgbs = [self.to_rgb1] + list(self.to_rgbs)
        lins = [sc.conv.modulation for sc in seq] + [t.conv.modulation for t in rgbs]
        nconv = len(seq)
        key = tuple((m.weight.data_ptr(), m.weight._version, m.bias._version) for m in lins)
        cache = getattr(self, "_sty_mod", None)
        if cache is None or cache[0] != key:
            cmax = max(256, max(m.weight.shape[0] for m in lins))
            w0 = lins[0].weight
            mw = w0.new_zeros(len(lins), cmax, w0.shape[1])
            mb = w0.new_zeros(len(lins), cmax)
            with torch.no_grad():
                for k, m in enumerate(lins):
                    c = m.weight.shape[0]
                    mw[k, :c] = m.weight * m.scale
                    mb[k, :c] = m.bias * m.lr_mul
            idx = list(range(nconv)) + [2 * k + 1 for k in range(len(rgbs))]
            cache = (key, mw, mb, idx, [m.weight.shape[0] for m in lins], cmax)
            self._sty_mod = cache
        _, mw, mb, idx, couts, cmax = cache
        layers = [i for i, sc in enumerate(seq) if split[i] and sc.conv.demodulate]
        packs = {i: self._pack(i, seq[i].conv) for i in layers}
        dkey = tuple(self._packs[i][0] for i in layers)
        dcache = getattr(self, "_sty_dem", None)
        if layers and (dcache is None or dcache[0] != dkey):
            omax = max(packs[i][2].shape[1] for i in layers)
            w0 = packs[layers[0]][2]
            dw = w0.new_zeros(len(layers), omax, cmax)
            de = w0.new_zeros(len(layers), omax)
            for j, i in enumerate(layers):
                cin, cout = packs[i][2].shape
                dw[j, :cout, :cin] = packs[i][2].t()
                de[j, :cout] = packs[i][3]
            dcache = (dkey, dw, de, omax)
            self._sty_dem = dcache
        B = latent.shape[0]
        lat = latent.contiguous()
        a = _lib.StyleArgs()
        a.B, a.n_latent, a.K, a.latent = B, lat.shape[1], lat.shape[2], _lib.ptr(lat)
        a.L, a.cmax, a.mod_w, a.mod_b = len(lins), cmax, _lib.ptr(mw), _lib.ptr(mb)
        offs, off = [], 0
        for k, c in enumerate(couts):
            a.mod_index[k], a.mod_c[k], a.mod_off[k] = idx[k], c, off
            offs.append(off)
            off += B * c
        mflat = torch.empty(off, device=lat.device)
        a.mods = _lib.ptr(mflat)
        dflat = None
        if layers:
            _, dw, de, omax = dcache
            a.J, a.omax, a.dem_w, a.dem_eps = len(layers), omax, _lib.ptr(dw), _lib.ptr(de)
            doffs, doff = [], 0
            for j, i in enumerate(layers):
                cout = packs[i][2].shape[1]
                a.dem_layer[j], a.dem_c[j], a.dem_off[j] = i, cout, doff
                doffs.append(doff)
                doff += B * cout
            dflat = torch.empty(doff, device=lat.device)
            a.demods = _lib.ptr(dflat)
        _lib.check(_lib.lib().sdfr_decoder_styles(a, _lib.stream_of(lat)), "sdfr_decoder_styles")
        mods = [mflat[o:o + B * c].view(B, c) for o, c in zip(offs, couts)]
        demods = {}
        if layers:
            for j, i in enumerate(layers):
                cout = packs[i][2].shape[1]
                demods[i] = dflat[doffs[j]:doffs[j] + B * cout].view(B, cout)
        return mods[:nconv], mods[nconv:], demods

    def _fused_noise(self, noise, B, device, dtype):
        """The per-layer noise maps of the fused path: the given ones, and every
        missing one (randomize_noise) sliced from ONE standard-normal draw of all of
        their elements, layer after layer -- one launch instead of one per layer (the
        module path draws each layer's map separately, NoiseInjection, so the two
        paths' random maps differ; their distribution does not)."""
        missing = [i for i, n in enumerate(noise) if n is None]
        if not missing:
            return noise
        sizes = [2 ** ((i + 2 * self.log_in_size + 1) // 2) for i in range(self.num_layers)]
        total = sum(B * sizes[i] * sizes[i] for i in missing)
        flat = torch.randn(total, device=device, dtype=dtype)
        out, off = list(noise), 0
        for i in missing:
            n = B * sizes[i] * sizes[i]
            out[i] = flat[off:off + n].view(B, 1, sizes[i], sizes[i])
            off += n
        return out

    def _rgb_base(self, tc):
        """ToRGB's scaled 1x1 weight [3, C] (tc.scale * weight), once per weight version."""
        key = (tc.weight.data_ptr(), tc.weight._version)
        cache = getattr(tc, "_sdfr_base", None)
        if cache is None or cache[0] != key:
            with torch.no_grad():
                cache = (key, tc.scale * tc.weight[0, :, :, 0, 0])
            tc._sdfr_base = cache
        return cache[1]

    def profile_convs(self, events):
        """Record `events[k] = (start, end)` around the k-th fused regular convolution of
        the next forward (None: stop); `conv_flops` counts their fp32-equivalent FLOPs."""
        self.conv_events, self._conv_ev, self.conv_flops = events, 0, 0

    @staticmethod
    def _fused_chunk(features, seq):
        """Faces per fused call: the largest activation of one face (a layer's input,
        or its raw output -- (2H+1) x (2W+1) for an upsampling layer -- in 4-byte
        elements) times the batch stays below 2^31 bytes (the 256^2 decoder: 63 faces)."""
        h, w = (features.shape[1:3] if features.dim() == 6 else features.shape[2:4])
        per_face = 0
        for sc in seq:
            cout, cin = sc.conv.weight.shape[1], sc.conv.weight.shape[2]
            per_face = max(per_face, h * w * cin * 4)
            if sc.conv.upsample:
                per_face = max(per_face, (2 * h + 1) * (2 * w + 1) * cout * 4)
                h, w = 2 * h, 2 * w
            per_face = max(per_face, h * w * cout * 4)
        return max(1, ((1 << 31) - 1) // per_face)

    @staticmethod
    def _noise_rows(noise, sl, B):
        """Faces ``sl`` of the per-layer noise maps: a [B, 1, h, w] map is sliced, a
        shared [1, 1, h, w] map (the decoder's fixed noise buffers) is kept."""
        return [n[sl] if n is not None and n.shape[0] == B else n for n in noise]

    @staticmethod
    def _style_rows(sty, sl):
        """Faces ``sl`` of _fused_styles' (mods, rgb_mods, demods): every modulation and
        demodulation is [B, C]."""
        mods, rgb_mods, demods = sty
        return ([m[sl] for m in mods], [m[sl] for m in rgb_mods],
                {i: d[sl] for i, d in demods.items()})

    def _fused_forward(self, features, latent, noise, sty=None):
        """Same computation as the module path: per layer one split-fp16 convolution
        (or MIOpen's) plus one sdfr_styled_epilogue on NHWC activations -- for the
        regular convolutions the epilogue runs inside the conv kernel
        (sdfr_conv3x3_f16x3_act); each activation is pre-multiplied by the next
        layer's modulation and the ToRGB layers are folded into the preceding
        epilogue."""
        cl = torch.channels_last
        B = features.shape[0]
        seq = [self.conv1] + list(self.convs)
        split = [self._conv_x(sc.conv) for sc in seq]     # layer i's input as hi/lo planes
        if sty is None:
            noise = self._fused_noise(noise, B, features.device, features.dtype)
            sty = self._fused_styles(latent, seq, split)
        chunk = self._fused_chunk(features, seq)
        if B > chunk:
            # the kernels index activations with 32-bit offsets (conv_launch: < 2^31 bytes
            # per tensor): larger batches run as chunks on the same noise maps and styles
            n_chunks = -(-B // chunk)
            chunk = -(-B // n_chunks)                     # balanced: 64 faces -> 2 x 32
            outs = []
            for b0 in range(0, B, chunk):
                sl = slice(b0, min(B, b0 + chunk))
                outs.append(self._fused_forward(features[sl], latent[sl],
                                                self._noise_rows(noise, sl, B),
                                                self._style_rows(sty, sl)))
            return torch.cat(outs, 0)
        mods, rgb_mods, demods = sty
        if features.dtype == torch.float16 and features.dim() == 6:
            # the renderer wrote features * mods[0] in the split layout already (ABI 12)
            if not split[0]:
                raise RuntimeError("decoder: split-NHWC features for a non-split first layer")
            x = features
        else:
            x = (modulate_to_nhwc_split if split[0] else modulate_to_nhwc)(features, mods[0])
        rgb = None
        for i, sc in enumerate(seq):
            mc = sc.conv
            last = i == len(seq) - 1
            cout = mc.weight.shape[1]
            if split[i]:
                packed, su, wsq, eps = self._pack(i, mc)
                demod_su = demods[i] if mc.demodulate else 1.0 / su.expand(B, -1)
            if (self.fuse_conv_act and split[i] and not mc.upsample and (last or split[i + 1])
                    and (x.shape[1] * x.shape[2]) % 256 == 0):
                # regular conv with the epilogue fused: the conv output stays on chip
                H, W = x.shape[1], x.shape[2]
                n = noise[i]
                rgb_base = rgb_s = None
                if i % 2 == 0:
                    # ToRGB's modulated weight base[o, c] * s[b, c] is formed inside the
                    # conv's epilogue (the same fp32 products as the module path's
                    # weight * style, without a [B, 3, C] multiply launch)
                    to_rgb = self.to_rgb1 if i == 0 else self.to_rgbs[i // 2 - 1]
                    tc = to_rgb.conv
                    rgb_base, rgb_s = self._rgb_base(tc), rgb_mods[i // 2]
                # (events run out: later convolutions go unrecorded, not an IndexError)
                ev = self.conv_events if (self.conv_events is not None
                                          and self._conv_ev < len(self.conv_events)) else None
                if ev is not None:
                    ev[self._conv_ev][0].record()
                x, part = conv3x3_f16x3_act(
                    x, packed, cout, demod=demod_su, bias=sc.activate.bias,
                    noise_weight=sc.noise.weight, noise=n,
                    s_next=None if last else mods[i + 1], store_y=not last, rgb_base=rgb_base,
                    rgb_s=rgb_s)
                if ev is not None:
                    ev[self._conv_ev][1].record()
                    self._conv_ev += 1
                    self.conv_flops += 2 * B * H * W * 9 * mc.weight.shape[2] * cout
                if part is not None:
                    rgb = rgb_finish(part, to_rgb.bias, skip=rgb if i else None, fir=self._fir)
                continue
            if (self.fuse_conv_t_blur and split[i] and mc.upsample and not last
                    and split[i + 1] and i % 2 == 1 and conv_t_act_supported(x, cout)):
                # upsampling conv with its blur and styled epilogue in the conv kernel
                # (sdfr_conv_t_act: the same bits as the two launches below)
                x = conv_t_act(x, packed, cout, fir=self._fir, demod=demod_su,
                               bias=sc.activate.bias, noise_weight=sc.noise.weight,
                               noise=noise[i], s_next=mods[i + 1])
                continue
            if split[i]:
                out = conv3x3_f16x3(x, packed, cout, transposed=mc.upsample)
                demod = demod_su              # result carries su (power of two): exact
            else:
                w = mc.scale * mc.weight[0]
                demod = (torch.rsqrt((mods[i] * mods[i]) @ (w * w).sum([2, 3]).t() + 1e-8)
                         if mc.demodulate else None)
                if mc.upsample:
                    out = F.conv_transpose2d(x, w.transpose(0, 1).contiguous(memory_format=cl),
                                             stride=2)
                else:
                    out = F.conv2d(x, w.contiguous(memory_format=cl), padding=mc.padding)
            if mc.upsample:
                H, W = out.shape[2] - 1, out.shape[3] - 1
            else:
                H, W = out.shape[2], out.shape[3]
            n = noise[i]
            rgb_w = rgb_b = None
            if i % 2 == 0:
                to_rgb = self.to_rgb1 if i == 0 else self.to_rgbs[i // 2 - 1]
                tc = to_rgb.conv
                s_rgb = rgb_mods[i // 2]
                rgb_w = self._rgb_base(tc)[None] * s_rgb[:, None, :]
                rgb_b = to_rgb.bias
            x, rgb_new = styled_epilogue(
                out, fir=self._fir, bias=sc.activate.bias, noise_weight=sc.noise.weight,
                noise=n, demod=demod, blur_up=mc.upsample,
                s_next=None if last else mods[i + 1], store_y=not last,
                rgb_w=rgb_w, rgb_b=rgb_b, skip=rgb if i else None,
                split_y=not last and split[i + 1])
            if rgb_new is not None:
                rgb = rgb_new
        return rgb


_SIDE_STREAMS = {}


def _tensors_of(x):
    """Every tensor inside nested tuples / lists / dicts (Decoder.prepare_fused's result:
    the demodulations are a dict of views of one flat buffer)."""
    if isinstance(x, torch.Tensor):
        yield x
    elif isinstance(x, dict):
        for y in x.values():
            yield from _tensors_of(y)
    elif isinstance(x, (tuple, list)):
        for y in x:
            yield from _tensors_of(y)


def _has(o, k):
    return k in o.keys() if hasattr(o, "keys") else hasattr(o, k)


class Generator(nn.Module):
    """Drop-in for sdf_model.py:1059-1216."""

    def __init__(self, model_opt, renderer_opt, blur_kernel=(1, 3, 3, 1), ema=False,
                 full_pipeline=True):
        super().__init__()
        self.size = model_opt.size
        self.style_dim = model_opt.style_dim * 2 if model_opt.psp else model_opt.style_dim
        self.num_layers = 1
        self.train_renderer = not model_opt.freeze_renderer
        self.full_pipeline = full_pipeline
        model_opt.feature_encoder_in_channels = renderer_opt.width
        self.is_train = not (ema or _has(model_opt, "is_test"))
        self.style = nn.Sequential(*[MappingLinear(self.style_dim, self.style_dim,
                                                   activation="fused_lrelu") for _ in range(3)])
        self.renderer = VolumeFeatureRenderer(renderer_opt, style_dim=self.style_dim,
                                              out_im_res=model_opt.renderer_spatial_output_dim)
        if self.full_pipeline:
            self.decoder = Decoder(model_opt, blur_kernel=blur_kernel)
        # fused inference: decoder prep (its mapping network, noise, modulations and
        # demodulations) on a side stream beside the renderer.  Round 3 measured it
        # within noise (profiles/round3_overlap_ab.json: the gather beside it slowed
        # 0.774 -> 0.801 ms); since the prep's small kernels were shortened in round 5
        # it is +0.8 % at 32 faces (3251 -> 3278 faces/s, six interleaved samples each,
        # scripts/overlap_b32.py) and neutral at one face, so it is on by default
        self.overlap_decoder_prep = True
        # the field kernel stores the decoder's first input (features x modulation,
        # split-NHWC) instead of NCHW features for modulate_nhwc_kernel to convert
        self.fuse_feature_split = True
        self.feature_split_min_batch = 4
        # repeated plain inference calls (eval.py's loop) replay a HIP graph of the
        # whole forward, captured on the second sighting of the call (graphs.py,
        # ForwardGraphCache): same results and random streams as the eager path
        self.graph_inference = True
        self._dec_key = None

    def _decoder_weights_unchanged(self):
        key = tuple((p.data_ptr(), p._version) for p in self.decoder.parameters())
        same = key == self._dec_key
        self._dec_key = key
        return same

    @staticmethod
    def _side_stream(device):
        # one per device for the process (kept off the module: a Stream does not deepcopy)
        st = _SIDE_STREAMS.get(device)
        if st is None:
            st = _SIDE_STREAMS[device] = torch.cuda.Stream(device=device)
        return st

    def mean_latent(self, n_latent, device, z=None):
        if z is None:
            z = torch.randn(n_latent, self.style_dim, device=device)
        renderer_latent = self.style(z)
        renderer_latent_mean = renderer_latent.mean(0, keepdim=True)
        decoder_latent_mean = (self.decoder.mean_latent(renderer_latent)
                               if self.full_pipeline else None)
        return [renderer_latent_mean, decoder_latent_mean]

    def get_latent(self, input):
        return self.style(input)

    def styles_and_noise_forward(self, styles, inject_index=None, truncation=1,
                                 truncation_latent=None, input_is_latent=False):
        if not input_is_latent:
            styles = [mapping_forward(self.style, s) for s in styles]
        if truncation < 1:
            styles = [truncation_latent[0] + truncation * (s - truncation_latent[0])
                      for s in styles]
        return styles

    def init_forward(self, styles, cam_poses, focals, near=0.88, far=1.12, t_rand=None):
        latent = self.styles_and_noise_forward(styles)
        return self.renderer.mlp_init_pass(cam_poses, focals, near, far, styles=latent[0],
                                           t_rand=t_rand)

    def forward(self, styles, cam_poses, focals, near=0.88, far=1.12, return_latents=False,
                inject_index=None, truncation=1, truncation_latent=None, input_is_latent=False,
                noise=None, randomize_noise=True, return_sdf=False, return_xyz=False,
                return_eikonal=False, project_noise=False, mesh_path=None, t_rand=None):
        kw = dict(return_latents=return_latents, inject_index=inject_index,
                  truncation=truncation, truncation_latent=truncation_latent,
                  input_is_latent=input_is_latent, noise=noise, randomize_noise=randomize_noise,
                  return_sdf=return_sdf, return_xyz=return_xyz, return_eikonal=return_eikonal,
                  project_noise=project_noise, mesh_path=mesh_path, t_rand=t_rand)
        if self.graph_inference and not self.training and not torch.is_grad_enabled():
            from .graphs import forward_cache
            cache = forward_cache(self)
            if cache.eligible(self, styles, cam_poses, focals, near, far, kw):
                out = cache(self, styles, cam_poses, focals, near, far, kw)
                if out is not None:
                    return out
        return self._forward_eager(styles, cam_poses, focals, near, far, **kw)

    def _forward_eager(self, styles, cam_poses, focals, near=0.88, far=1.12,
                       return_latents=False, inject_index=None, truncation=1,
                       truncation_latent=None, input_is_latent=False, noise=None,
                       randomize_noise=True, return_sdf=False, return_xyz=False,
                       return_eikonal=False, project_noise=False, mesh_path=None, t_rand=None):
        grad_on = self.is_train and self.train_renderer
        # Fused inference: the decoder's feature-independent prep (its mapping network,
        # noise maps, per-layer modulations / demodulations: ~12 small launches) runs
        # before the renderer -- on a side stream beside it while the decoder's weight
        # caches are warm (weights unchanged since the previous call), else in order
        # on this stream, so the caches a weight update rebuilds, and the ones it
        # frees, never cross streams.  On the side stream the renderer's own mapping
        # network goes there too: the renderer enqueues its sample geometry and hash-grid
        # gather (which do not read the styles) ahead of its wait on `styles_ev` (ABI 11).
        # Either way the device RNG is drawn in the same order (decoder noise, then the
        # renderer's sampling offsets).
        prepared, side, styles_ev = None, None, None
        B, dev = cam_poses.shape[0], cam_poses.device
        kw = dict(noise=noise, inject_index=inject_index, truncation=truncation,
                  truncation_latent=truncation_latent, input_is_latent=input_is_latent,
                  randomize_noise=randomize_noise)
        # features needing grad (renderer trained, or latents requiring grad) take the
        # decoder's autograd path: no prep then (Decoder.forward re-checks as well)
        pre_grad = grad_on and (
            any(p.requires_grad for p in self.renderer.parameters())
            or any(p.requires_grad for p in self.style.parameters())
            or any(s.requires_grad for s in styles))
        capturing = cam_poses.is_cuda and torch.cuda.is_current_stream_capturing()
        # (a small eager batch is host-bound: the stream switch would cost more than
        # the overlap saves; inside a graph capture it costs nothing at replay)
        if (self.full_pipeline and cam_poses.is_cuda and not project_noise and not pre_grad
                and self.overlap_decoder_prep and (B >= 8 or capturing)
                and self.decoder.fused_ready(dev) and self._decoder_weights_unchanged()):
            main = torch.cuda.current_stream(dev)
            side = self._side_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                with torch.set_grad_enabled(grad_on):
                    latent = self.styles_and_noise_forward(styles, inject_index, truncation,
                                                           truncation_latent, input_is_latent)
                prepared = self.decoder.prepare_fused(latent, B, dev, **kw)
                # (after the prep: the field kernel also reads its first modulation)
                styles_ev = torch.cuda.Event()
                styles_ev.record(side)
            if not capturing:
                for t in list(_tensors_of(prepared)) + list(_tensors_of(latent)):
                    t.record_stream(main)            # made on `side`, used on `main`
        else:
            with torch.set_grad_enabled(grad_on):
                latent = self.styles_and_noise_forward(styles, inject_index, truncation,
                                                       truncation_latent, input_is_latent)
            render_grad = grad_on and (
                any(p.requires_grad for p in self.renderer.parameters())
                or any(s.requires_grad for s in latent))
            if (self.full_pipeline and cam_poses.is_cuda and not project_noise and not render_grad
                    and self.decoder.fused_ready(dev)):
                prepared = self.decoder.prepare_fused(latent, B, dev, **kw)
        # the fused decoder's first layer input (features x its modulation, split-NHWC)
        # straight from the field kernel's feature store (ABI 12): one streaming pass less
        # (from 4 faces: below that the field kernel splits rays into segments and the
        # merge kernel would scatter 2-B split stores instead of coalesced NCHW rows)
        feat_mod = None
        if (prepared is not None and self.fuse_feature_split
                and B >= self.feature_split_min_batch
                and self.decoder._conv_x(self.decoder.conv1.conv)):
            feat_mod = prepared[2][0][0]
        with torch.set_grad_enabled(grad_on):
            lat0 = latent[0][:, 0] if input_is_latent else latent[0]
            thumb_rgb, features, sdf, mask, xyz, eikonal_term = self.renderer(
                cam_poses, focals, near, far, styles=lat0, return_eikonal=return_eikonal,
                t_rand=t_rand, styles_event=styles_ev, feat_mod=feat_mod)
        if self.full_pipeline:
            # (the side stream's work ends at styles_ev, which the renderer made this
            # stream wait on before its FiLM prep -- every render entry does, ABI 11 --
            # so the decoder needs no second join: one right here would sit behind the
            # field kernel as a barrier packet, ~10 us of idle GPU per call)
            rgb, decoder_latent = self.decoder(
                features, latent, transform=cam_poses if project_noise else None,
                return_latents=return_latents, inject_index=inject_index, truncation=truncation,
                truncation_latent=truncation_latent, noise=noise,
                input_is_latent=input_is_latent, randomize_noise=randomize_noise,
                mesh_path=mesh_path, prepared=prepared)
        else:
            rgb = None
        if return_latents:
            return rgb, decoder_latent
        out = (rgb, thumb_rgb)
        if return_xyz:
            out += (xyz,)
        if return_sdf:
            out += (sdf,)
        if return_eikonal:
            out += (eikonal_term,)
        if return_xyz:
            out += (mask,)
        return out
