"""Stage-2 ("full pipeline") GAN training, data-parallel over RCCL / xGMI.

Mirrors training_utils.train_full_pipeline (training_utils.py:552-881) with the
pieces it calls: the StyleGAN2 Discriminator (sdf_model.py:1401-1510), the
losses (sdf_losses.py:27-65) and the sampling / EMA helpers (sdf_utils.py:64-93).

One process per GPU.  The renderer is frozen in stage 2 (freeze_renderer; the
Generator runs it under no_grad, sdf_model.py:1174), so it takes the fused HIP
forward path and its parameters -- and the renderer mapping network's -- never
get gradients: they are excluded from DDP, which then bucket-all-reduces only the
decoder's 23 MB and the discriminator's 115 MB of fp32 gradients.
Gradient accumulation over the reference's chunks runs under no_sync() so each
optimizer step all-reduces once.  The reference never wraps its models in DDP
(SURVEY.md §0.4); this module is the data-parallel form of the same step.
"""
from __future__ import annotations

import math
import random
from contextlib import nullcontext

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import autograd, nn
from torch.profiler import record_function

from .camera import generate_camera_params
from .decoder_ops import FusedLeakyReLU
from .generator import Blur, EqualLinear, Generator, StyledConv


# ---------------------------------------------------------------------------
# discriminator (sdf_model.py:541-578, 846-881, 1401-1510)
# ---------------------------------------------------------------------------
class EqualConv2d(nn.Module):
    def __init__(self, in_channel, out_channel, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(out_channel, in_channel, kernel_size, kernel_size))
        self.scale = 1 / math.sqrt(in_channel * kernel_size ** 2)
        self.stride = stride
        self.padding = padding
        self.bias = nn.Parameter(torch.zeros(out_channel)) if bias else None

    def forward(self, input):
        return F.conv2d(input, self.weight * self.scale, bias=self.bias, stride=self.stride,
                        padding=self.padding)


class ConvLayer(nn.Sequential):
    def __init__(self, in_channel, out_channel, kernel_size, downsample=False,
                 blur_kernel=(1, 3, 3, 1), bias=True, activate=True):
        layers = []
        if downsample:
            p = (len(blur_kernel) - 2) + (kernel_size - 1)
            layers.append(Blur(blur_kernel, pad=((p + 1) // 2, p // 2)))
            stride, padding = 2, 0
        else:
            stride, padding = 1, kernel_size // 2
        layers.append(EqualConv2d(in_channel, out_channel, kernel_size, padding=padding,
                                  stride=stride, bias=bias and not activate))
        if activate:
            layers.append(FusedLeakyReLU(out_channel, bias=bias))
        super().__init__(*layers)


class ResBlock(nn.Module):
    def __init__(self, in_channel, out_channel, blur_kernel=(1, 3, 3, 1), merge=False):
        super().__init__()
        cin = 2 * in_channel if merge else in_channel
        self.conv1 = ConvLayer(cin, in_channel, 3)
        self.conv2 = ConvLayer(in_channel, out_channel, 3, downsample=True)
        self.skip = ConvLayer(cin, out_channel, 1, downsample=True, activate=False, bias=False)

    def forward(self, input):
        out = self.conv2(self.conv1(input))
        return (out + self.skip(input)) / math.sqrt(2)


class Discriminator(nn.Module):
    """StyleGAN2 residual discriminator on size^2 RGB (sdf_model.py:1418)."""

    def __init__(self, opt, blur_kernel=(1, 3, 3, 1)):
        super().__init__()
        cm = opt.channel_multiplier
        channels = {4: 512, 8: 512, 16: 512, 32: 512, 64: 256 * cm, 128: 128 * cm,
                    256: 64 * cm, 512: 32 * cm, 1024: 16 * cm}
        size = opt.size
        convs = [ConvLayer(3, channels[size], 1)]
        in_channel = channels[size]
        for i in range(int(math.log(size, 2)), 2, -1):
            out_channel = channels[2 ** (i - 1)]
            convs.append(ResBlock(in_channel, out_channel, blur_kernel))
            in_channel = out_channel
        self.convs = nn.Sequential(*convs)
        self.stddev_group = 4
        self.stddev_feat = 1
        self.final_conv = ConvLayer(in_channel + 1, channels[4], 3)
        self.final_linear = nn.Sequential(
            EqualLinear(channels[4] * 4 * 4, channels[4], activation="fused_lrelu"),
            EqualLinear(channels[4], 1))

    def get_feat(self, input):
        out = self.convs(input)
        batch, channel, height, width = out.shape
        group = min(batch, self.stddev_group)
        if batch % group != 0:
            group = 3 if batch % 3 == 0 else 2
        stddev = out.view(group, -1, self.stddev_feat, channel // self.stddev_feat, height, width)
        stddev = torch.sqrt(stddev.var(0, unbiased=False) + 1e-8)
        stddev = stddev.mean([2, 3, 4], keepdims=True).squeeze(2)
        stddev = stddev.repeat(group, 1, height, width)
        out = self.final_conv(torch.cat([out, stddev], 1))
        return out.view(batch, -1)

    def forward(self, input):
        return self.final_linear(self.get_feat(input))[:, :1]


# ---------------------------------------------------------------------------
# losses (sdf_losses.py:27-65)
# ---------------------------------------------------------------------------
def d_logistic_loss(real_pred, fake_pred):
    return F.softplus(-real_pred).mean() + F.softplus(fake_pred).mean()


def d_r1_loss(real_pred, real_img):
    grad_real, = autograd.grad(outputs=real_pred.sum(), inputs=real_img, create_graph=True)
    return grad_real.pow(2).reshape(grad_real.shape[0], -1).sum(1).mean()


def g_nonsaturating_loss(fake_pred):
    return F.softplus(-fake_pred).mean()


def g_content_loss(fake_img, fake_img_up):
    return F.l1_loss(fake_img_up, fake_img)


def g_path_regularize(fake_img, latents, mean_path_length, decay=0.01):
    noise = torch.randn_like(fake_img) / math.sqrt(fake_img.shape[2] * fake_img.shape[3])
    grad, = autograd.grad(outputs=(fake_img * noise).sum(), inputs=latents, create_graph=True,
                          only_inputs=True)
    path_lengths = torch.sqrt(grad.pow(2).sum(2).mean(1))
    path_mean = mean_path_length + decay * (path_lengths.mean() - mean_path_length)
    path_penalty = (path_lengths - path_mean).pow(2).mean()
    return path_penalty, path_mean.detach(), path_lengths


# ---------------------------------------------------------------------------
# helpers (sdf_utils.py:64-93, distributed.py)
# ---------------------------------------------------------------------------
def requires_grad(params, flag=True):
    for p in params:
        p.requires_grad = flag


@torch.no_grad()
def accumulate(model1, model2, decay=0.999):
    """EMA of model2's parameters into model1 (sdf_utils.py:64-69).  The update runs
    on the parameters themselves (not ``.data``), so it bumps their version
    counters: the fused decoder's packed-weight caches and GraphedGenerator key on
    (data_ptr, version) and must see every EMA step.  Two foreach launches per
    device / dtype instead of two per parameter: the same mul-then-add per element
    (test_gpu_train.py::test_accumulate_foreach_bit_identical pins it against the
    per-parameter loop)."""
    par2 = dict(model2.named_parameters())
    p1, p2 = [], []
    for k, p in model1.named_parameters():
        p1.append(p)
        p2.append(par2[k].detach())
    if not p1:
        return
    torch._foreach_mul_(p1, decay)
    torch._foreach_add_(p1, p2, alpha=1 - decay)


@torch.no_grad()
def accumulate_loop(model1, model2, decay=0.999):
    """The per-parameter form of ``accumulate`` (sdf_utils.py:64-69 verbatim in
    operations): the pin for the foreach one."""
    par1 = dict(model1.named_parameters())
    par2 = dict(model2.named_parameters())
    for k in par1.keys():
        par1[k].mul_(decay).add_(par2[k].detach(), alpha=1 - decay)


def make_noise(batch, latent_dim, n_noise, device):
    if n_noise == 1:
        return torch.randn(batch, latent_dim, device=device)
    return torch.randn(n_noise, batch, latent_dim, device=device).unbind(0)


def mixing_noise(batch, latent_dim, prob, device):
    if prob > 0 and random.random() < prob:
        return make_noise(batch, latent_dim, 2, device)
    return [make_noise(batch, latent_dim, 1, device)]


def _dist_on():
    """A process group exists: the collectives and DDP run (at any world size, so a
    world-1 RCCL group exercises the same calls as eight ranks)."""
    return dist.is_available() and dist.is_initialized()


def _world():
    return dist.get_world_size() if _dist_on() else 1


def reduce_loss_dict(loss_dict):
    """Mean over ranks of every scalar loss (one all-reduce of a packed vector)."""
    keys = sorted(loss_dict)
    if not keys:
        return {}
    vals = torch.stack([loss_dict[k].detach().float().reshape(()) for k in keys])
    if _dist_on():
        dist.all_reduce(vals)
        vals /= _world()
    return dict(zip(keys, vals))


def allreduce_grads(params):
    """Mean of the gradients over ranks as ONE flat all-reduce: for a backward
    that bypasses the DDP wrapper (the stage-1 sphere init calls
    ``g_module.init_forward``, training_utils.py:309, so under DDP the
    reference's replicas drift apart there)."""
    world = _world()
    grads = [p.grad for p in params if p.grad is not None]
    if not _dist_on() or not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    flat /= world
    off = 0
    for g in grads:
        g.copy_(flat[off:off + g.numel()].view_as(g))
        off += g.numel()


# ---------------------------------------------------------------------------
# the data-parallel stage-2 trainer
# ---------------------------------------------------------------------------
class FullPipelineTrainer:
    """Generator + EMA copy + Discriminator + optimizers of stage 2, each rank
    holding full replicas; ``step(real_imgs)`` is one iteration of the reference
    loop (D step with R1 every d_reg_every, G step, path regularisation every
    g_reg_every, EMA).

    The renderer is frozen here, as in the reference (training_utils.py:176).  A
    variant that trains it in stage 2 AND keeps path regularisation would
    differentiate the renderer's HIP training GEMMs twice (autograd.grad with
    create_graph through the ngp FiLM layers): their once-differentiable backward
    raises then (linear.py ``_once``) rather than dropping that term -- such a run
    needs the layers built with ``twice=True``, as the SIREN eikonal path uses."""

    def __init__(self, opt, device, seed=0):
        self.opt, self.t, self.device = opt, opt.training, device
        self.world = _world()
        self.dist = _dist_on()
        torch.manual_seed(seed)                   # identical initial replicas on every rank
        random.seed(seed)
        self.generator = Generator(opt.model, opt.rendering).to(device)
        self.generator_test = Generator(opt.model, opt.rendering, ema=True).to(device).eval()
        self.discriminator = Discriminator(opt.model).to(device)
        # trained in stage 2: the decoder, minus StyledConv.bias, which the reference
        # declares but never uses (sdf_model.py:810; FusedLeakyReLU has its own bias)
        unused = {id(m.bias) for m in self.generator.modules() if isinstance(m, StyledConv)}
        self.g_train = [p for n, p in self.generator.named_parameters()
                        if n.startswith("decoder.") and id(p) not in unused]
        train_ids = {id(p) for p in self.g_train}
        frozen = [p for p in self.generator.parameters() if id(p) not in train_ids]
        requires_grad(frozen, False)              # renderer + mapping: no grads in stage 2
        t = self.t
        g_ratio = t.g_reg_every / (t.g_reg_every + 1) if t.g_reg_every > 0 else 1
        d_ratio = t.d_reg_every / (t.d_reg_every + 1)
        # The reference builds one param group per decoder parameter, every one at the
        # same lr and betas (config.py:206-215).  Adam is elementwise, so a single group
        # gives the same update bit for bit (test_train_step.py::test_g_adam_one_group_
        # equals_per_parameter_groups) with ~6 foreach launches per step instead of ~6
        # per parameter.  checkpoint.load_into folds a per-group state into it.
        self.optimizer = torch.optim.Adam(self.g_train, lr=t.lr * g_ratio,
                                          betas=(0 ** g_ratio, 0.99 ** g_ratio))
        self.optimizer_d = torch.optim.Adam(self.discriminator.parameters(), lr=t.lr * d_ratio,
                                            betas=(0 ** d_ratio, 0.99 ** d_ratio))
        accumulate(self.generator_test, self.generator, 0)
        self.g_module, self.d_module = self.generator, self.discriminator
        if self.dist:
            from torch.nn.parallel import DistributedDataParallel as DDP
            kw = dict(broadcast_buffers=False)
            if device.type == "cuda":
                kw.update(device_ids=[device.index], output_device=device.index)
            self.generator = DDP(self.generator, **kw)
            self.discriminator = DDP(self.discriminator, **kw)
        self.mean_path_length = 0.0
        self.accum = 0.5 ** (32 / (10 * 1000))
        self.iteration = 0
        # decoder noise drawn per forward as the reference (True), or the decoder's
        # fixed noise buffers (False: reproducible gradients, tests)
        self.randomize_noise = True

    def _cams(self, n):
        c = self.opt.camera
        return generate_camera_params(self.t.renderer_output_size, self.device, batch=n,
                                      uniform=c.uniform, azim_range=c.azim, elev_range=c.elev,
                                      fov_ang=c.fov, dist_radius=c.dist_radius)

    @staticmethod
    def _sync(model, last):
        """no_sync() for every chunk but the last: one all-reduce per optimizer step."""
        return nullcontext() if last or not hasattr(model, "no_sync") else model.no_sync()

    def d_backward(self, noise, cams, real_imgs, d_regularize):
        """The discriminator half-step's gradients (training_utils.py:661-712): over
        the batch in chunks, the fake images from the frozen-path generator, the
        logistic loss and (every d_reg_every) R1, accumulated locally and
        all-reduced once, on the last chunk.  Returns the last chunk's terms."""
        t = self.t
        batch, chunk = real_imgs.shape[0], t.chunk
        cam, focal, near, far = cams[:4]
        requires_grad(self.g_train, False)
        requires_grad(self.d_module.parameters(), True)
        self.d_module.zero_grad(set_to_none=True)
        r1_loss = torch.zeros((), device=real_imgs.device)
        for j in range(0, batch, chunk):
            last = j + chunk >= batch
            with self._sync(self.discriminator, last):
                with torch.no_grad():
                    gen_imgs, _ = self.g_module([n[j:j + chunk] for n in noise], cam[j:j + chunk],
                                                focal[j:j + chunk], near[j:j + chunk],
                                                far[j:j + chunk],
                                                randomize_noise=self.randomize_noise)
                real = real_imgs[j:j + chunk].detach().requires_grad_(d_regularize)
                fake_pred = self.discriminator(gen_imgs)
                real_pred = self.discriminator(real)
                d_gan_loss = d_logistic_loss(real_pred, fake_pred)
                if d_regularize:
                    r1_loss = t.r1 * 0.5 * d_r1_loss(real_pred, real) * t.d_reg_every
                else:
                    r1_loss = torch.zeros_like(r1_loss)
                (d_gan_loss + r1_loss).backward()
        return d_gan_loss, r1_loss, real_pred, fake_pred

    def g_backward(self, chunk_inputs, n_chunks):
        """The generator half-step's gradients (training_utils.py:717-742): per chunk
        (noise, cameras) from ``chunk_inputs`` -- drawn lazily by step() so the RNG
        order is the reference's -- the non-saturating loss plus 0.001 x L1 to the
        4x nearest-upsampled thumbnail; one all-reduce on the last chunk."""
        requires_grad(self.g_train, True)
        requires_grad(self.d_module.parameters(), False)
        for k, (noise, cams) in enumerate(chunk_inputs):
            cam, focal, near, far = cams[:4]
            with self._sync(self.generator, k == n_chunks - 1):
                fake_img, fake_thumb = self.generator(noise, cam, focal, near, far,
                                                      randomize_noise=self.randomize_noise)
                fake_up = F.interpolate(fake_thumb, scale_factor=4)   # nn.Upsample(4), nearest
                g_gan_loss = g_nonsaturating_loss(self.d_module(fake_img))
                (g_gan_loss + 0.001 * g_content_loss(fake_img, fake_up)).backward()
        return g_gan_loss

    def _path_step(self, style_dim, batch, chunk):
        """Path length regularisation (training_utils.py:744-776).  As the reference,
        every pass of the chunk loop runs the WHOLE path batch (its loop index is
        unused, :760-763): path_batch / chunk passes on the same latents and cameras
        (fresh decoder noise each), gradients and the path-length EMA accumulated
        over them."""
        t, dev = self.t, self.device
        pbs = max(1, batch // t.path_batch_shrink)
        noise = mixing_noise(pbs, style_dim, t.mixing, dev)
        cam, focal, near, far, _ = self._cams(pbs)
        for j in range(0, pbs, chunk):
            last = j + chunk >= pbs
            with self._sync(self.generator, last):
                img, latents = self.generator(noise, cam, focal, near, far,
                                              return_latents=True,
                                              randomize_noise=self.randomize_noise)
                path_loss, self.mean_path_length, path_lengths = g_path_regularize(
                    img, latents, self.mean_path_length)
                w = t.path_regularize * t.g_reg_every * path_loss
                if t.path_batch_shrink:
                    w = w + 0 * img[0, 0, 0, 0]
                w.backward()
        self.optimizer.step()
        self.g_module.zero_grad(set_to_none=True)
        if self.dist:
            mpl = torch.as_tensor(self.mean_path_length, device=dev, dtype=torch.float32)
            dist.all_reduce(mpl)
            self.mean_path_length = mpl / self.world
        return path_loss, path_lengths

    def step(self, real_imgs):
        t, dev = self.t, self.device
        i = self.iteration
        style_dim = self.opt.model.style_dim
        batch, chunk = real_imgs.shape[0], t.chunk
        loss = {}

        # --- discriminator (training_utils.py:652-716)
        d_regularize = i % t.d_reg_every == 0
        with record_function("stage2.d_step"):
            noise = mixing_noise(batch, style_dim, t.mixing, dev)
            cams = self._cams(batch)
            d_gan_loss, r1_loss, real_pred, fake_pred = self.d_backward(noise, cams, real_imgs,
                                                                        d_regularize)
            self.optimizer_d.step()
        loss.update(d=d_gan_loss, real_score=real_pred.mean(), fake_score=fake_pred.mean(),
                    r1=r1_loss.mean())

        # --- generator (training_utils.py:717-742)
        n_chunks = len(range(0, batch, chunk))
        inputs = ((mixing_noise(chunk, style_dim, t.mixing, dev), self._cams(chunk))
                  for _ in range(n_chunks))
        with record_function("stage2.g_step"):
            g_gan_loss = self.g_backward(inputs, n_chunks)
            self.optimizer.step()
            self.g_module.zero_grad(set_to_none=True)
        loss["g"] = g_gan_loss

        # --- path length regularisation (training_utils.py:744-776)
        path_loss = torch.zeros((), device=dev)
        path_lengths = torch.zeros((), device=dev)
        if t.g_reg_every > 0 and i % t.g_reg_every == 0:
            with record_function("stage2.path_reg"):
                path_loss, path_lengths = self._path_step(style_dim, batch, chunk)
        loss.update(path=path_loss, path_length=path_lengths.mean())

        accumulate(self.generator_test, self.g_module, self.accum)
        self.iteration += 1
        return reduce_loss_dict(loss)

    def state_dict(self):
        """{g, d, g_ema} as the reference's checkpoints (training_utils.py:857-880)."""
        return {"g": self.g_module.state_dict(), "d": self.d_module.state_dict(),
                "g_ema": self.generator_test.state_dict()}


# ---------------------------------------------------------------------------
# stage 1: the volume renderer on its own (training_utils.py:197-551)
# ---------------------------------------------------------------------------
class VolumeRenderDiscConv2d(nn.Module):
    """sdf_model.py:1224-1249."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True,
                 activate=False):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding,
                              bias=bias and not activate)
        self.activate = activate
        if self.activate:
            self.activation = FusedLeakyReLU(out_channels, bias=bias, scale=1)
            coef = math.sqrt(1 / (in_channels * kernel_size * kernel_size))
            nn.init.uniform_(self.activation.bias, a=-coef, b=coef)

    def forward(self, input):
        out = self.conv(input)
        return self.activation(out) if self.activate else out


_COORD_PLANES = {}


def coord_planes(dim_y, dim_x, device, pad=0):
    """[1, 2 + pad, dim_y, dim_x]: the y and x coordinate planes exactly as
    sdf_model.py:1252-1275 computes them (arange / (n - 1) * 2 - 1 in fp32), then
    ``pad`` zero planes.  Built once per (size, device, pad): the discriminator runs
    ten CoordConv layers per forward and a dozen forwards per training step, and
    rebuilding the planes cost ~12 small launches each time."""
    key = (dim_y, dim_x, str(device), pad)
    t = _COORD_PLANES.get(key)
    if t is None:
        with torch.inference_mode(False), torch.no_grad():
            xx = torch.arange(dim_x, dtype=torch.float32, device=device).repeat(1, 1, dim_y, 1)
            yy = torch.arange(dim_y, dtype=torch.float32, device=device).repeat(1, 1, dim_x, 1)
            yy = yy.transpose(2, 3)
            xx = (xx / (dim_x - 1)) * 2 - 1
            yy = (yy / (dim_y - 1)) * 2 - 1
            z = torch.zeros(1, pad, dim_y, dim_x, dtype=torch.float32, device=device)
            t = torch.cat([yy, xx, z], dim=1).contiguous()
        _COORD_PLANES[key] = t
    return t


class AddCoords(nn.Module):
    """sdf_model.py:1252-1275: append the y, x pixel coordinates in [-1, 1]."""

    def forward(self, input_tensor, pad=0):
        b, _, dim_y, dim_x = input_tensor.shape
        planes = coord_planes(dim_y, dim_x, input_tensor.device, pad)
        return torch.cat([input_tensor, planes.expand(b, -1, -1, -1)], dim=1)


class CoordConv2d(nn.Module):
    """sdf_model.py:1278-1296.

    On the GPU the convolution's input channels (C + 2 coordinate channels: 130, 258,
    402 in the stage-1 discriminator) are zero-padded to a multiple of ``pad_to``,
    input and weight alike: the extra channels contribute exact zeros, the
    parameters and state-dict keys are unchanged, and MIOpen can pick its
    implicit-GEMM / Winograd solvers instead of the naive fallback it uses for
    channel counts that are not a multiple of 4 (``pad_to = 1`` turns it off)."""

    pad_to = 8

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        self.addcoords = AddCoords()
        self.conv = nn.Conv2d(in_channels + 2, out_channels, kernel_size, stride=stride,
                              padding=padding, bias=bias)

    def forward(self, input_tensor):
        pad = -(input_tensor.shape[1] + 2) % self.pad_to
        if not input_tensor.is_cuda or pad == 0:
            return self.conv(self.addcoords(input_tensor))
        # coordinates and zero channels appended by one concatenation
        x = self.addcoords(input_tensor, pad)
        w = F.pad(self.conv.weight, (0, 0, 0, 0, 0, pad))
        return F.conv2d(x, w, self.conv.bias, self.conv.stride, self.conv.padding)


class CoordConvLayer(nn.Module):
    """sdf_model.py:1299-1322."""

    def __init__(self, in_channel, out_channel, kernel_size, bias=True, activate=True):
        super().__init__()
        self.activate = activate
        self.padding = kernel_size // 2 if kernel_size > 2 else 0
        self.conv = CoordConv2d(in_channel, out_channel, kernel_size, padding=self.padding,
                                stride=1, bias=bias and not activate)
        if activate:
            self.activation = FusedLeakyReLU(out_channel, bias=bias, scale=1)
        coef = math.sqrt(1 / (in_channel * kernel_size * kernel_size))
        nn.init.uniform_(self.activation.bias, a=-coef, b=coef)

    def forward(self, input):
        out = self.conv(input)
        return self.activation(out) if self.activate else out


class VolumeRenderResBlock(nn.Module):
    """sdf_model.py:1325-1351."""

    def __init__(self, in_channel, out_channel):
        super().__init__()
        self.conv1 = CoordConvLayer(in_channel, out_channel, 3)
        self.conv2 = CoordConvLayer(out_channel, out_channel, 3)
        self.pooling = nn.AvgPool2d(2)
        self.downsample = nn.AvgPool2d(2)
        self.skip = (VolumeRenderDiscConv2d(in_channel, out_channel, 1)
                     if out_channel != in_channel else None)

    def forward(self, input):
        out = self.pooling(self.conv2(self.conv1(input)))
        skip_in = self.downsample(input)
        if self.skip is not None:
            skip_in = self.skip(skip_in)
        return (out + skip_in) / math.sqrt(2)


class VolumeRenderDiscriminator(nn.Module):
    """sdf_model.py:1354-1398: judges the renderer's 64^2 thumbnails, with a
    viewpoint (azimuth, elevation) regression head unless no_viewpoint_loss."""

    def __init__(self, opt):
        super().__init__()
        init_size = opt.renderer_spatial_output_dim
        self.viewpoint_loss = not opt.no_viewpoint_loss
        final_out_channel = 3 if self.viewpoint_loss else 1
        channels = {2: 400, 4: 400, 8: 400, 16: 400, 32: 256, 64: 128, 128: 64}
        convs = [VolumeRenderDiscConv2d(3, channels[init_size], 1, activate=True)]
        log_size = int(math.log(init_size, 2))
        in_channel = channels[init_size]
        for i in range(log_size - 1, 0, -1):
            out_channel = channels[2 ** i]
            convs.append(VolumeRenderResBlock(in_channel, out_channel))
            in_channel = out_channel
        self.convs = nn.Sequential(*convs)
        self.final_conv = VolumeRenderDiscConv2d(in_channel, final_out_channel, 2)

    def forward(self, input):
        out = self.final_conv(self.convs(input))
        gan_preds = out[:, 0:1].view(-1, 1)
        viewpoints_preds = out[:, 1:].view(-1, 2) if self.viewpoint_loss else None
        return gan_preds, viewpoints_preds


def viewpoints_loss(viewpoint_pred, viewpoint_target):
    """sdf_losses.py:7-10."""
    return F.smooth_l1_loss(viewpoint_pred, viewpoint_target)


def eikonal_loss(eikonal_term, sdf=None, beta=100):
    """sdf_losses.py:13-24: (|grad sdf| - 1)^2 and the minimal-surface term."""
    eik = 0 if eikonal_term is None else ((eikonal_term.norm(dim=-1) - 1) ** 2).mean()
    if sdf is None:
        surf = torch.tensor(0.0, device=eikonal_term.device)
    else:
        surf = torch.exp(-beta * torch.abs(sdf)).mean()
    return eik, surf


def _coordinates(n, device):
    r = torch.arange(0, n, dtype=torch.long, device=device)
    x, y, z = torch.meshgrid(r, r, r, indexing="ij")
    return torch.stack([x, y, z], dim=-1)


def smoothness(generator, bounding_box, styles, device, sample_points=32, voxel_size=0.1,
               margin=0.05):
    """smoothLoss.py:5-27: total variation of the hash-grid features over a random
    32^3 voxel block inside the bounding box ([3, 2] min / max per axis)."""
    offset_max = bounding_box[:, 1] - bounding_box[:, 0] - (sample_points - 1) * voxel_size \
        - 2 * margin
    offset = torch.rand(3).to(offset_max) * offset_max + margin
    coords = _coordinates(sample_points - 1, "cpu").float().to(bounding_box)
    pts = (coords + torch.rand((1, 1, 1, 3)).to(bounding_box)) * voxel_size \
        + bounding_box[:, 0] + offset
    pts = ((pts - bounding_box[:, 0]) / (bounding_box[:, 1] - bounding_box[:, 0])).to(device)
    sdf = generator.renderer.network.query_sdf(pts, styles)
    tv_x = torch.pow(sdf[1:, ...] - sdf[:-1, ...], 2).sum()
    tv_y = torch.pow(sdf[:, 1:, ...] - sdf[:, :-1, ...], 2).sum()
    tv_z = torch.pow(sdf[:, :, 1:, ...] - sdf[:, :, :-1, ...], 2).sum()
    return (tv_x + tv_y + tv_z) / (sample_points ** 3)


class RendererTrainer:
    """Stage 1: Generator(full_pipeline=False) + EMA copy + VolumeRenderDiscriminator
    with the reference's optimizers (config.py:196-200: Adam, G lr 2e-5, D lr 2e-4,
    betas (0, 0.9)).  The renderer trains through the op-by-op path: every
    hash-grid / SH evaluation is the HIP encoder op with its HIP backward (table
    gradients by fp32 atomics, dy_dx for the eikonal term), so it needs the GPU.
    ``sphere_init_step()`` is one iteration of the SDF-to-sphere initialisation,
    ``step(real_thumbs)`` one D + G iteration (training_utils.py:287-451)."""

    def __init__(self, opt, device, seed=0):
        self.opt, self.t, self.device = opt, opt.training, device
        self.world = _world()
        self.dist = _dist_on()
        torch.manual_seed(seed)
        random.seed(seed)
        self.generator = Generator(opt.model, opt.rendering, full_pipeline=False).to(device)
        self.generator_test = Generator(opt.model, opt.rendering, ema=True,
                                        full_pipeline=False).to(device).eval()
        self.discriminator = VolumeRenderDiscriminator(opt.model).to(device)
        accumulate(self.generator_test, self.generator, 0)
        self.optimizer = torch.optim.Adam(self.generator.parameters(), lr=2e-5, betas=(0.0, 0.9))
        self.optimizer_d = torch.optim.Adam(self.discriminator.parameters(), lr=2e-4,
                                            betas=(0.0, 0.9))
        self.g_module, self.d_module = self.generator, self.discriminator
        if self.dist:
            from torch.nn.parallel import DistributedDataParallel as DDP
            kw = dict(broadcast_buffers=False)
            if device.type == "cuda":
                kw.update(device_ids=[device.index], output_device=device.index)
            self.generator = DDP(self.generator, **kw)
            self.discriminator = DDP(self.discriminator, **kw)
        self.accum = 0.5 ** (32 / (10 * 1000))
        self.iteration = 0

    def _cams(self, n):
        c = self.opt.camera
        return generate_camera_params(self.t.renderer_output_size, self.device, batch=n,
                                      uniform=c.uniform, azim_range=c.azim, elev_range=c.elev,
                                      fov_ang=c.fov, dist_radius=c.dist_radius)

    _sync = staticmethod(FullPipelineTrainer._sync)

    # how the ranks agree on the sphere initialisation: "broadcast" -- every rank runs
    # the reference's single-GPU loop (batch 3 per step, no collective per step) and
    # sphere_init_finish() broadcasts rank 0's generator and optimizer state once;
    # "allreduce" -- the gradients of every step are averaged over the ranks (one flat
    # all-reduce of all 54.6 MB per 6.4 ms step: the hash table's gradient is the last
    # one the backward produces, so it cannot overlap it)
    sphere_init_sync = "broadcast"

    def sphere_init_step(self, batch=3):
        """MLP init to a sphere SDF (training_utils.py:287-317): L1(sdf, |x| - r)."""
        noise = mixing_noise(batch, self.t.style_dim, self.t.mixing, self.device)
        cam, focal, near, far, _ = self._cams(batch)
        sdf, target = self.g_module.init_forward(noise, cam, focal, near, far)
        loss = F.l1_loss(sdf, target)
        loss.backward()
        if self.sphere_init_sync == "allreduce":
            allreduce_grads(list(self.g_module.parameters()))
        self.optimizer.step()
        self.g_module.zero_grad(set_to_none=True)
        return loss.detach()

    def sphere_init_finish(self):
        """End of the sphere initialisation: with ``sphere_init_sync == "broadcast"`` every
        rank takes rank 0's generator parameters and Adam moments (one broadcast per
        tensor, once), so the replicas enter stage-1 training identical."""
        if not _dist_on() or self.sphere_init_sync != "broadcast":
            return
        with torch.no_grad():
            for p in self.g_module.parameters():
                dist.broadcast(p.data, 0)
                st = self.optimizer.state.get(p, {})
                for k in sorted(st):
                    v = st[k]
                    if isinstance(v, torch.Tensor) and v.device == p.device:
                        dist.broadcast(v, 0)

    def d_backward(self, noise, cams, real_imgs):
        """The discriminator half-step's gradients (training_utils.py:346-389): fake
        thumbnails generated in chunks, then ONE discriminator pass over the batch
        (logistic loss + R1 + viewpoint regression), all-reduced by DDP."""
        t = self.t
        batch, chunk = real_imgs.shape[0], t.chunk
        zero = torch.zeros((), device=real_imgs.device)
        cam, focal, near, far, gt_view = cams
        requires_grad(self.g_module.parameters(), False)
        requires_grad(self.d_module.parameters(), True)
        self.d_module.zero_grad(set_to_none=True)
        gen = []
        for j in range(0, batch, chunk):
            _, fake = self.g_module([n[j:j + chunk] for n in noise], cam[j:j + chunk],
                                    focal[j:j + chunk], near[j:j + chunk], far[j:j + chunk])
            gen.append(fake)
        gen = torch.cat(gen, 0)
        fake_pred, fake_view_pred = self.discriminator(gen.detach())
        view = t.view_lambda > 0
        d_view = t.view_lambda * viewpoints_loss(fake_view_pred, gt_view) if view else zero
        real = real_imgs.detach().requires_grad_(True)
        real_pred, _ = self.discriminator(real)
        d_gan = d_logistic_loss(real_pred, fake_pred)
        r1 = t.r1 * 0.5 * d_r1_loss(real_pred, real)
        (d_gan + r1 + d_view).backward()
        return d_gan, r1, d_view, real_pred, fake_pred

    def step(self, real_imgs):
        t, dev = self.t, self.device
        batch, chunk = real_imgs.shape[0], t.chunk
        loss = {}

        # --- discriminator (training_utils.py:336-394)
        noise = mixing_noise(batch, t.style_dim, t.mixing, dev)
        cams = self._cams(batch)
        d_gan, r1, d_view, real_pred, fake_pred = self.d_backward(noise, cams, real_imgs)
        self.optimizer_d.step()
        loss.update(d=d_gan, r1=r1, d_view=d_view, real_score=real_pred.mean(),
                    fake_score=fake_pred.mean())

        # --- generator (training_utils.py:396-451)
        n_chunks = len(range(0, batch, chunk))
        inputs = ((mixing_noise(chunk, t.style_dim, t.mixing, dev), self._cams(chunk))
                  for _ in range(n_chunks))
        g_gan, g_view, g_eik, g_surf, g_smooth = self.g_backward(inputs, n_chunks)
        self.optimizer.step()
        self.g_module.zero_grad(set_to_none=True)
        loss.update(g=g_gan, g_view=g_view, g_eikonal=g_eik, g_minimal_surface=g_surf,
                    g_smooth=g_smooth)
        accumulate(self.generator_test, self.g_module, self.accum)
        self.iteration += 1
        return reduce_loss_dict(loss)

    def g_backward(self, chunk_inputs, n_chunks):
        """The generator half-step's gradients (training_utils.py:396-440): per chunk
        the adversarial, viewpoint, eikonal, minimal-surface and smoothness terms,
        accumulated locally and all-reduced on the last chunk."""
        t, dev = self.t, self.device
        view = t.view_lambda > 0
        with_sdf = getattr(t, "with_sdf", True)
        zero = torch.zeros((), device=dev)
        requires_grad(self.g_module.parameters(), True)
        requires_grad(self.d_module.parameters(), False)
        eik_on, surf_on = with_sdf and t.eikonal_lambda > 0, t.min_surf_lambda > 0
        g_view = g_eik = g_surf = g_smooth = zero
        for k, (noise, cams) in enumerate(chunk_inputs):
            cam, focal, near, far, gt_view = cams
            with self._sync(self.generator, k == n_chunks - 1):
                out = self.generator(noise, cam, focal, near, far, return_sdf=surf_on,
                                     return_eikonal=eik_on)
                fake = out[1]
                sdf = out[2] if surf_on else None
                eik_term = out[2 + int(surf_on)] if eik_on else None
                fake_pred, fake_view_pred = self.d_module(fake)
                if view:
                    g_view = t.view_lambda * viewpoints_loss(fake_view_pred, gt_view)
                if eik_on:
                    g_eik, g_surf = eikonal_loss(eik_term, sdf=sdf, beta=t.min_surf_beta)
                    g_eik = t.eikonal_lambda * g_eik
                    if surf_on:
                        g_surf = t.min_surf_lambda * g_surf
                    # fixed box of the reference (training_utils.py:433-436); only the
                    # hash-grid network has query_sdf (the reference raises for SIREN)
                    if hasattr(self.g_module.renderer.network, "query_sdf"):
                        box = torch.tensor([[-1.0, 7.0], [-1.3, 3.7], [-1.7, 1.4]], device=dev)
                        g_smooth = 1000 * smoothness(self.g_module, box, noise, dev)
                g_gan = g_nonsaturating_loss(fake_pred)
                (g_gan + g_view + g_eik + g_surf + g_smooth).backward()
        return g_gan, g_view, g_eik, g_surf, g_smooth

    def state_dict(self):
        """{g, d, g_ema} as the reference's volume_renderer checkpoints."""
        return {"g": self.g_module.state_dict(), "d": self.d_module.state_dict(),
                "g_ema": self.generator_test.state_dict()}
