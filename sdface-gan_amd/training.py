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
    par1 = dict(model1.named_parameters())
    par2 = dict(model2.named_parameters())
    for k in par1.keys():
        par1[k].data.mul_(decay).add_(par2[k].data, alpha=1 - decay)


def make_noise(batch, latent_dim, n_noise, device):
    if n_noise == 1:
        return torch.randn(batch, latent_dim, device=device)
    return torch.randn(n_noise, batch, latent_dim, device=device).unbind(0)


def mixing_noise(batch, latent_dim, prob, device):
    if prob > 0 and random.random() < prob:
        return make_noise(batch, latent_dim, 2, device)
    return [make_noise(batch, latent_dim, 1, device)]


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def reduce_loss_dict(loss_dict):
    """Mean over ranks of every scalar loss (one all-reduce of a packed vector)."""
    keys = sorted(loss_dict)
    if not keys:
        return {}
    vals = torch.stack([loss_dict[k].detach().float().reshape(()) for k in keys])
    if _world() > 1:
        dist.all_reduce(vals)
        vals /= _world()
    return dict(zip(keys, vals))


# ---------------------------------------------------------------------------
# the data-parallel stage-2 trainer
# ---------------------------------------------------------------------------
class FullPipelineTrainer:
    """Generator + EMA copy + Discriminator + optimizers of stage 2, each rank
    holding full replicas; ``step(real_imgs)`` is one iteration of the reference
    loop (D step with R1 every d_reg_every, G step, path regularisation every
    g_reg_every, EMA)."""

    def __init__(self, opt, device, seed=0):
        self.opt, self.t, self.device = opt, opt.training, device
        self.world = _world()
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
        self.optimizer = torch.optim.Adam([{"params": [p], "lr": t.lr * g_ratio}
                                           for p in self.g_train],
                                          lr=t.lr * g_ratio, betas=(0 ** g_ratio, 0.99 ** g_ratio))
        self.optimizer_d = torch.optim.Adam(self.discriminator.parameters(), lr=t.lr * d_ratio,
                                            betas=(0 ** d_ratio, 0.99 ** d_ratio))
        accumulate(self.generator_test, self.generator, 0)
        self.g_module, self.d_module = self.generator, self.discriminator
        if self.world > 1:
            from torch.nn.parallel import DistributedDataParallel as DDP
            kw = dict(broadcast_buffers=False)
            if device.type == "cuda":
                kw.update(device_ids=[device.index], output_device=device.index)
            self.generator = DDP(self.generator, **kw)
            self.discriminator = DDP(self.discriminator, **kw)
        self.mean_path_length = 0.0
        self.accum = 0.5 ** (32 / (10 * 1000))
        self.iteration = 0

    def _cams(self, n):
        c = self.opt.camera
        return generate_camera_params(self.t.renderer_output_size, self.device, batch=n,
                                      uniform=c.uniform, azim_range=c.azim, elev_range=c.elev,
                                      fov_ang=c.fov, dist_radius=c.dist_radius)

    @staticmethod
    def _sync(model, last):
        """no_sync() for every chunk but the last: one all-reduce per optimizer step."""
        return nullcontext() if last or not hasattr(model, "no_sync") else model.no_sync()

    def step(self, real_imgs):
        t, dev = self.t, self.device
        i = self.iteration
        style_dim = self.opt.model.style_dim
        batch, chunk = real_imgs.shape[0], t.chunk
        loss = {}

        # --- discriminator (training_utils.py:652-716)
        requires_grad(self.g_train, False)
        requires_grad(self.d_module.parameters(), True)
        self.d_module.zero_grad(set_to_none=True)
        d_regularize = i % t.d_reg_every == 0
        noise = mixing_noise(batch, style_dim, t.mixing, dev)
        cam, focal, near, far, _ = self._cams(batch)
        r1_loss = torch.zeros((), device=dev)
        for j in range(0, batch, chunk):
            last = j + chunk >= batch
            with self._sync(self.discriminator, last):
                with torch.no_grad():
                    gen_imgs, _ = self.g_module([n[j:j + chunk] for n in noise], cam[j:j + chunk],
                                                focal[j:j + chunk], near[j:j + chunk],
                                                far[j:j + chunk])
                real = real_imgs[j:j + chunk].detach().requires_grad_(d_regularize)
                fake_pred = self.discriminator(gen_imgs)
                real_pred = self.discriminator(real)
                d_gan_loss = d_logistic_loss(real_pred, fake_pred)
                if d_regularize:
                    r1_loss = t.r1 * 0.5 * d_r1_loss(real_pred, real) * t.d_reg_every
                else:
                    r1_loss = torch.zeros_like(r1_loss)
                (d_gan_loss + r1_loss).backward()
        self.optimizer_d.step()
        loss.update(d=d_gan_loss, real_score=real_pred.mean(), fake_score=fake_pred.mean(),
                    r1=r1_loss.mean())

        # --- generator (training_utils.py:717-742)
        requires_grad(self.g_train, True)
        requires_grad(self.d_module.parameters(), False)
        for j in range(0, batch, chunk):
            last = j + chunk >= batch
            with self._sync(self.generator, last):
                noise = mixing_noise(chunk, style_dim, t.mixing, dev)
                cam, focal, near, far, _ = self._cams(chunk)
                fake_img, fake_thumb = self.generator(noise, cam, focal, near, far)
                fake_up = F.interpolate(fake_thumb, scale_factor=4)   # nn.Upsample(4), nearest
                g_gan_loss = g_nonsaturating_loss(self.d_module(fake_img))
                (g_gan_loss + 0.001 * g_content_loss(fake_img, fake_up)).backward()
        self.optimizer.step()
        self.g_module.zero_grad(set_to_none=True)
        loss["g"] = g_gan_loss

        # --- path length regularisation (training_utils.py:744-776)
        path_loss = torch.zeros((), device=dev)
        path_lengths = torch.zeros((), device=dev)
        if t.g_reg_every > 0 and i % t.g_reg_every == 0:
            pbs = max(1, batch // t.path_batch_shrink)
            noise = mixing_noise(pbs, style_dim, t.mixing, dev)
            cam, focal, near, far, _ = self._cams(pbs)
            for j in range(0, pbs, chunk):
                last = j + chunk >= pbs
                with self._sync(self.generator, last):
                    img, latents = self.generator([n[j:j + chunk] for n in noise],
                                                  cam[j:j + chunk], focal[j:j + chunk],
                                                  near[j:j + chunk], far[j:j + chunk],
                                                  return_latents=True)
                    path_loss, self.mean_path_length, path_lengths = g_path_regularize(
                        img, latents, self.mean_path_length)
                    w = t.path_regularize * t.g_reg_every * path_loss
                    if t.path_batch_shrink:
                        w = w + 0 * img[0, 0, 0, 0]
                    w.backward()
            self.optimizer.step()
            self.g_module.zero_grad(set_to_none=True)
            if self.world > 1:
                mpl = torch.as_tensor(self.mean_path_length, device=dev, dtype=torch.float32)
                dist.all_reduce(mpl)
                self.mean_path_length = mpl / self.world
        loss.update(path=path_loss, path_length=path_lengths.mean())

        accumulate(self.generator_test, self.g_module, self.accum)
        self.iteration += 1
        return reduce_loss_dict(loss)

    def state_dict(self):
        """{g, d, g_ema} as the reference's checkpoints (training_utils.py:857-880)."""
        return {"g": self.g_module.state_dict(), "d": self.d_module.state_dict(),
                "g_ema": self.generator_test.state_dict()}
