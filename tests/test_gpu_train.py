"""GPU: the training configurations on one MI355X.

configs[2] (ffhq_256_sdf_ngp train.py) and configs[4] (the ngp=0 SIREN generator):
one full-size stage-2 FullPipelineTrainer step (batch 8, chunk 2, 256^2: the frozen
renderer on the fused HIP forward, the decoder trained on the module path), one
stage-1 RendererTrainer sphere-init + D/G step at 64^2 (chunk 2: every hash-grid
evaluation on the HIP encoder forward / backward, dy_dx for the eikonal term), for
both networks; then the data-parallel paths with two processes sharing the GPU over
gloo: a DDP stage-2 step (replicas stay identical) and bench.py's own multi-rank
timing (barrier + MAX over ranks, value = all ranks' faces / time).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
REPO = Path(__file__).resolve().parents[1]


def _snap(module, prefixes):
    return {k: v.detach().clone() for k, v in module.state_dict().items()
            if k.startswith(prefixes)}


def _changed(before, module):
    now = module.state_dict()
    return [k for k, v in before.items() if not torch.equal(v, now[k])]


@pytest.mark.parametrize("ngp", [True, False], ids=["ngp", "siren"])
def test_stage2_full_size_step(sdfr, ngp):
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = sdfr.vol_render_opt(ngp=ngp)                     # size 256, batch 8, chunk 2
    assert (opt.training.batch, opt.training.chunk, opt.model.size) == (8, 2, 256)
    tr = FullPipelineTrainer(opt, DEV, seed=0)
    frozen = _snap(tr.g_module, ("renderer.", "style."))
    dec = _snap(tr.g_module, ("decoder.",))
    d0 = _snap(tr.d_module, ("",))
    cam, focal, near, far, _ = sdfr.generate_camera_params(64, DEV, batch=2)
    with torch.no_grad():                                  # stage 2: the fused renderer
        assert tr.g_module.renderer._fused_ok(cam, torch.zeros(2, 256, device=DEV), False)
    torch.manual_seed(1)
    for _ in range(2):                                     # i = 0: R1 and path regularisation
        losses = tr.step(torch.rand(8, 3, 256, 256, device=DEV) * 2 - 1)
        for k, v in losses.items():
            assert torch.isfinite(v), (k, v)
    assert not _changed(frozen, tr.g_module), "frozen renderer / mapping was updated"
    assert len(_changed(dec, tr.g_module)) > 10
    assert len(_changed(d0, tr.d_module)) > 10
    ema = tr.generator_test.state_dict()
    assert any(not torch.equal(ema[k], v) for k, v in tr.g_module.state_dict().items()
               if k.startswith("decoder.") and k.endswith("weight"))


def test_accumulate_foreach_bit_identical(sdfr):
    """The EMA as two foreach launches == the reference's per-parameter mul_ / add_
    (sdf_utils.py:64-69) on the GPU's kernels, and it bumps every parameter's version
    (the decoder's weight caches key on it); the stage-2 generator Adam as one group ==
    the reference's per-parameter groups (config.py:206-215), foreach kernels."""
    import copy
    from sdface_gan_amd.training import accumulate, accumulate_loop
    opt = sdfr.vol_render_opt(ngp=True)
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(DEV)
    e1 = copy.deepcopy(g)
    with torch.no_grad():
        for p in g.parameters():
            p.add_(torch.randn_like(p))
    e2 = copy.deepcopy(e1)
    v0 = [p._version for p in e1.parameters()]
    for decay in (0.5 ** (32 / 10000), 0.999):
        accumulate(e1, g, decay)
        accumulate_loop(e2, g, decay)
    assert all(p._version > v for p, v in zip(e1.parameters(), v0))
    for (k, a), b in zip(e1.named_parameters(), e2.parameters()):
        assert torch.equal(a, b), k
    params = [p for n, p in g.named_parameters() if n.startswith("decoder.")]
    r = 4 / 5
    kw = dict(lr=2e-3 * r, betas=(0 ** r, 0.99 ** r))
    pa = [p.detach().clone().requires_grad_() for p in params]
    pb = [p.detach().clone().requires_grad_() for p in params]
    oa = torch.optim.Adam([{"params": [p], "lr": kw["lr"]} for p in pa], **kw)
    ob = torch.optim.Adam(pb, **kw)
    for _ in range(3):
        grads = [torch.randn_like(p) for p in pa]
        for x, y, gr in zip(pa, pb, grads):
            x.grad, y.grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)


@pytest.mark.parametrize("ngp", [True, False], ids=["ngp", "siren"])
def test_stage1_step_64(sdfr, ngp):
    from sdface_gan_amd.training import RendererTrainer
    opt = sdfr.vol_render_opt(ngp=ngp, train_renderer=True)    # 64^2 thumbs, batch 8, chunk 2
    tr = RendererTrainer(opt, DEV, seed=0)
    g0 = _snap(tr.g_module, ("renderer.",))
    d0 = _snap(tr.d_module, ("",))
    torch.manual_seed(2)
    init = tr.sphere_init_step(batch=3)
    assert torch.isfinite(init)
    losses = tr.step(torch.rand(8, 3, 64, 64, device=DEV) * 2 - 1)
    for k, v in losses.items():
        assert torch.isfinite(v), (k, v)
    assert float(losses["g_eikonal"]) > 0
    changed = _changed(g0, tr.g_module)
    if ngp:
        assert "renderer.network.encoder.embeddings" in changed     # HIP table gradients
    assert "renderer.network.sigma_linear.weight" in changed
    assert len(_changed(d0, tr.d_module)) > 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, str(REPO))
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = sdfr.vol_render_opt(batch=2, chunk=1)
    tr = FullPipelineTrainer(opt, torch.device("cuda", 0), seed=3)
    torch.manual_seed(50 + rank)
    losses = tr.step(torch.rand(2, 3, 256, 256, device="cuda") * 2 - 1)
    torch.save({"losses": {k: float(v) for k, v in losses.items()},
                "d": {k: v.cpu() for k, v in tr.d_module.state_dict().items()},
                "dec": {k: v.cpu() for k, v in tr.g_module.state_dict().items()
                        if k.startswith("decoder.")}},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_world2_on_one_gpu(tmp_path):
    """Two ranks on cuda:0 over gloo: one stage-2 DDP step; replicas bit-identical."""
    mp.spawn(_ddp_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for part in ("d", "dec"):
        for k, v in r0[part].items():
            assert torch.equal(v, r1[part][k]), f"{part} {k} diverged"
    assert r0["losses"] == r1["losses"]


def test_bench_multi_rank_timing_world2():
    """bench.py's multi-rank path (torchrun, barrier + MAX-over-ranks timing, value =
    all ranks' faces / time) with two gloo ranks sharing the GPU."""
    env = dict(os.environ, SDFR_BENCH_BACKEND="gloo", SDFR_BENCH_SAME_DEVICE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(REPO / "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "4",
           "--no-cpu-baseline", "--no-extras"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]                # rank 0 prints one line
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["scaling"] == "weak"
    assert rec["value"] > 0
    assert abs(rec["value"] - 2 * 4 * 3 / (rec["ms_per_step"] * 3 / 1e3)) < 1e-6 * rec["value"]


# ------------------------------------------------------------------ ngp DDP gradients
# Stage 1 on the ngp network (the 12.66 M-row hash table: the dominant all-reduce of
# SURVEY.md §5), world 2 over gloo with both ranks on cuda:0: after one d_backward and
# one g_backward with perturb 0, every gradient equals a single process's on the
# concatenated batch (discriminator: equal; generator: x 1/2, per-chunk losses summed
# over 2x the chunks) -- training_utils.py:346-440, sdf_utils.py:344-379.
def _ngp_stage1_opt(sdfr, ngp=True):
    from tests.test_train_renderer import stage1_opt
    opt = stage1_opt(sdfr, ngp=ngp, res=16, samples=8, batch=2, chunk=1)
    opt.rendering.perturb = 0
    return opt


def _to_dev(x):
    if isinstance(x, torch.Tensor):
        return x.to(DEV)
    if isinstance(x, (list, tuple)):
        return type(x)(_to_dev(v) for v in x)
    return x


def _chunk_seeded_smoothness():
    """The smoothness term draws its voxel block from the CPU RNG (smoothLoss.py:5-27):
    seed it from the chunk's own latents so that a rank and the single process draw
    the same block for the same chunk."""
    from sdface_gan_amd import training
    orig = training.smoothness

    def smoothness(generator, box, styles, device, *a, **k):
        torch.manual_seed(int(abs(float(styles[0].flatten()[0])) * 1e6) % (2 ** 31))
        return orig(generator, box, styles, device, *a, **k)
    training.smoothness = smoothness
    return orig


def _beta_term_sum():
    """sum_i |t_i| of renderer.sigmoid_beta's gradient, t_i = dL/dsigma_i dsigma_i/dbeta
    over every sample of every backward (sigma = sigmoid(x / beta) / beta, x = -sdf,
    sdf_model.py:227-229): the scale of the reordering error of that scalar's sum."""
    from sdface_gan_amd.renderer import VolumeFeatureRenderer as VR
    orig = VR.sdf_activation
    acc = {"abs": 0.0, "n": 0}

    def sdf_activation(self, input):
        out = orig(self, input)
        if out.requires_grad:
            beta, x = self.sigmoid_beta.detach(), input.detach()
            sg = torch.sigmoid(x / beta)
            dsdb = -sg * (1 - sg) * x / beta ** 3 - sg / beta ** 2

            def hook(g):
                acc["abs"] += float((g * dsdb).abs().sum(dtype=torch.float64))
                acc["n"] += g.numel()
            out.register_hook(hook)
        return out
    VR.sdf_activation = sdf_activation
    return orig, acc


def _ngp_grads(tr, noise, cams, real, chunks):
    tr.d_backward(_to_dev(noise), _to_dev(cams), _to_dev(real))
    d = {n: p.grad.detach().cpu() for n, p in tr.d_module.named_parameters()}
    tr.g_backward(iter(_to_dev(chunks)), len(chunks))
    g = {n: p.grad.detach().cpu() for n, p in tr.g_module.named_parameters()
         if p.grad is not None}
    return d, g


def _ngp_grad_worker(rank, world, port, out_dir, ngp=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    torch.backends.cudnn.deterministic = True
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, str(REPO))
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd.training import RendererTrainer
    from tests.test_train_renderer import _stage1_inputs
    opt = _ngp_stage1_opt(sdfr, ngp)
    tr = RendererTrainer(opt, DEV, seed=5)
    _chunk_seeded_smoothness()
    d, g = _ngp_grads(tr, *_stage1_inputs(sdfr, opt, rank))
    torch.save({"d": d, "g": g}, os.path.join(out_dir, f"ngp_grad{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("ngp", [True, False], ids=["ngp", "siren"])
def test_stage1_ddp_gradients_equal_single_process(sdfr, tmp_path, ngp):
    """configs[2] (ngp) and configs[4] (SIREN, ngp=0: the eikonal loss reaches the MLP
    through the double backward on the HIP training GEMMs)."""
    from sdface_gan_amd.training import RendererTrainer
    from tests.test_train_renderer import _stage1_inputs
    mp.spawn(_ngp_grad_worker, args=(2, _free_port(), str(tmp_path), ngp), nprocs=2, join=True)
    opt = _ngp_stage1_opt(sdfr, ngp)
    ins = [_stage1_inputs(sdfr, opt, r) for r in (0, 1)]
    noise = [torch.cat([ins[0][0][0], ins[1][0][0]])]
    cams = tuple(torch.cat([a, b]) for a, b in zip(ins[0][1], ins[1][1]))
    real = torch.cat([ins[0][2], ins[1][2]])
    chunks = ins[0][3] + ins[1][3]
    opt.training.batch *= 2
    from sdface_gan_amd import training
    from sdface_gan_amd.renderer import VolumeFeatureRenderer as VR
    torch.backends.cudnn.deterministic = True        # MIOpen: deterministic solvers
    orig = _chunk_seeded_smoothness()
    orig_act, beta_terms = _beta_term_sum()
    runs = []
    try:
        for _ in range(2):                 # twice: the single process's own run-to-run spread
            beta_terms["abs"], beta_terms["n"] = 0.0, 0
            tr = RendererTrainer(opt, DEV, seed=5)
            runs.append(_ngp_grads(tr, noise, cams, real, chunks))
    finally:
        training.smoothness = orig
        VR.sdf_activation = orig_act
    d, g = runs[0]
    # which gradients are not bit-identical between two identical single-process steps:
    # the binned hash-table gradient sums its per-bin entries with LDS atomics (order
    # varies run to run); everything else must be deterministic
    varies = sorted(k for k in list(runs[0][0]) + list(runs[0][1])
                    if not torch.equal(runs[0][0].get(k, runs[0][1].get(k)),
                                       runs[1][0].get(k, runs[1][1].get(k))))
    print("run-to-run varying gradients:", varies)
    # and, without deterministic MIOpen solvers, the discriminator's first convolution's
    # weight gradient (MIOpen backward-weights, measured in round 5)
    assert set(varies) <= {"renderer.network.encoder.embeddings", "convs.0.conv.weight"}, varies
    table = "renderer.network.encoder.embeddings"
    if ngp:
        assert table in g and float(g[table].abs().max()) > 0
    else:
        assert float(g["renderer.network.pts_linears.3.weight"].abs().max()) > 0
    for rank in (0, 1):
        r = torch.load(tmp_path / f"ngp_grad{rank}.pt", weights_only=True)
        for what, got, ref, scale in (("discriminator", r["d"], d, 1.0),
                                      ("generator", r["g"], g, 0.5)):
            assert set(got) == set(ref), what
            for k, v in got.items():
                want = ref[k] * scale
                # fp32 sums in a different order (atomics / binned table gradient,
                # the all-reduce): relative to the tensor's largest entry; for
                # renderer.sigmoid_beta -- one cancelling sum of n = 8192 terms t_i,
                # |g| ~ 3e-7 against sum |t_i| ~ 3e-5 -- a reordered-sum bound
                # c sqrt(n) u sum |t_i| (u = 2^-24) from the terms measured in this run;
                # c = 16: the world-2 value landed up to ~9.4 sqrt(n) u sum |t_i| from the
                # single process's over round 6's runs (the single process is bit-stable,
                # profiles/round6_beta_grad_ab.txt)
                tol = 2e-5 * float(want.abs().max())
                if k == "renderer.sigmoid_beta":
                    tol = max(tol, 16 * beta_terms["n"] ** 0.5 * 2.0 ** -24
                              * beta_terms["abs"] * scale)
                assert torch.allclose(v, want, rtol=2e-4, atol=tol), \
                    (f"{what} {k}: max |diff| {float((v - want).abs().max()):.3e} "
                     f"(max |ref| {float(want.abs().max()):.3e}, tol {tol:.3e}, "
                     f"beta terms {beta_terms})")
        if not ngp:
            continue
        # the hashed levels (5-15) carry most of the table's gradient rows
        off = int(tr.g_module.renderer.network.encoder.offsets[5])
        hashed = r["g"][table][off:]
        assert int((hashed != 0).any(1).sum()) > 1000


def test_renderer_grads_survive_frozen_decoder(sdfr):
    """Grad enabled, decoder frozen, renderer trainable: the decoder takes
    its autograd path (not the fused inference path) so the renderer gets gradients."""
    opt = sdfr.vol_render_opt()                      # full pipeline (features out)
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(DEV)
    g.is_train, g.train_renderer = True, True
    for p in g.decoder.parameters():
        p.requires_grad_(False)
    cam, focal, near, far, _ = sdfr.generate_camera_params(64, DEV, batch=1)
    z = torch.randn(1, 256, device=DEV)
    rgb, thumb = g([z], cam, focal, near, far)
    assert rgb.requires_grad
    rgb.mean().backward()
    w = g.renderer.network.views_linears.weight
    assert w.grad is not None and float(w.grad.abs().max()) > 0
    assert g.renderer.network.encoder.embeddings.grad is not None
