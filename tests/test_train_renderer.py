"""Stage-1 (volume renderer) training, training_utils.py:197-551: the
RendererTrainer's sphere initialisation and D + G iterations.

CPU: the SIREN network (configs[4]) on a world of 2 gloo processes -- the
renderer and the VolumeRenderDiscriminator train, both stay bit-identical across
ranks (DDP all-reduce), losses are finite and reduced over ranks.
GPU: the ngp network, where every hash-grid evaluation runs the HIP encoder
forward and its HIP backward (table gradients by fp32 atomics, dy_dx for the
eikonal term) -- the hash table itself must be updated by the G step."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def stage1_opt(sdfr, ngp, res=8, samples=4, batch=2, chunk=1):
    opt = sdfr.vol_render_opt(ngp=ngp, train_renderer=True, size=32, batch=batch, chunk=chunk)
    opt.model.renderer_spatial_output_dim = res
    opt.training.renderer_output_size = res
    opt.rendering.N_samples = samples
    return opt


def test_volume_render_discriminator_shapes(sdfr):
    from sdface_gan_amd.training import VolumeRenderDiscriminator
    opt = stage1_opt(sdfr, ngp=False, res=64)
    torch.manual_seed(0)
    d = VolumeRenderDiscriminator(opt.model)
    gan, view = d(torch.randn(3, 3, 64, 64))
    assert gan.shape == (3, 1) and view.shape == (3, 2)
    # channel plan of sdf_model.py:1361-1387 at 64^2: 3->128 (1x1), 5 res blocks, 2x2 head
    assert d.convs[0].conv.out_channels == 128
    assert [b.conv2.conv.conv.out_channels for b in list(d.convs)[1:]] == [256, 400, 400, 400, 400]
    assert d.final_conv.conv.kernel_size == (2, 2)


def test_add_coords_matches_reference_formula(sdfr):
    """AddCoords with its cached planes == sdf_model.py:1252-1275 rebuilt per call,
    bit for bit, with and without the zero channels CoordConv2d pads with; the
    gradient reaches only the input channels."""
    from sdface_gan_amd.training import AddCoords
    torch.manual_seed(0)
    for b, c, hh, ww in [(3, 5, 7, 9), (2, 128, 16, 16), (1, 1, 2, 2)]:
        x = torch.randn(b, c, hh, ww, requires_grad=True)
        xx = torch.arange(ww, dtype=torch.float32).repeat(1, 1, hh, 1)
        yy = torch.arange(hh, dtype=torch.float32).repeat(1, 1, ww, 1).transpose(2, 3)
        xx = (xx / (ww - 1)) * 2 - 1
        yy = (yy / (hh - 1)) * 2 - 1
        ref = torch.cat([x, yy.repeat(b, 1, 1, 1), xx.repeat(b, 1, 1, 1)], dim=1)
        assert torch.equal(AddCoords()(x), ref)
        out = AddCoords()(x, 3)
        assert out.shape == (b, c + 5, hh, ww)
        assert torch.equal(out[:, :c + 2], ref) and not out[:, c + 2:].any()
        out.sum().backward()
        assert torch.equal(x.grad, torch.ones_like(x))


def test_eikonal_loss_known_answer(sdfr):
    from sdface_gan_amd.training import eikonal_loss
    g = torch.tensor([[3.0, 4.0, 0.0], [0.0, 0.0, 1.0]])          # norms 5, 1
    sdf = torch.tensor([0.0, 0.01])
    eik, surf = eikonal_loss(g, sdf=sdf, beta=100)
    assert torch.allclose(eik, torch.tensor(8.0))                  # ((5-1)^2 + 0) / 2
    assert torch.allclose(surf, (1 + torch.exp(torch.tensor(-1.0))) / 2)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd.training import RendererTrainer
    opt = stage1_opt(sdfr, ngp=False)
    tr = RendererTrainer(opt, torch.device("cpu"), seed=5)
    before = {k: v.clone() for k, v in tr.g_module.state_dict().items()}
    torch.manual_seed(200 + rank)
    init_loss = float(tr.sphere_init_step(batch=2))
    # each rank ran its own sphere-init step (no per-step collective); the finish
    # hands every rank rank 0's generator and Adam moments
    sd = tr.g_module.state_dict()
    mine = {k: v.clone() for k, v in sd.items()}
    tr.sphere_init_finish()
    adam = [tr.optimizer.state[p]["exp_avg"].clone() for p in tr.g_module.parameters()
            if p in tr.optimizer.state]
    losses = []
    for _ in range(2):
        real = torch.rand(opt.training.batch, 3, 8, 8) * 2 - 1
        losses.append({k: float(v) for k, v in tr.step(real).items()})
    torch.save({"losses": losses, "init": init_loss, "real": real, "pre_finish": mine,
                "adam": adam,
                "d": tr.d_module.state_dict(), "g": tr.g_module.state_dict(),
                "g_before": before},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_stage1_ddp_two_ranks_stay_in_sync(sdfr, tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert not torch.equal(r0["real"], r1["real"])
    # before the finish the two sphere inits differed (different data per rank) ...
    assert any(not torch.equal(v, r1["pre_finish"][k]) for k, v in r0["pre_finish"].items()
               if k.startswith("renderer.network."))
    # ... after it both ranks hold rank 0's generator and optimizer moments
    assert all(torch.equal(a, b) for a, b in zip(r0["adam"], r1["adam"])) and r0["adam"]
    for k in r0["d"]:
        assert torch.equal(r0["d"][k], r1["d"][k]), f"discriminator {k} diverged"
    trained = 0
    for k, v in r0["g"].items():
        assert torch.equal(v, r1["g"][k]), f"generator {k} diverged"
        if k.startswith("renderer.network.") and k.endswith("weight"):
            trained += int(not torch.equal(v, r0["g_before"][k]))
    assert trained > 0, "no renderer weight was trained"
    assert r0["losses"] == r1["losses"]
    for step in r0["losses"]:
        assert set(step) >= {"d", "r1", "d_view", "g", "g_view", "g_eikonal",
                             "g_minimal_surface"}
        for k, v in step.items():
            assert torch.isfinite(torch.tensor(v)), (k, v)
    assert torch.isfinite(torch.tensor(r0["init"]))


@pytest.mark.gpu
def test_stage1_ngp_step_updates_hash_table(sdfr):
    from sdface_gan_amd.training import RendererTrainer
    dev = torch.device("cuda:0")
    opt = stage1_opt(sdfr, ngp=True, res=16, samples=8, batch=2, chunk=1)
    tr = RendererTrainer(opt, dev, seed=7)
    table = tr.g_module.renderer.network.encoder.embeddings
    before = table.detach().clone()
    torch.manual_seed(11)
    init = tr.sphere_init_step(batch=2)
    assert torch.isfinite(init)
    after_init = table.detach().clone()
    assert not torch.equal(before, after_init), "sphere init did not reach the hash table"
    real = torch.rand(2, 3, 16, 16, device=dev) * 2 - 1
    loss = tr.step(real)
    for k, v in loss.items():
        assert torch.isfinite(v).all(), (k, v)
    assert float(loss["g_eikonal"]) > 0 and float(loss["g_smooth"]) >= 0
    assert not torch.equal(after_init, table.detach()), "G step did not reach the hash table"
    torch.cuda.synchronize()


# --------------------------------------------------------------------------- correctness
# Stage 1: ONE discriminator pass over the batch (mean losses, no batch statistics:
# DDP grad == single-process grad) and per-chunk generator losses accumulated over
# the chunks (DDP grad == single-process grad / world).  Sampling offsets off
# (perturb 0) so the renderer is a deterministic function of the fixed inputs.
def _stage1_inputs(sdfr, opt, rank):
    torch.manual_seed(300 + rank)
    b, res = opt.training.batch, opt.training.renderer_output_size
    noise = [torch.randn(b, 256)]
    cams = sdfr.generate_camera_params(res, "cpu", batch=b)
    real = torch.rand(b, 3, res, res) * 2 - 1
    chunks = [([torch.randn(opt.training.chunk, 256)],
               sdfr.generate_camera_params(res, "cpu", batch=opt.training.chunk))
              for _ in range(0, b, opt.training.chunk)]
    return noise, cams, real, chunks


def _stage1_grads(tr, noise, cams, real, chunks):
    tr.d_backward(noise, cams, real)
    d = {n: p.grad.clone() for n, p in tr.d_module.named_parameters()}
    tr.g_backward(iter(chunks), len(chunks))
    g = {n: p.grad.clone() for n, p in tr.g_module.named_parameters() if p.grad is not None}
    return d, g


def _det_stage1_opt(sdfr):
    opt = stage1_opt(sdfr, ngp=False)
    opt.rendering.perturb = 0
    return opt


def _grad_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd.training import RendererTrainer
    opt = _det_stage1_opt(sdfr)
    tr = RendererTrainer(opt, torch.device("cpu"), seed=5)
    d, g = _stage1_grads(tr, *_stage1_inputs(sdfr, opt, rank))
    torch.save({"d": d, "g": g}, os.path.join(out_dir, f"grad{rank}.pt"))
    dist.destroy_process_group()


def test_stage1_ddp_gradients_equal_single_process(sdfr, tmp_path):
    from sdface_gan_amd.training import RendererTrainer
    port = _free_port()
    mp.spawn(_grad_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    opt = _det_stage1_opt(sdfr)
    ins = [_stage1_inputs(sdfr, opt, r) for r in (0, 1)]
    noise = [torch.cat([ins[0][0][0], ins[1][0][0]])]
    cams = tuple(torch.cat([a, b]) for a, b in zip(ins[0][1], ins[1][1]))
    real = torch.cat([ins[0][2], ins[1][2]])
    chunks = ins[0][3] + ins[1][3]
    opt.training.batch *= 2
    threads = torch.get_num_threads()
    torch.set_num_threads(2)                      # the workers' CPU reduction order
    try:
        tr = RendererTrainer(opt, torch.device("cpu"), seed=5)
        d, g = _stage1_grads(tr, noise, cams, real, chunks)
    finally:
        torch.set_num_threads(threads)
    for rank in (0, 1):
        r = torch.load(tmp_path / f"grad{rank}.pt", weights_only=True)
        for what, got, ref, scale in (("discriminator", r["d"], d, 1.0),
                                      ("generator", r["g"], g, 0.5)):
            assert set(got) == set(ref), what
            for k, v in got.items():
                want = ref[k] * scale
                tol = 1e-5 * max(1e-3, float(want.abs().max()))
                assert torch.allclose(v, want, rtol=1e-4, atol=tol), \
                    f"{what} {k}: max |diff| {float((v - want).abs().max()):.3e}"
