"""Data-parallel stage-2 training: the FullPipelineTrainer on a
world of 2 gloo processes on CPU.  The SIREN renderer (configs[4]'s network) is
used because it runs on CPU; the ngp renderer's HIP encoders need the GPU.

Checks: after two iterations (D step with R1, G step, path regularisation, EMA,
chunked gradient accumulation under no_sync) the discriminator and decoder are
bit-identical on both ranks (the gradient all-reduce ran), the frozen renderer
and mapping network are untouched, the losses are finite and the replicated
batches differ per rank (independent data)."""
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


def tiny_opt(sdfr):
    opt = sdfr.vol_render_opt(ngp=False, size=32, batch=2, chunk=1)
    opt.model.renderer_spatial_output_dim = 8
    opt.training.renderer_output_size = 8
    opt.rendering.N_samples = 4
    opt.training.d_reg_every = 1
    opt.training.g_reg_every = 1
    return opt


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = tiny_opt(sdfr)
    tr = FullPipelineTrainer(opt, torch.device("cpu"), seed=3)
    before = {k: v.clone() for k, v in tr.g_module.state_dict().items()}
    torch.manual_seed(100 + rank)                 # per-rank data and noise
    losses = []
    for _ in range(2):
        real = torch.rand(opt.training.batch, 3, 32, 32) * 2 - 1
        losses.append({k: float(v) for k, v in tr.step(real).items()})
    torch.save({"losses": losses, "real": real,
                "d": tr.d_module.state_dict(), "g": tr.g_module.state_dict(),
                "g_before": before, "ema": tr.generator_test.state_dict()},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_two_ranks_stay_in_sync(sdfr, tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert not torch.equal(r0["real"], r1["real"])
    for k in r0["d"]:
        assert torch.equal(r0["d"][k], r1["d"][k]), f"discriminator {k} diverged"
    changed = 0
    for k, v in r0["g"].items():
        assert torch.equal(v, r1["g"][k]), f"generator {k} diverged"
        if k.startswith("decoder.") and k.endswith("weight"):
            changed += int(not torch.equal(v, r0["g_before"][k]))
        if k.startswith("renderer.") or k.startswith("style."):
            assert torch.equal(v, r0["g_before"][k]), f"frozen {k} was updated"
    assert changed > 0, "no decoder weight was trained"
    for step in r0["losses"]:
        for k, v in step.items():
            assert torch.isfinite(torch.tensor(v)), (k, v)
    assert r0["losses"] == r1["losses"]           # reduced over ranks


def test_single_process_step(sdfr):
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = tiny_opt(sdfr)
    tr = FullPipelineTrainer(opt, torch.device("cpu"), seed=1)
    out = tr.step(torch.rand(2, 3, 32, 32) * 2 - 1)
    assert set(out) == {"d", "real_score", "fake_score", "r1", "g", "path", "path_length"}
    sd = tr.state_dict()
    assert set(sd) == {"g", "d", "g_ema"}
    assert any(k.startswith("final_linear") for k in sd["d"])


# --------------------------------------------------------------------------- correctness
# the world-2 gradients equal a single process's on the concatenated
# batch.  Inputs (latents, cameras, real images) are fixed per rank; the decoder's
# noise comes from its fixed buffers (randomize_noise False) and the renderer's
# sampling offsets are off (perturb 0), so both runs see the same function.  Stage 2 accumulates per-chunk mean losses (training_utils.py:
# 661-742) and DDP averages over ranks, so DDP grad == single-process grad / world.
def _det_opt(sdfr):
    opt = tiny_opt(sdfr)
    opt.rendering.perturb = 0
    return opt


def _stage2_inputs(sdfr, opt, rank):
    torch.manual_seed(100 + rank)
    b, res = opt.training.batch, opt.training.renderer_output_size
    noise = [torch.randn(b, 256)]
    cams = sdfr.generate_camera_params(res, "cpu", batch=b)
    real = torch.rand(b, 3, 32, 32) * 2 - 1
    chunks = []
    for _ in range(0, b, opt.training.chunk):
        chunks.append(([torch.randn(opt.training.chunk, 256)],
                       sdfr.generate_camera_params(res, "cpu", batch=opt.training.chunk)))
    return noise, cams, real, chunks


def _stage2_grads(tr, noise, cams, real, chunks):
    tr.randomize_noise = False
    tr.d_backward(noise, cams, real, True)
    d = {n: p.grad.clone() for n, p in tr.d_module.named_parameters()}
    tr.g_backward(iter(chunks), len(chunks))
    g = {n: p.grad.clone() for n, p in tr.g_module.named_parameters() if p.grad is not None}
    return d, g


def _grad_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = _det_opt(sdfr)
    tr = FullPipelineTrainer(opt, torch.device("cpu"), seed=3)
    d, g = _stage2_grads(tr, *_stage2_inputs(sdfr, opt, rank))
    torch.save({"d": d, "g": g}, os.path.join(out_dir, f"grad{rank}.pt"))
    dist.destroy_process_group()


def _close_grads(ddp, single, scale, what):
    assert set(ddp) == set(single), what
    for k, v in ddp.items():
        ref = single[k] * scale
        tol = 1e-5 * max(1e-3, float(ref.abs().max()))
        assert torch.allclose(v, ref, rtol=1e-4, atol=tol), \
            f"{what} {k}: max |diff| {float((v - ref).abs().max()):.3e} scale {float(ref.abs().max()):.3e}"


def test_ddp_gradients_equal_single_process_concatenated_batch(sdfr, tmp_path):
    from sdface_gan_amd.training import FullPipelineTrainer
    port = _free_port()
    mp.spawn(_grad_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "grad0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "grad1.pt", weights_only=True)
    opt = _det_opt(sdfr)
    ins = [_stage2_inputs(sdfr, opt, r) for r in (0, 1)]
    noise = [torch.cat([ins[0][0][0], ins[1][0][0]])]
    cams = tuple(torch.cat([a, b]) for a, b in zip(ins[0][1], ins[1][1]))
    real = torch.cat([ins[0][2], ins[1][2]])
    chunks = ins[0][3] + ins[1][3]
    opt.training.batch *= 2
    threads = torch.get_num_threads()
    torch.set_num_threads(2)                      # the workers' CPU reduction order
    try:
        tr = FullPipelineTrainer(opt, torch.device("cpu"), seed=3)
        d, g = _stage2_grads(tr, noise, cams, real, chunks)
    finally:
        torch.set_num_threads(threads)
    for r in (r0, r1):
        _close_grads(r["d"], d, 0.5, "discriminator")
        _close_grads(r["g"], g, 0.5, "decoder")
    assert all(k.startswith("decoder.") for k in g)
