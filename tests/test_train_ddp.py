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
