"""Checkpoint layout, resume and stage gating (training_utils.py:197-226, 318-324,
526-547, 555-606, 858-879; sdf_utils.py:382-401; train.py:69-89; eval.py:73-77),
on CPU with the SIREN network (configs[4]'s renderer; the ngp encoders need the GPU)."""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _stage2_opt(sdfr):
    opt = sdfr.vol_render_opt(ngp=False, size=32, batch=2, chunk=1)
    opt.model.renderer_spatial_output_dim = 8
    opt.training.renderer_output_size = 8
    opt.rendering.N_samples = 4
    opt.training.d_reg_every = 2
    opt.training.g_reg_every = 2
    return opt


def _stage1_opt(sdfr):
    opt = sdfr.vol_render_opt(ngp=False, train_renderer=True, size=32, batch=2, chunk=1)
    opt.model.renderer_spatial_output_dim = 8
    opt.training.renderer_output_size = 8
    opt.rendering.N_samples = 4
    return opt


def _loader(res, seed):
    g = torch.Generator().manual_seed(seed)
    while True:
        yield torch.rand(2, 3, res, res, generator=g) * 2 - 1


def _reseed(s):
    torch.manual_seed(s)
    random.seed(s)


def test_get_ckpt_nums(sdfr, tmp_path):
    from sdface_gan_amd import checkpoint as ck
    assert ck.get_ckpt_nums(tmp_path / "missing") is None
    assert ck.get_ckpt_nums(tmp_path) is None
    for n in ("models_0001000.pt", "models_0000500.pt", "models_x.pt", "other_0002000.pt"):
        (tmp_path / n).write_bytes(b"")
    assert ck.get_ckpt_nums(tmp_path) == "1000"
    p = ck.ckpt_path(tmp_path, "exp", 2, 42)
    assert p == tmp_path / "exp" / "full_pipeline" / "models_0000042.pt"


def test_stage2_save_resume_bit_identical(sdfr, tmp_path):
    """Two uninterrupted iterations after a checkpoint == the same two iterations
    after resuming from it in a fresh trainer (same RNG seed for the data draws)."""
    from sdface_gan_amd import checkpoint as ck
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = _stage2_opt(sdfr)
    cpu = torch.device("cpu")
    a = FullPipelineTrainer(opt, cpu, seed=3)
    data = _loader(32, 0)
    for _ in range(2):
        a.step(next(data))
    ck.save(ck.ckpt_path(tmp_path, "exp", 2, a.iteration - 1), a)
    payload = ck.load_file(ck.ckpt_path(tmp_path, "exp", 2, 1))
    assert {"g", "d", "g_ema", "g_optim", "d_optim"} <= set(payload)
    tail = [next(data) for _ in range(2)]
    _reseed(11)
    for x in tail:
        a.step(x)
    b = FullPipelineTrainer(opt, cpu, seed=99)          # different init: the load must matter
    assert ck.resume(b, tmp_path, "exp", 2) == 2
    assert b.mean_path_length == payload["mean_path_length"]
    _reseed(11)
    for x in tail:
        b.step(x)
    for name, sa, sb in (("g", a.g_module, b.g_module), ("d", a.d_module, b.d_module),
                         ("g_ema", a.generator_test, b.generator_test)):
        for k, v in sa.state_dict().items():
            assert torch.equal(v, sb.state_dict()[k]), f"{name}.{k}"
    assert a.iteration == b.iteration == 4


@pytest.mark.parametrize("reference_resume_ema", [True, False])
def test_stage2_resume_ema(sdfr, tmp_path, reference_resume_ema):
    """Stage-2 resume: by default g_ema := g after the checkpoint load, as the reference
    (training_utils.py:615-616 runs on every start); reference_resume_ema=False keeps
    the checkpoint's g_ema."""
    from sdface_gan_amd import checkpoint as ck
    from sdface_gan_amd import pipeline
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = _stage2_opt(sdfr)
    cpu = torch.device("cpu")
    a = FullPipelineTrainer(opt, cpu, seed=3)
    data = _loader(32, 0)
    for _ in range(2):
        a.step(next(data))
    ck.save(ck.ckpt_path(tmp_path, "exp", 2, 1), a)
    saved = ck.load_file(ck.ckpt_path(tmp_path, "exp", 2, 1))
    dec = [k for k in saved["g"] if k.startswith("decoder.") and "weight" in k]
    assert any(not torch.equal(saved["g"][k], saved["g_ema"][k]) for k in dec)
    tr = pipeline.train_full_pipeline(opt, "exp", data, cpu, tmp_path, iters=0,
                                      reference_resume_ema=reference_resume_ema)
    want = saved["g"] if reference_resume_ema else saved["g_ema"]
    got = tr.generator_test.state_dict()
    for k in dec:
        assert torch.equal(got[k], want[k]), k


@pytest.mark.parametrize("foreach", [True, False])
def test_g_adam_one_group_equals_per_parameter_groups(foreach):
    """The stage-2 generator optimizer as one param group gives the reference's
    per-parameter groups' update (config.py:206-215) bit for bit, and a state saved in
    the per-group layout loads into it (checkpoint.merge_param_groups)."""
    from sdface_gan_amd import checkpoint as ck
    g = torch.Generator().manual_seed(0)
    shapes = [(64, 32, 3, 3), (64,), (1, 3, 64, 1, 1), (512, 512), (3,)]
    p0 = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(4)]
    ratio = 4 / 5
    kw = dict(lr=2e-3 * ratio, betas=(0 ** ratio, 0.99 ** ratio), foreach=foreach)

    def run(grouped, steps, params=None, opt=None):
        ps = params or [p.clone().requires_grad_() for p in p0]
        if opt is None:
            opt = torch.optim.Adam([{"params": [p], "lr": kw["lr"]} for p in ps] if grouped
                                   else ps, **kw)
        for gs in steps:
            for p, gr in zip(ps, gs):
                p.grad = gr.clone()
            opt.step()
        return ps, opt

    ref, ref_opt = run(True, grads)
    one, _ = run(False, grads)
    for a, b in zip(ref, one):
        assert torch.equal(a, b)
    # two steps in the per-group layout, saved; two more in the single group
    half, half_opt = run(True, grads[:2])
    ps = [p.detach().clone().requires_grad_() for p in half]
    opt = torch.optim.Adam(ps, **kw)
    opt.load_state_dict(ck.merge_param_groups(half_opt.state_dict(), opt))
    run(False, grads[2:], ps, opt)
    for a, b in zip(ref, ps):
        assert torch.equal(a, b)
    bad = ref_opt.state_dict()
    bad["param_groups"][1]["lr"] = 1.0
    with pytest.raises(ValueError, match="differ"):
        ck.merge_param_groups(bad, opt)


def test_load_size_matched(sdfr):
    from sdface_gan_amd import checkpoint as ck
    opt = _stage2_opt(sdfr)
    g = sdfr.Generator(opt.model, opt.rendering)
    sd = {k: v.clone() + 1 for k, v in g.state_dict().items()}
    k0 = "renderer.network.rgb_linear.weight"
    sd[k0] = torch.zeros(5, 5)                          # wrong shape: skipped
    copied = ck.load_size_matched(g, sd)
    assert k0 not in copied and len(copied) == len(sd) - 1
    assert torch.equal(g.state_dict()["style.0.weight"], sd["style.0.weight"])


def test_two_stage_pipeline_gating_and_files(sdfr, tmp_path):
    """train.py's gating: stage 1 writes the sphere init, a periodic checkpoint and
    vol_renderer.pt; stage 2 starts from vol_renderer.pt's g_ema (size-matched) and
    writes full_pipeline.pt; then nothing is left to train."""
    from sdface_gan_amd import checkpoint as ck
    from sdface_gan_amd import pipeline
    cpu = torch.device("cpu")
    assert ck.stage_plan(tmp_path, "exp") == (True, True)
    o1 = _stage1_opt(sdfr)
    t1 = pipeline.train_vol_render(o1, "exp", _loader(8, 1), cpu, tmp_path, iters=2,
                                   sphere_init_iters=1)
    d = tmp_path / "exp"
    assert (d / "sdf_init_models.pt").exists() and (d / "vol_renderer.pt").exists()
    assert (d / "volume_renderer" / "models_0000000.pt").exists()     # i % 1000 == 0
    assert ck.stage_plan(tmp_path, "exp") == (False, True)
    assert ck.stage_plan(tmp_path, "exp", wod=True) == (False, True)
    o2 = _stage2_opt(sdfr)
    t2 = pipeline.train_full_pipeline(o2, "exp", _loader(32, 2), cpu, tmp_path, iters=1)
    assert (d / "full_pipeline.pt").exists()
    assert ck.stage_plan(tmp_path, "exp") == (False, False)
    vol = ck.load_file(d / "vol_renderer.pt")["g_ema"]
    full = t2.g_module.state_dict()
    for k, v in vol.items():                             # renderer frozen in stage 2
        if k.startswith("renderer."):
            assert torch.equal(full[k], v), k
    assert t1.iteration == 2
    # a second stage-1 run resumes after the newest periodic checkpoint (iteration 0)
    t1b = pipeline.train_vol_render(o1, "exp", _loader(8, 1), cpu, tmp_path, iters=1,
                                    sphere_init_iters=1)
    assert t1b.iteration == 2


def _stage1_worker(rank, world, port, root):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd import checkpoint as ck
    from sdface_gan_amd import pipeline
    # rank 1 looks at a directory whose contents disagree with rank 0's (a lagging
    # view of a shared file system, exaggerated): a bogus sphere-init file and a
    # bogus periodic checkpoint.  Following its own view it would skip the sphere
    # init and its save() barrier, or resume elsewhere -- and hang the job.
    ckdir = os.path.join(root, f"r{rank}")
    if rank == 1:
        os.makedirs(os.path.join(ckdir, "exp", "volume_renderer"), exist_ok=True)
        open(os.path.join(ckdir, "exp", ck.SPHERE_INIT), "wb").close()
        open(os.path.join(ckdir, "exp", "volume_renderer", "models_0000500.pt"), "wb").close()
    plan = ck.stage_plan(ckdir, "exp")
    tr = pipeline.train_vol_render(_stage1_opt(sdfr), "exp", _loader(8, 1 + rank),
                                   torch.device("cpu"), ckdir, iters=2, sphere_init_iters=1)
    torch.save({"plan": plan, "it": tr.iteration, "g": tr.g_module.state_dict()},
               os.path.join(root, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_stage1_ranks_follow_rank0_file_decisions(sdfr, tmp_path):
    """World of 2 gloo ranks through train_vol_render's sphere init, periodic
    checkpoint and save_final (each save a barrier): every branch taken from the
    checkpoint directory is rank 0's (checkpoint.agree), so the ranks enter the same
    collectives and finish with identical weights; only rank 0 writes."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_stage1_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    assert tuple(r0["plan"]) == tuple(r1["plan"]) == (True, True)
    assert r0["it"] == r1["it"] == 2
    for k, v in r0["g"].items():
        assert torch.equal(v, r1["g"][k]), k
    d0, d1 = tmp_path / "r0" / "exp", tmp_path / "r1" / "exp"
    assert (d0 / "sdf_init_models.pt").exists() and (d0 / "vol_renderer.pt").exists()
    assert not (d1 / "vol_renderer.pt").exists()          # rank 1 never writes
