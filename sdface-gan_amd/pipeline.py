"""train.py's SDF branch: stage gating, sphere initialisation, the two training
stages and their checkpoints (train.py:69-147, training_utils.py:197-881).

    need_vol, need_full = checkpoint.stage_plan(ckpt_dir, expname, wod)
    if need_vol:  train_vol_render(opt_stage1, expname, loader, device, ckpt_dir)
    if need_full: train_full_pipeline(opt_stage2, expname, loader, device, ckpt_dir)

``loader`` yields real image batches: 64^2 thumbnails for stage 1, 256^2 images for
stage 2 (the reference's lmdb MultiResolutionDataset yields both; dataset IO is out
of scope).  Each function returns its trainer.

Stage-2 resume: the reference re-initialises g_ema to the generator's weights after
loading a checkpoint (training_utils.py:615-616 runs on every start, resumed or not),
discarding the saved EMA.  ``train_full_pipeline(..., reference_resume_ema=True)`` (the
default) does the same, so a resumed run follows the reference's; with ``False`` a
resumed run keeps the checkpoint's g_ema and equals an uninterrupted run.
"""
from __future__ import annotations

from . import checkpoint as ck
from .training import FullPipelineTrainer, RendererTrainer, accumulate


def train_vol_render(opt, expname, loader, device, checkpoints_dir, iters=10000,
                     sphere_init_iters=10000, seed=0, on_step=None):
    """Stage 1 (training_utils.py:197-549): resume from the newest
    volume_renderer/models_*.pt, else start from sdf_init_models.pt, else run the
    sphere initialisation and write it; then up to ``iters`` iterations
    (the reference runs 10,000 per invocation, :333) with periodic checkpoints and
    the final vol_renderer.pt."""
    tr = RendererTrainer(opt, device, seed=seed)
    t = opt.training
    start = ck.resume(tr, checkpoints_dir, expname, 1)
    init_path = ck.exp_dir(checkpoints_dir, expname) / ck.SPHERE_INIT
    with_sdf = getattr(t, "with_sdf", True)
    if start == 0 and with_sdf and not getattr(t, "no_sphere_init", False):
        if ck.agree(init_path.exists()):
            ck.load_into(tr, ck.load_file(init_path))
            tr.iteration = 0
        else:
            for _ in range(sphere_init_iters):
                tr.sphere_init_step()
            tr.sphere_init_finish()
            accumulate(tr.generator_test, tr.g_module, 0)
            ck.save(init_path, tr, with_optim=False)
    for idx in range(iters):
        i = idx + start
        if i > t.iter:
            break
        tr.iteration = i
        losses = tr.step(next(loader))
        if on_step is not None:
            on_step(i, losses)
        if ck.stage1_checkpoint_due(i):
            ck.save(ck.ckpt_path(checkpoints_dir, expname, 1, i), tr)
    ck.save_final(tr, checkpoints_dir, expname, 1)
    return tr


def train_full_pipeline(opt, expname, loader, device, checkpoints_dir, iters=None, wod=False,
                        seed=0, on_step=None, reference_resume_ema=True):
    """Stage 2 (training_utils.py:552-881): resume from the newest
    full_pipeline/models_*.pt, else copy the size-matching g_ema entries of
    vol_renderer.pt (sdf_init_models.pt with ``wod``) into the generator; then set
    g_ema := g (on a resume only with ``reference_resume_ema``, as the reference
    does, training_utils.py:615-616) and train with periodic checkpoints and the
    final full_pipeline.pt."""
    tr = FullPipelineTrainer(opt, device, seed=seed)
    t = opt.training
    start = ck.resume(tr, checkpoints_dir, expname, 2)
    if start == 0:
        src = ck.exp_dir(checkpoints_dir, expname) / (ck.SPHERE_INIT if wod else ck.STAGE_FINAL[1])
        ck.load_size_matched(tr.g_module, ck.load_file(src)["g_ema"])
    if start == 0 or reference_resume_ema:
        accumulate(tr.generator_test, tr.g_module, 0)
    n = t.iter if iters is None else iters
    for idx in range(n):
        i = idx + start
        if i > t.iter:
            break
        tr.iteration = i
        losses = tr.step(next(loader))
        if on_step is not None:
            on_step(i, losses)
        if ck.stage2_checkpoint_due(i):
            ck.save(ck.ckpt_path(checkpoints_dir, expname, 2, i), tr)
    ck.save_final(tr, checkpoints_dir, expname, 2)
    return tr
