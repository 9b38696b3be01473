"""Checkpoints and stage orchestration of SDFace-GAN's two-stage training.

The reference's layout (training_utils.py, train.py, sdf_utils.py), kept file for
file so its checkpoints load here and these load there:

  <checkpoints_dir>/<expname>/volume_renderer/models_{iter:07d}.pt   stage 1, periodic
  <checkpoints_dir>/<expname>/sdf_init_models.pt                     after the sphere init
  <checkpoints_dir>/<expname>/vol_renderer.pt                        stage 1, final
  <checkpoints_dir>/<expname>/full_pipeline/models_{iter:07d}.pt     stage 2, periodic
  <checkpoints_dir>/<expname>/full_pipeline.pt                       stage 2, final

Each file is ``{"g", "d", "g_ema"}`` state dicts (training_utils.py:318-324,
526-547, 858-879).  Writes add ``g_optim`` / ``d_optim`` (which the reference's
stage-1 resume reads when present, training_utils.py:223-225) and this framework's
``iteration`` / ``mean_path_length`` so a resumed run continues exactly; the
reference ignores extra keys.

Resume picks the highest ``models_*.pt`` (``get_ckpt_nums``, sdf_utils.py:382-401)
and restarts at that iteration + 1 (training_utils.py:216-219).  Eval / mesh
extraction and the stage-2 start copy only the size-matching ``g_ema`` entries
(eval.py:73-77, sdf_mesh.py:235-240, training_utils.py:600-606).  Stage gating is
train.py:69-89: stage 1 runs while ``vol_renderer.pt`` is missing, stage 2 while
``full_pipeline.pt`` is missing (``--wod``: stage 2 only, from the sphere init).

Checkpoints are written by rank 0 only; every rank reads them; decisions taken from
the directory's contents are rank 0's, broadcast (``agree``).  Loading uses
``torch.load(weights_only=True)``: state dicts, optimizer states and numbers only.
"""
from __future__ import annotations

import os
import re
from pathlib import Path

import torch

STAGE_DIRS = {1: "volume_renderer", 2: "full_pipeline"}
STAGE_FINAL = {1: "vol_renderer.pt", 2: "full_pipeline.pt"}
SPHERE_INIT = "sdf_init_models.pt"


def _rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def agree(value):
    """Rank 0's ``value`` on every rank.  The file-system decisions that gate a
    collective (resume point, sphere-init present, stages left; save() is a barrier
    and every training step an all-reduce) are taken by rank 0 alone, so a rank with
    a lagging view of a shared directory cannot skip a collective the others enter."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    box = [value]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def exp_dir(checkpoints_dir, expname) -> Path:
    return Path(checkpoints_dir) / expname


def get_ckpt_nums(folder):
    """Largest N of the ``models_N.pt`` files in ``folder`` as a string, or None
    (sdf_utils.py:382-401; a missing folder has none)."""
    if not os.path.isdir(folder):
        return None
    nums = [int(m.group(1)) for f in os.listdir(folder)
            if (m := re.match(r"models_(\d+)\.pt", f))]
    return str(max(nums)) if nums else None


def ckpt_path(checkpoints_dir, expname, stage, iteration) -> Path:
    return exp_dir(checkpoints_dir, expname) / STAGE_DIRS[stage] / f"models_{str(iteration).zfill(7)}.pt"


def trainer_payload(trainer, with_optim=True):
    d = {"g": trainer.g_module.state_dict(), "d": trainer.d_module.state_dict(),
         "g_ema": trainer.generator_test.state_dict(), "iteration": int(trainer.iteration)}
    if hasattr(trainer, "mean_path_length"):
        d["mean_path_length"] = float(trainer.mean_path_length)
    if with_optim:
        d["g_optim"] = trainer.optimizer.state_dict()
        d["d_optim"] = trainer.optimizer_d.state_dict()
    return d


def _barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def save(path, trainer, with_optim=True):
    """Write ``{g, d, g_ema[, g_optim, d_optim, iteration, mean_path_length]}`` (rank 0).
    Collective when a process group is up: every rank calls it and leaves only once
    the file is in place, so no rank can read a checkpoint rank 0 is still writing
    (stage 2 loads vol_renderer.pt right after stage 1's save_final)."""
    path = Path(path)
    if _rank() == 0:
        path.parent.mkdir(parents=True, exist_ok=True)
        tmp = path.with_suffix(".tmp")
        torch.save(trainer_payload(trainer, with_optim), tmp)
        os.replace(tmp, path)
    _barrier()
    return path if _rank() == 0 else None


def load_file(path, map_location="cpu"):
    return torch.load(path, map_location=map_location, weights_only=True)


def merge_param_groups(state, optimizer):
    """An optimizer state saved with one param group per parameter (the reference's
    generator optimizer layout, config.py:206-215, and this trainer's before round 6)
    as the single group ``optimizer`` has: parameter ids in group order, the
    hyperparameters of the first group (identical in every group there)."""
    groups = state["param_groups"]
    if len(optimizer.param_groups) != 1 or len(groups) <= 1:
        return state
    keys = {k for g in groups for k in g if k != "params"}
    for k in keys:
        if any(g.get(k) != groups[0].get(k) for g in groups):
            raise ValueError(f"g_optim: param groups differ in {k!r}; cannot merge them")
    merged = dict(groups[0], params=[i for g in groups for i in g["params"]])
    return {"state": state["state"], "param_groups": [merged]}


def load_into(trainer, ckpt):
    """Restore g / d / g_ema (and the optimizers, iteration and path-length EMA when
    the file has them) into ``trainer`` (training_utils.py:220-225)."""
    trainer.g_module.load_state_dict(ckpt["g"])
    trainer.d_module.load_state_dict(ckpt["d"])
    trainer.generator_test.load_state_dict(ckpt["g_ema"])
    if "g_optim" in ckpt:
        trainer.optimizer.load_state_dict(merge_param_groups(ckpt["g_optim"],
                                                             trainer.optimizer))
        trainer.optimizer_d.load_state_dict(ckpt["d_optim"])
    if "iteration" in ckpt:
        trainer.iteration = int(ckpt["iteration"])
    if "mean_path_length" in ckpt and hasattr(trainer, "mean_path_length"):
        trainer.mean_path_length = float(ckpt["mean_path_length"])


def resume(trainer, checkpoints_dir, expname, stage):
    """Load the stage's newest periodic checkpoint if there is one; returns the
    iteration to start from (that checkpoint's + 1, or 0)."""
    folder = exp_dir(checkpoints_dir, expname) / STAGE_DIRS[stage]
    last = agree(get_ckpt_nums(folder))
    if last is None:
        return 0
    load_into(trainer, load_file(folder / f"models_{last.zfill(7)}.pt"))
    trainer.iteration = int(last) + 1
    return trainer.iteration


def load_size_matched(module, state_dict):
    """Copy the entries of ``state_dict`` whose shape matches the module's
    (eval.py:73-77); returns the names copied."""
    own = module.state_dict()
    copied = [k for k, v in state_dict.items() if k in own and v.size() == own[k].size()]
    own.update({k: state_dict[k] for k in copied})
    module.load_state_dict(own)
    return copied


def stage_plan(checkpoints_dir, expname, wod=False):
    """(train stage 1?, train stage 2?) as train.py:69-89."""
    d = exp_dir(checkpoints_dir, expname)
    need_vol = not (d / STAGE_FINAL[1]).exists()
    need_full = not (d / STAGE_FINAL[2]).exists()
    if wod:
        need_vol, need_full = False, True
    return agree((need_vol, need_full))


def save_final(trainer, checkpoints_dir, expname, stage):
    return save(exp_dir(checkpoints_dir, expname) / STAGE_FINAL[stage], trainer, with_optim=False)


def stage1_checkpoint_due(i):
    """Stage-1 periodic checkpoints: every 10k iterations, every 1k below 10k
    (training_utils.py:525)."""
    return i % 10000 == 0 or (i < 10000 and i % 1000 == 0)


def stage2_checkpoint_due(i):
    """Stage-2 periodic checkpoints: every 10k iterations (training_utils.py:857)."""
    return i % 10000 == 0
