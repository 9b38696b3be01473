"""Option groups consumed by Generator / VolumeFeatureRenderer.

Same groups, names and defaults as ``SDFOptions`` (sdf_utils.py:447-594) and the
fix-ups of ``get_vol_render_opt`` (training_utils.py:144-193), on plain
argparse (configargparse / munch are not dependencies here).
"""
from __future__ import annotations

import argparse


class AttrDict(dict):
    """dict with attribute access (the reference uses munch.Munch)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def copy(self):
        return AttrDict(self)


_GROUPS = {
    "dataset": [("--dataset_path", str, "./data/ffhq")],
    "experiment": [("--expname", str, "ffhq1024x1024"), ("--ckpt", str, "300000"),
                   ("--continue_training", bool, False)],
    "training": [("--checkpoints_dir", str, "./out"), ("--iter", int, 300000),
                 ("--batch", int, 4), ("--chunk", int, 1), ("--val_n_sample", int, 8),
                 ("--d_reg_every", int, 16), ("--g_reg_every", int, 4),
                 ("--local_rank", int, 0), ("--mixing", float, 0.9), ("--lr", float, 0.002),
                 ("--r1", float, 10), ("--view_lambda", float, 15),
                 ("--eikonal_lambda", float, 0.1), ("--min_surf_lambda", float, 0.05),
                 ("--min_surf_beta", float, 100.0), ("--path_regularize", float, 2),
                 ("--path_batch_shrink", int, 2), ("--wandb", bool, False),
                 ("--no_sphere_init", bool, False)],
    "inference": [("--results_dir", str, "./evaluations"), ("--truncation_ratio", float, 0.5),
                  ("--truncation_mean", int, 10000), ("--identities", int, 16),
                  ("--num_views_per_id", int, 1), ("--no_surface_renderings", bool, False),
                  ("--fixed_camera_angles", bool, False), ("--azim_video", bool, False)],
    "model": [("--size", int, 256), ("--style_dim", int, 256),
              ("--channel_multiplier", int, 2), ("--n_mlp", int, 8),
              ("--lr_mapping", float, 0.01), ("--renderer_spatial_output_dim", int, 64),
              ("--project_noise", bool, False)],
    "camera": [("--uniform", bool, False), ("--azim", float, 0.3), ("--elev", float, 0.15),
               ("--fov", float, 6), ("--dist_radius", float, 0.12)],
    "rendering": [("--depth", int, 8), ("--width", int, 256), ("--no_sdf", bool, False),
                  ("--no_z_normalize", bool, False), ("--static_viewdirs", bool, False),
                  ("--N_samples", int, 24), ("--no_offset_sampling", bool, False),
                  ("--perturb", float, 1.), ("--raw_noise_std", float, 0.),
                  ("--force_background", bool, False), ("--return_xyz", bool, False),
                  ("--return_sdf", bool, False)],
}


class SDFOptions:
    def __init__(self):
        self.parser = argparse.ArgumentParser(add_help=False)
        self._groups = {}
        for title, args in _GROUPS.items():
            g = self.parser.add_argument_group(title)
            self._groups[title] = [a[0].lstrip("-") for a in args]
            for flag, typ, default in args:
                if typ is bool:
                    g.add_argument(flag, action="store_true")
                else:
                    g.add_argument(flag, type=typ, default=default)

    def parse(self, input=()):
        args = self.parser.parse_args(list(input))
        opt = AttrDict()
        for title, names in self._groups.items():
            opt[title] = AttrDict({n: getattr(args, n) for n in names})
        return opt


def vol_render_opt(ngp=True, fc=False, train_renderer=False, size=256, batch=8, chunk=2,
                   extra=()):
    """get_vol_render_opt (training_utils.py:144-193) without its side effects."""
    opt = SDFOptions().parse(["--size", str(size), "--batch", str(batch), "--chunk", str(chunk)]
                             + list(extra))
    if train_renderer:
        opt.model.freeze_renderer = False
        opt.model.no_viewpoint_loss = opt.training.view_lambda == 0.0
        opt.training.camera = opt.camera
        opt.training.renderer_output_size = opt.model.renderer_spatial_output_dim
        opt.training.style_dim = opt.model.style_dim
        opt.training.with_sdf = not opt.rendering.no_sdf
        if opt.training.with_sdf and opt.training.min_surf_lambda > 0:
            opt.rendering.return_sdf = True
        opt.training.iter = 200001
        opt.rendering.no_features_output = True
    else:
        opt.training.camera = opt.camera
        opt.training.size = opt.model.size
        opt.training.renderer_output_size = opt.model.renderer_spatial_output_dim
        opt.training.style_dim = opt.model.style_dim
        opt.model.freeze_renderer = True
        opt.model.no_viewpoint_loss = opt.training.view_lambda == 0.0
    opt.training.distributed = False
    opt.training.start_iter = 0
    opt.rendering.type = "ngp" if ngp else "sdf"
    opt.rendering.fc = int(fc)
    opt.model.psp = 0
    return opt
