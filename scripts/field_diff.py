"""Outputs of the fused renderer (the libsdfr.so SDFR_LIB names) vs the reference fixture
(render_face64 / render_small, with sdf/xyz when present): max |diff| per output, split
into segments or not (profiling aid for the field-kernel variants, not a test)."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402
from tests.test_gpu_render import make_renderer, sd_for, _inputs  # noqa: E402

sdfr = load()
gd = Path(__file__).resolve().parents[1] / "tests" / "golden"
for name, flags in (("render_small", {}), ("render_face64", dict(return_sdf=True, return_xyz=True))):
    g = np.load(gd / f"{name}.npz")
    for maxseg in (1, 0):
        ren = make_renderer(sdfr, sd_for(gd, 1.0), int(g["res"]), int(g["n_samples"]), "f16x3", **flags)
        ren.max_field_segments = maxseg
        cam, focal, near, far, lat, tr = _inputs(g)
        with torch.no_grad():
            rgb, feat, sdf, mask, xyz, _ = ren(cam, focal, near, far, styles=lat, t_rand=tr)
        out = {"rgb": rgb, "features": feat, "sdf": sdf, "xyz": xyz, "mask": mask}
        msg = []
        for k, v in out.items():
            if v is not None and k in g.files:
                d = np.abs(v.cpu().numpy().reshape(g[k].shape) - g[k])
                msg.append(f"{k} {d.max():.2e}")
        print(name, "maxseg", maxseg, " ".join(msg), flush=True)
