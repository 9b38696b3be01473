"""A/B of the decoder prep overlap (Generator.overlap_decoder_prep) in ONE process:
bench.py's step at B = 32, the two settings interleaved over several rounds, per
setting the median ms per step and the renderer's stage times (hash grid, field)
from the library's HIP events.  Prints one JSON line."""
import json
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from sdfr_loader import load  # noqa: E402


def main(rounds=6, steps=20, B=32):
    sdfr = load()
    dev = torch.device("cuda", 0)
    g, opt = bench.build_generator(sdfr, dev, 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000)
    res, N = opt.model.renderer_spatial_output_dim, opt.rendering.N_samples

    def step():
        z = torch.randn(B, 256, device=dev, generator=gen)
        cam, focal, near, far, _ = sdfr.generate_camera_params(
            res, dev, batch=B, azim_range=opt.camera.azim, elev_range=opt.camera.elev,
            fov_ang=opt.camera.fov, dist_radius=opt.camera.dist_radius)
        with torch.no_grad():
            return g([z], cam, focal, near, far)[0]
    out = {True: [], False: []}
    for r in range(rounds):
        for ov in (True, False) if r % 2 == 0 else (False, True):
            g.overlap_decoder_prep = ov
            for _ in range(3):
                step()
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
            for e4 in evs:
                for e in e4:
                    e.record()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                g.renderer.stage_events = evs[k]
                step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps * 1e3
            g.renderer.stage_events = None
            enc = sum(e[1].elapsed_time(e[2]) for e in evs) / steps
            fld = sum(e[2].elapsed_time(e[3]) for e in evs) / steps
            out[ov].append((dt, enc, fld))
    rec = {}
    for ov, v in out.items():
        rec["overlap" if ov else "in_order"] = {
            "ms_per_step_median": statistics.median(x[0] for x in v),
            "encode_ms_median": statistics.median(x[1] for x in v),
            "field_ms_median": statistics.median(x[2] for x in v),
            "ms_per_step_all": [round(x[0], 3) for x in v]}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
