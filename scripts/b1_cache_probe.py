"""Batch-1 rate of the plain Generator.forward call (its own graph cache) against
GraphedGenerator, in a fresh process and after bench.py's B = 32 steps, with and without
the Python garbage collector's generations frozen: which process state makes the plain
call slower than the wrapper in bench.py's extras (profiling aid).

    python scripts/b1_cache_probe.py
"""
import gc
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    from sdfr_loader import load
    sdfr = load()
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    g, opt = bench.build_generator(sdfr, dev, seed=0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000)

    res = opt.model.renderer_spatial_output_dim

    def step(nb):
        z = torch.randn(nb, opt.model.style_dim, device=dev, generator=gen)
        cam, focal, near, far, _ = sdfr.generate_camera_params(
            res, dev, batch=nb, azim_range=opt.camera.azim, elev_range=opt.camera.elev,
            fov_ang=opt.camera.fov, dist_radius=opt.camera.dist_radius)
        with torch.no_grad():
            rgb, _ = g([z], cam, focal, near, far, truncation=1, truncation_latent=None)
        return rgb

    gg = sdfr.GraphedGenerator(g)

    def graphed(nb):
        return gg.random_faces(nb, res, azim_range=opt.camera.azim, elev_range=opt.camera.elev,
                               fov_ang=opt.camera.fov, dist_radius=opt.camera.dist_radius)[0]

    def rate(fn, n=600, warm=5):
        for _ in range(warm):
            fn(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn(1)
        torch.cuda.synchronize()
        return n / (time.perf_counter() - t0)

    def line(tag):
        print(f"{tag:28s} plain {rate(step):7.1f}  graphed {rate(graphed):7.1f}  "
              f"plain {rate(step):7.1f}", flush=True)

    line("fresh process")
    for _ in range(25):
        step(32)
    torch.cuda.synchronize()
    line("after 25 B=32 steps")
    gc.collect()
    gc.freeze()
    line("gc frozen")
    gc.unfreeze()
    gc.disable()
    line("gc disabled")
    gc.enable()
    g.renderer.stage_events = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    g.renderer.stage_events = None
    line("again")


if __name__ == "__main__":
    main()
