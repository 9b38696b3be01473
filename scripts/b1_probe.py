"""bench.py's B = 1 extras in isolation (eager step with latent + camera draws and
random decoder noise; the same replayed from GraphedGenerator.random_faces), for
per-kernel profiling.  Profiling aid.
    python scripts/b1_probe.py [steps]"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from sdfr_loader import load  # noqa: E402


def main():
    sdfr = load()
    dev = torch.device("cuda", 0)
    g, opt = bench.build_generator(sdfr, dev, 0)
    res = opt.model.renderer_spatial_output_dim
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    cam_kw = dict(azim_range=opt.camera.azim, elev_range=opt.camera.elev, fov_ang=opt.camera.fov,
                  dist_radius=opt.camera.dist_radius)

    def step(nb=1):
        z = torch.randn(nb, opt.model.style_dim, device=dev, generator=gen)
        cam, focal, near, far, _ = sdfr.generate_camera_params(res, dev, batch=nb, **cam_kw)
        with torch.no_grad():
            return g([z], cam, focal, near, far, truncation=1, truncation_latent=None)[0]

    gg = sdfr.GraphedGenerator(g)

    def graphed(nb=1):
        return gg.random_faces(nb, res, **cam_kw)[0]

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    for name, fn in (("eager", step), ("graph", graphed)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        print(f"{name}: {dt * 1e3:.3f} ms/face = {1 / dt:.0f} faces/s", flush=True)


if __name__ == "__main__":
    main()
