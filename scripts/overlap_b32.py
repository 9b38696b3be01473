"""Eager Generator.forward at B faces (bench.py's step) with and without the decoder
prep on a side stream beside the renderer (Generator.overlap_decoder_prep), interleaved
(profiling aid, not a test).   python scripts/overlap_b32.py [B]"""
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(B=32, reps=6, n=20):
    sdfr = load()
    dev = torch.device("cuda", 0)
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    g.renderer.rng_device = "device"
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)

    def step():
        z = torch.randn(B, 256, device=dev, generator=gen)
        cam, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
        with torch.no_grad():
            return g([z], cam, focal, near, far)[0]
    res = {}
    for ov in (False, True) * 2:
        g.overlap_decoder_prep = ov
        for _ in range(3):
            step()
    for _ in range(reps):
        for ov in (False, True):
            g.overlap_decoder_prep = ov
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                step()
            torch.cuda.synchronize()
            res.setdefault(ov, []).append(B * n / (time.perf_counter() - t0))
    for ov, v in res.items():
        print(f"B={B} overlap_decoder_prep={ov}: median {statistics.median(v):.1f} faces/s  "
              f"({', '.join(f'{x:.0f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 32)
