"""Run only the fused renderer (B faces, 64^2 x 24) K times: a short, clean target
for rocprofv3 counter passes on the field kernel (profiling aid, not a test).
    python scripts/render_only.py [f16x3|fp32] [ngp|siren|fc]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(B=32, K=3, precision="f16x3", net="ngp"):
    sdfr = load()
    dev = "cuda:0"
    opt = sdfr.vol_render_opt(ngp=net == "ngp", fc=net == "fc")
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    ren = g.renderer
    ren.rng_device = "device"
    ren.field_precision = precision
    ext, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
    with torch.no_grad():
        lat = g.style(torch.randn(B, 256, device=dev))
        for _ in range(K):
            ren(ext, focal, near, far, styles=lat)
    torch.cuda.synchronize()
    print("render_only done", flush=True)


if __name__ == "__main__":
    main(precision=sys.argv[1] if len(sys.argv) > 1 else "f16x3",
         net=sys.argv[2] if len(sys.argv) > 2 else "ngp")
