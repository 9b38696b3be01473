"""Run only the fused StyleGAN2 decoder (B faces, 64^2 features -> 256^2) K times:
a short target for rocprofv3 counter passes on the conv kernels (profiling aid)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(B=32, K=3):
    sdfr = load()
    dev = "cuda:0"
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    feats = torch.randn(B, 256, 64, 64, device=dev) * 0.3
    with torch.no_grad():
        lat = g.style(torch.randn(B, 256, device=dev))
        for _ in range(K):
            g.decoder(feats, [lat])
    torch.cuda.synchronize()
    print("decoder_only done", flush=True)


if __name__ == "__main__":
    main()
