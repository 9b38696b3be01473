"""upfirdn2d (sdfr_upfirdn2d) timing at the stage-2 discriminator / decoder-training
shapes: forward and its gradient op, HIP events, algorithmic bytes (input + output,
fp32) per call -> GB/s.

    python scripts/ufd_time.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main():
    sdfr = load()
    ops = sdfr.decoder_ops
    dev = "cuda:0"
    f = torch.tensor([1.0, 3.0, 3.0, 1.0], device=dev)
    k = torch.outer(f, f)
    k = k / k.sum()
    cases = [("D blur 256^2 x128 pad(2,2)", (2, 128, 256, 256), 1, 1, (2, 2)),
             ("D skip blur 256^2 x128 pad(1,1)", (2, 128, 256, 256), 1, 1, (1, 1)),
             ("D blur 128^2 x256", (2, 256, 128, 128), 1, 1, (2, 2)),
             ("D blur 64^2 x512", (2, 512, 64, 64), 1, 1, (2, 2)),
             ("dec conv_t blur 257^2 x128 pad(1,1)", (2, 128, 257, 257), 1, 1, (1, 1)),
             ("ToRGB upsample 128^2 x3", (2, 3, 128, 128), 2, 1, (2, 1)),
             ("ToRGB upsample grad (down 2)", (2, 3, 259, 259), 1, 2, (2, 2))]
    for name, shape, up, down, pad in cases:
        x = torch.randn(*shape, device=dev)
        kk = k * up * up
        for _ in range(3):
            y = ops.upfirdn2d(x, kk, up=up, down=down, pad=pad)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            y = ops.upfirdn2d(x, kk, up=up, down=down, pad=pad)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        nbytes = 4 * (x.numel() + y.numel())
        print(f"{name:40s} {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
