"""Median time of the decoder epilogues (sdfr_styled_epilogue) at the bench
workload's layer shapes (B=32), for each libsdfr.so given on the command line (each
in its own subprocess; profiling aid, not a test).  GB/s = algorithmic bytes moved
(conv read, y written as split fp16, rgb/skip/noise) / time.
    python scripts/epi_time.py [lib.so ...]"""
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

CHILD = r'''
import statistics, sys, torch
sys.path.insert(0, sys.argv[1])
from sdfr_loader import load
sdfr = load()
from sdface_gan_amd import decoder_ops as ops
dev = "cuda:0"; B = 32
# (C, H, blur_up, rgb, skip, store_y, next C): conv1+ToRGB, up1 blur, conv128+ToRGB, up2 blur, conv256+ToRGB(last)
LAYERS = [(512, 64, False, True, False, True), (256, 128, True, False, False, True),
          (256, 128, False, True, True, True), (128, 256, True, False, False, True),
          (128, 256, False, True, True, False)]
fir = [0.125, 0.375, 0.375, 0.125]
tot = 0.0
for C, H, blur, rgb, skip, sy in LAYERS:
    g = torch.Generator(device=dev).manual_seed(C + H)
    Hc = H + 1 if blur else H
    conv = torch.randn(B, C, Hc, Hc, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    kw = dict(fir=fir, bias=torch.randn(C, device=dev), noise_weight=torch.full((1,), 0.1, device=dev),
              noise=torch.randn(B, 1, H, H, device=dev), demod=torch.rand(B, C, device=dev),
              s_next=torch.rand(B, C, device=dev) if sy else None, store_y=sy, split_y=sy,
              blur_up=blur)
    if rgb:
        kw.update(rgb_w=torch.randn(B, 3, C, device=dev), rgb_b=torch.randn(3, device=dev),
                  skip=torch.randn(B, 3, H // 2, H // 2, device=dev) if skip else None)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for r in range(12):
        ev[0].record()
        ops.styled_epilogue(conv, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        if r >= 2: ts.append(ev[0].elapsed_time(ev[1]))
    med = statistics.median(ts)
    tot += med
    nbytes = B * C * Hc * Hc * 4 + (B * C * H * H * 4 if sy else 0) + B * H * H * 4
    if rgb: nbytes += B * 3 * H * H * 4 + (B * 3 * H * H if skip else 0)
    print(f"  C {C:4d} H {H:4d} {'blur' if blur else 'plain'} {'rgb' if rgb else '   '}  "
          f"{med*1e3:8.1f} us  {nbytes / med / 1e6:7.0f} GB/s")
print(f"  total {tot:.3f} ms")
'''


def main():
    libs = sys.argv[1:] or [str(REPO / "sdface-gan_amd" / "lib" / "libsdfr.so")]
    for lib in libs:
        env = dict(os.environ, SDFR_LIB=str(Path(lib).resolve()))
        print(lib, flush=True)
        r = subprocess.run([sys.executable, "-c", CHILD, str(REPO)], env=env)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
