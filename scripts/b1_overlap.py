"""Batch-1 graphed generator (GraphedGenerator.random_faces, eval.py's call) with and
without the decoder prep on a side stream (Generator.overlap_decoder_prep), interleaved,
many replays per sample (profiling aid, not a test).
    python scripts/b1_overlap.py [B]"""
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(B=1, reps=5, n=200):
    sdfr = load()
    dev = torch.device("cuda", 0)
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    g.renderer.rng_device = "device"
    res = {}
    graphs = {}
    for ov in (False, True):
        g.overlap_decoder_prep = ov
        graphs[ov] = sdfr.GraphedGenerator(g)
        for _ in range(5):
            graphs[ov].random_faces(B, 64)
    torch.cuda.synchronize()
    for _ in range(reps):
        for ov in (False, True):
            gg = graphs[ov]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                gg.random_faces(B, 64)
            torch.cuda.synchronize()
            res.setdefault(ov, []).append(B * n / (time.perf_counter() - t0))
    for ov, v in res.items():
        print(f"B={B} overlap_decoder_prep={ov}: median {statistics.median(v):.1f} faces/s  "
              f"({', '.join(f'{x:.0f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
