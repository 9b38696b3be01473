"""B = 1 graphed generation (GraphedGenerator.random_faces, eval.py's loop body) with the
field kernel's split feature store on (feature_split_min_batch 1: the merge kernel
writes the decoder's split-NHWC input) and off (4: NCHW features + modulate_nhwc),
interleaved; prints faces/s medians (profiling aid, not a test)."""
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(reps=7, n=200):
    sdfr = load()
    dev = torch.device("cuda", 0)
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    g.renderer.rng_device = "device"
    ggs = {}
    for m in (4, 1):
        g.feature_split_min_batch = m
        gg = sdfr.GraphedGenerator(g)
        gg.random_faces(1, 64)
        ggs[m] = gg
    res = {}
    for _ in range(reps):
        for m, gg in ggs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                gg.random_faces(1, 64)
            torch.cuda.synchronize()
            res.setdefault(m, []).append(n / (time.perf_counter() - t0))
    for m, v in res.items():
        print(f"feature_split_min_batch={m}: median {statistics.median(v):.1f} faces/s "
              f"({', '.join(f'{x:.0f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
