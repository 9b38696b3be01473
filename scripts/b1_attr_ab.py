"""B = 1 graphed generation (GraphedGenerator.random_faces, eval.py's loop body) under two
values of one Generator attribute (each captured into its own graph), interleaved;
prints faces/s medians (profiling aid, not a test).
    python scripts/b1_attr_ab.py overlap_decoder_prep True False"""
import ast
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(attr, values, reps=7, n=200):
    sdfr = load()
    dev = torch.device("cuda", 0)
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    g.renderer.rng_device = "device"
    obj, name = g, attr
    while "." in name:
        head, name = name.split(".", 1)
        obj = getattr(obj, head)
    ggs = {}
    for v in values:
        setattr(obj, name, v)
        gg = sdfr.GraphedGenerator(g)
        gg.random_faces(1, 64)
        ggs[repr(v)] = gg
    res = {}
    for _ in range(reps):
        for k, gg in ggs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                gg.random_faces(1, 64)
            torch.cuda.synchronize()
            res.setdefault(k, []).append(n / (time.perf_counter() - t0))
    for k, v in res.items():
        print(f"{attr}={k}: median {statistics.median(v):.1f} faces/s "
              f"({', '.join(f'{x:.0f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], [ast.literal_eval(a) for a in sys.argv[2:]])
