"""Can Generator.forward (fused renderer + fused decoder) be captured in a HIP
graph, and what does replay buy at eval.py's batch of 1?  Profiling aid.
    python scripts/graph_probe.py [B ...]"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main():
    sdfr = load()
    dev = torch.device("cuda", 0)
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    for B in [int(b) for b in sys.argv[1:]] or [1, 8]:
        z = torch.randn(B, 256, device=dev)
        cam, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
        tr = torch.rand(B, 64, 64, device=dev)

        def fwd():
            with torch.no_grad():
                return g([z], cam, focal, near, far, t_rand=tr, randomize_noise=False)[0]

        ref = fwd().clone()
        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            fwd()
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / 20
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                fwd()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = fwd()
        graph.replay()
        torch.cuda.synchronize()
        same = bool(torch.equal(out, ref))
        t0 = time.perf_counter()
        for _ in range(20):
            graph.replay()
        torch.cuda.synchronize()
        rep = (time.perf_counter() - t0) / 20
        print(json.dumps({"B": B, "eager_ms": eager * 1e3, "graph_ms": rep * 1e3,
                          "eager_faces_s": B / eager, "graph_faces_s": B / rep,
                          "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
