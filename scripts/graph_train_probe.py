"""Probe: can a stage-2 chunk (G half-step forward + backward, D half-step without R1)
be captured as a HIP graph on this stack (MIOpen convolutions, the fused renderer, our
ctypes ops), and what does a replay cost against the eager chunk?

    python scripts/graph_train_probe.py
"""
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    sdfr = load()
    from sdface_gan_amd import training as T
    opt = sdfr.vol_render_opt(ngp=True)
    tr = T.FullPipelineTrainer(opt, dev, seed=0)
    tr.g_module.renderer.rng_device = "device"
    torch.manual_seed(1)
    real = torch.rand(8, 3, 256, 256, device=dev) * 2 - 1
    for _ in range(2):
        tr.step(real)
    torch.cuda.synchronize()
    G, D = tr.g_module, tr.d_module
    sd = opt.model.style_dim

    # static inputs of one chunk of 2
    z = torch.randn(2, sd, device=dev)
    cam, focal, near, far, _ = tr._cams(2)
    real2 = real[:2].clone()

    def g_chunk():
        img, thumb = G([z], cam, focal, near, far, randomize_noise=True)
        up = F.interpolate(thumb, scale_factor=4)
        loss = T.g_nonsaturating_loss(D(img)) + 0.001 * T.g_content_loss(img, up)
        loss.backward()
        return loss

    def d_chunk():
        with torch.no_grad():
            img, _ = G([z], cam, focal, near, far, randomize_noise=True)
        loss = T.d_logistic_loss(D(real2), D(img))
        loss.backward()
        return loss

    def prep(which):
        g_on = which == "g"
        T.requires_grad(tr.g_train, g_on)
        T.requires_grad(D.parameters(), not g_on)
        for p in (tr.g_train if g_on else D.parameters()):
            if p.grad is None:
                p.grad = torch.zeros_like(p)

    def eager_time(fn, n=6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        return th / n * 1e3, (time.perf_counter() - t0) / n * 1e3

    for which, fn in (("g", g_chunk), ("d", d_chunk)):
        prep(which)
        h, w = eager_time(fn)
        print(f"[{which}] eager chunk: host {h:.2f} ms, wall {w:.2f} ms", flush=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                out = fn()
        except Exception as e:                      # noqa: BLE001  (a probe: report it)
            print(f"[{which}] capture FAILED: {type(e).__name__}: {str(e)[:400]}", flush=True)
            torch.cuda.synchronize()
            continue
        torch.cuda.synchronize()
        h, w = eager_time(g.replay, 10)
        print(f"[{which}] graph replay: host {h:.2f} ms, wall {w:.2f} ms, loss {float(out):.4f}",
              flush=True)


if __name__ == "__main__":
    main()
