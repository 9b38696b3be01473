"""Decoder layer timings on the GPU (profiling aid, not a test).

Times each StyleGAN2 decoder convolution of the ffhq 256 config at B faces in
NCHW and channels_last, with MIOpen heuristics (benchmark=False) and with
MIOpen find (benchmark=True), plus the whole Decoder.forward.
"""
import json
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(iters):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2]


def main(B=32):
    sdfr = load()
    dev = "cuda:0"
    out = {}
    # (name, cin, cout, H, transpose)
    convs = [("conv1_64", 256, 512, 64, False), ("up_64to128", 512, 256, 64, True),
             ("conv_128", 256, 256, 128, False), ("up_128to256", 256, 128, 128, True),
             ("conv_256", 128, 128, 256, False)]
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        for name, cin, cout, H, tr in convs:
            x = torch.randn(B, cin, H, H, device=dev)
            w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
            for layout in ("nchw", "nhwc"):
                xx = x.contiguous(memory_format=torch.channels_last) if layout == "nhwc" else x
                ww = (w.transpose(0, 1).contiguous() if tr else w)
                if layout == "nhwc":
                    ww = ww.contiguous(memory_format=torch.channels_last)
                if tr:
                    fn = lambda: F.conv_transpose2d(xx, ww, stride=2)  # noqa: E731
                else:
                    fn = lambda: F.conv2d(xx, ww, padding=1)  # noqa: E731
                ms = timeit(fn)
                flop = 2 * B * H * H * cin * cout * 9
                key = f"{name}/{layout}/bench={int(bench)}"
                out[key] = {"ms": ms, "tflops": flop / ms / 1e9}
                print(f"{key:36s} {ms:8.3f} ms {flop / ms / 1e9:7.1f} TFLOP/s", flush=True)
            del x, w
    torch.backends.cudnn.benchmark = False

    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    feats = torch.randn(B, 256, 64, 64, device=dev)
    lat = [torch.randn(B, 256, device=dev)]
    with torch.no_grad():
        for bench in (False, True):
            torch.backends.cudnn.benchmark = bench
            ms = timeit(lambda: g.decoder(feats, lat))
            out[f"decoder/bench={int(bench)}"] = ms
            print(f"decoder forward bench={int(bench)}: {ms:.3f} ms", flush=True)
    Path("gpurun_out").mkdir(exist_ok=True)
    Path("gpurun_out/decoder_bench.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"done in {time.time() - t:.1f}s")
