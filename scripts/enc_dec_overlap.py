"""Probe: does the hash-grid encode of the next batch (TA/L2-bound, 48 VGPRs, no LDS) run
beside the decoder's convolutions (conv_h_kernel leaves 80 VGPRs per SIMD lane free)?
Times n decoders alone, n encodes alone, and both on two streams (the encode's stream
waiting on an event recorded just before each decoder, or enqueued first), B = 32
(profiling aid, not a test).   python scripts/enc_dec_overlap.py"""
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(B=32, n=10, reps=5):
    sdfr = load()
    dev = torch.device("cuda", 0)
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    with torch.no_grad():
        g.renderer.network.encoder.embeddings.uniform_(-1, 1)
    ren = g.renderer
    ren.rng_device = "device"
    ext, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
    tr = torch.rand(B, 64, 64, device=dev)
    feats = torch.randn(B, 256, 64, 64, device=dev) * 0.3
    side = torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream(dev)
    with torch.no_grad():
        lat = g.style(torch.randn(B, 256, device=dev))
        rlat = lat

        def dec():
            g.decoder(feats, [lat])

        def enc():
            ren.fused_forward(ext, focal, near, far, rlat, t_rand=tr, encode_only=True)

        def both_event():
            for _ in range(n):
                e = torch.cuda.Event()
                e.record(main_s)
                side.wait_event(e)
                with torch.cuda.stream(side):
                    enc()
                dec()
            main_s.wait_stream(side)

        def both_first():
            for _ in range(n):
                e = torch.cuda.Event()
                e.record(main_s)
                side.wait_event(e)
                with torch.cuda.stream(side):
                    enc()
                e2 = torch.cuda.Event()
                e2.record(side)
                dec()
                main_s.wait_event(e2)

        def serial():
            for _ in range(n):
                enc()
                dec()

        def only(f):
            def run():
                for _ in range(n):
                    f()
            return run

        cases = {"decoder": only(dec), "encode": only(enc), "serial": serial,
                 "overlap(event)": both_event, "overlap(enc first, joined)": both_first}
        for f in cases.values():
            f()
        torch.cuda.synchronize()
        res = {}
        for _ in range(reps):
            for k, f in cases.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(main_s)
                f()
                e1.record(main_s)
                torch.cuda.synchronize()
                res.setdefault(k, []).append(e0.elapsed_time(e1) / n)
    for k, v in res.items():
        print(f"{k:28s} median {statistics.median(v):.3f} ms per batch  "
              f"({', '.join(f'{x:.3f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
