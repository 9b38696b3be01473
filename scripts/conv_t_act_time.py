"""The upsampling StyledConv at the bench's shapes (B = 32: 64^2 x 512 -> 128^2 x 256 and
128^2 x 256 -> 256^2 x 128): sdfr_conv_t_act (blur + epilogue in conv_t_kernel, border
kernel) against sdfr_conv3x3_f16x3 (transposed) + sdfr_styled_epilogue (blur_up),
interleaved, HIP events; checks the outputs are bit-identical.

    python scripts/conv_t_act_time.py [reps]"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    sdfr = load()
    ops = sdfr.decoder_ops
    dev = "cuda:0"
    fir = [0.25, 0.75, 0.75, 0.25]
    for (B, Cin, Cout, H) in ((32, 512, 256, 64), (32, 256, 128, 128)):
        g = torch.Generator(device=dev).manual_seed(H)
        x = torch.randn(B, Cin, H, H, device=dev, generator=g)
        w = torch.randn(Cout, Cin, 3, 3, device=dev, generator=g)
        packed, su = ops.conv_pack_weights(w, 1 / math.sqrt(Cin * 9))
        xs = ops.split_nhwc(x)
        demod = (torch.rand(B, Cout, device=dev, generator=g) + 0.5) / su
        bias = torch.randn(Cout, device=dev, generator=g) * 0.1
        nw = torch.tensor([0.3], device=dev)
        nz = torch.randn(B, 1, 2 * H, 2 * H, device=dev, generator=g)
        sn = torch.rand(B, Cout, device=dev, generator=g) + 0.5

        def fused():
            return ops.conv_t_act(xs, packed, Cout, fir=fir, demod=demod, bias=bias,
                                  noise_weight=nw, noise=nz, s_next=sn)

        def two():
            raw = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True)
            return ops.styled_epilogue(raw, fir=fir, bias=bias, noise_weight=nw, noise=nz,
                                       demod=demod, blur_up=True, s_next=sn, store_y=True,
                                       split_y=True)[0]
        a, b = fused(), two()
        torch.cuda.synchronize()
        same = torch.equal(a, b)
        t = {"fused": [], "two": []}
        for _ in range(reps):
            for name, fn in (("fused", fused), ("two", two)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                t[name].append(e0.elapsed_time(e1) * 1e3)
        med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
        print(f"B={B} {Cin}->{Cout} {H}^2->{2 * H}^2: fused {med['fused']:.1f} us, "
              f"conv+epilogue {med['two']:.1f} us, bit-identical {same}", flush=True)


if __name__ == "__main__":
    main()
