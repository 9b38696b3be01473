"""Median time of the fused regular convolutions (sdfr_conv3x3_f16x3_act: conv + styled
epilogue + ToRGB partials) at the three regular decoder layers of the bench workload
(B=32), for each libsdfr.so given on the command line (each in its own subprocess;
profiling aid, not a test).  Prints a hash of the outputs so variants can be compared
for bit-identity.
    python scripts/conv_act_time.py [lib.so ...]"""
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

CHILD = r'''
import hashlib, statistics, sys, torch
sys.path.insert(0, sys.argv[1])
from sdfr_loader import load
sdfr = load()
from sdface_gan_amd import decoder_ops as ops
dev = "cuda:0"; B = int(sys.argv[3])
# (Cin, Cout, H): conv1 at 64^2, conv at 128^2, conv at 256^2
LAYERS = [(256, 512, 64), (256, 256, 128), (128, 128, 256)]
reps = int(sys.argv[2])
tot = 0.0
h = hashlib.sha1()
res = []
for Cin, Cout, H in LAYERS:
    torch.manual_seed(0)
    xs = ops.split_nhwc(torch.randn(B, Cin, H, H, device=dev))
    w = torch.randn(Cout, Cin, 3, 3, device=dev)
    packed, su = ops.conv_pack_weights(w, 1.0 / (Cin * 9) ** 0.5)
    kw = dict(demod=(torch.rand(B, Cout, device=dev) + 0.5) / su, bias=torch.randn(Cout, device=dev),
              noise_weight=torch.full((1,), 0.1, device=dev), noise=torch.randn(B, 1, H, H, device=dev),
              s_next=torch.rand(B, Cout, device=dev) + 0.5, rgb_w=torch.randn(B, 3, Cout, device=dev))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for r in range(reps + 2):
        ev[0].record()
        ys, part = ops.conv3x3_f16x3_act(xs, packed, Cout, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        if r >= 2: ts.append(ev[0].elapsed_time(ev[1]))
    med = statistics.median(ts)
    tot += med
    h.update(ys.cpu().numpy().tobytes()); h.update(part.cpu().numpy().tobytes())
    fl = 2 * B * H * H * 9 * Cin * Cout
    res.append(f"{Cin}x{Cout}@{H}: {med:.3f} ms {fl / med / 1e9:.0f} TF ({3 * fl / med / 1e9:.0f} issued)")
print(f"out {h.hexdigest()[:12]} total {tot:.3f} ms | " + " | ".join(res))
'''


def main():
    libs = sys.argv[1:] or [str(REPO / "sdface-gan_amd/lib/libsdfr.so")]
    B = os.environ.get("B", "32")
    for lib in libs:
        env = dict(os.environ, SDFR_LIB=str(REPO / lib) if not lib.startswith("/") else lib)
        out = subprocess.run([sys.executable, "-c", CHILD, str(REPO), "10", B], env=env,
                             capture_output=True, text=True, timeout=300)
        res = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else \
            f"FAILED rc={out.returncode}: {out.stderr.strip().splitlines()[-3:]}"
        print(f"{lib:48s} {res}", flush=True)


if __name__ == "__main__":
    main()
