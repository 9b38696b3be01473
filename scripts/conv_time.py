"""Median time of the split-fp16 decoder convolution (conv_x_kernel) at every decoder
layer shape of the bench workload (B=32, 64^2 -> 256^2), for each libsdfr.so given on
the command line (each in its own subprocess; profiling aid, not a test).
    python scripts/conv_time.py [lib.so ...]        (default: the in-tree library)
TFLOP/s columns: fp32-equivalent useful rate, and issued fp16 MFMA rate (x3)."""
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
import os
dev = "cuda:0"; B = int(os.environ.get("B", "32"))
# (Cin, Cout, H_in, transposed): conv1, up 64->128, conv 128, up 128->256, conv 256
LAYERS = [(256, 512, 64, False), (512, 256, 64, True), (256, 256, 128, False),
          (256, 128, 128, True), (128, 128, 256, False)]
reps = int(sys.argv[2])
tot = 0.0
for Cin, Cout, H, tr in LAYERS:
    torch.manual_seed(0)
    x = torch.randn(B, Cin, H, H, device=dev)
    xs = ops.split_nhwc(x)
    w = torch.randn(Cout, Cin, 3, 3, device=dev)
    packed, su = ops.conv_pack_weights(w, 1.0 / (Cin * 9) ** 0.5)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for r in range(reps + 2):
        ev[0].record()
        ops.conv3x3_f16x3(xs, packed, Cout, transposed=tr, split_k=True)
        ev[1].record()
        torch.cuda.synchronize()
        if r >= 2: ts.append(ev[0].elapsed_time(ev[1]))
    med = statistics.median(ts)
    tot += med
    fl = 2.0 * B * H * H * 9 * Cin * Cout
    print(f"  Cin {Cin:4d} Cout {Cout:4d} H {H:4d} {'T' if tr else ' '}  {med*1e3:8.1f} us  "
          f"{fl / med / 1e9:7.1f} TF useful  {3 * fl / med / 1e9:7.1f} TF issued "
          f"({3 * fl / med / 1e9 / 2500 * 100:4.1f}% of 2.5 PF)")
print(f"  total {tot:.3f} ms")
'''


def main():
    reps = os.environ.get("REPS", "10")
    libs = sys.argv[1:] or [str(REPO / "sdface-gan_amd" / "lib" / "libsdfr.so")]
    for lib in libs:
        env = dict(os.environ, SDFR_LIB=str(Path(lib).resolve()))
        print(lib, flush=True)
        r = subprocess.run([sys.executable, "-c", CHILD, str(REPO), reps], env=env)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
