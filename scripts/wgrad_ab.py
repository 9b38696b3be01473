"""A/B of the weight-gradient GEMM (sdfr_linear_wgrad_f16x3) across library builds: per
build (SDFR_LIB, one subprocess each) an exact hash of gW and the median time per call on
the stage-1 shapes (M = 2 faces x 64^2 x 24 rows; N = 256; K = 256, 272, 260, 32) with
per-column magnitudes spread over 2^-20 .. 2^4 (the running column scales change often).
Profiling aid; builds that claim bit-identity must print the same hashes.
    python scripts/wgrad_ab.py <lib.so> [<lib.so> ...]"""
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

CHILD = r'''
import statistics, sys, torch
sys.path.insert(0, sys.argv[1])
from sdfr_loader import load
load()
from sdface_gan_amd.linear import _wgrad
dev = "cuda:0"; M, N = 2 * 4096 * 24, 256
g = torch.Generator(device=dev).manual_seed(0)
def spread(rows, cols):
    t = torch.randn(rows, cols, device=dev, generator=g)
    e = torch.randint(-20, 5, (rows // 4096 + 1, cols), device=dev, generator=g).float()
    return t * torch.exp2(e).repeat_interleave(4096, 0)[:rows]
gy = spread(M, N)
out = []
for K in (256, 272, 260, 32):
    x = spread(M, K)
    w = _wgrad(gy, x); torch.cuda.synchronize()
    v = w.reshape(-1).view(torch.int32).to(torch.int64)
    hsh = int(((v * (torch.arange(v.numel(), device=dev) % 9973 + 1)) % (1 << 61)).sum())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(15):
        e0.record(); _wgrad(gy, x); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    t = statistics.median(ts[3:])
    out.append(f"K={K}: {t:.1f} us ({M * (N + K) * 4 / t / 1e6:.2f} TB/s) hash {hsh}")
print("  |  ".join(out))
'''


def main():
    for lib in sys.argv[1:]:
        env = dict(os.environ, SDFR_LIB=str(Path(lib).resolve()))
        r = subprocess.run([sys.executable, "-c", CHILD, str(REPO)], env=env,
                           capture_output=True, text=True, timeout=300)
        out = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-800:]
        print(f"{lib}: {out}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
