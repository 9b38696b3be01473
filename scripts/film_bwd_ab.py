"""A/B of the FiLM backward kernels (sdfr_film_backward / sdfr_film_backward_grad) across
library builds: per build (SDFR_LIB, one subprocess each) an exact hash of every output
on seeded SIREN stage-1 shapes (2 faces x 64^2 x 24 rows, 256 columns) and the median
time per call.  Profiling aid; the hashes of builds that claim bit-identity must agree.
    python scripts/film_bwd_ab.py <lib.so> [<lib.so> ...]"""
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
from sdface_gan_amd.linear import _film_bwd, _film_bwd2
dev = "cuda:0"; F_, R, N = 2, 4096 * 24, 256
g = torch.Generator(device=dev).manual_seed(0)
ds = torch.randn(F_ * R, N, device=dev, generator=g)
y = torch.randn(F_ * R, N, device=dev, generator=g) * 0.05
gm = 30 + 3 * torch.randn(F_, N, device=dev, generator=g)
bt = 0.25 * torch.randn(F_, N, device=dev, generator=g)
gdy = torch.randn(F_ * R, N, device=dev, generator=g)
gdg = torch.randn(F_, N, device=dev, generator=g)
gdb = torch.randn(F_, N, device=dev, generator=g)
def h(ts):
    v = torch.cat([t.reshape(-1).view(torch.int32).to(torch.int64) for t in ts])
    w = torch.arange(v.numel(), device=dev, dtype=torch.int64) % 9973 + 1
    return int(((v * w) % (1 << 61)).sum())
def med(fn, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(n):
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts[3:])
o1 = _film_bwd(ds, y, gm, bt); o2 = _film_bwd2(ds, y, gm, bt, gdy, gdg, gdb)
torch.cuda.synchronize()
t1 = med(lambda: _film_bwd(ds, y, gm, bt))
t2 = med(lambda: _film_bwd2(ds, y, gm, bt, gdy, gdg, gdb))
print(f"film_bwd {t1:.1f} us ({3 * F_ * R * N * 4 / t1 / 1e6:.2f} TB/s) hash {h(o1)}  "
      f"film_bwd2 {t2:.1f} us ({5 * F_ * R * N * 4 / t2 / 1e6:.2f} TB/s) hash {h(o2)}")
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
