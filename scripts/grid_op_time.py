"""Drop-in hash-grid op (GridEncoder / sdfr_grid_encode_{forward,backward}, the
reference's _grid_encode interface, grid.py:27-89) at the fused path's sample
count: median ms of forward, forward with dy_dx (requires_grad inputs, the
eikonal case) and backward, per libsdfr.so given (SDFR_LIB per subprocess), with
an exact checksum of the outputs.  Profiling aid, not a test.
    [S=samples] [ORDER=uniform|tile] python scripts/grid_op_time.py [lib.so ...]
ORDER=tile feeds the renderer's own sample points in its tile order."""
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
dev = "cuda:0"
torch.manual_seed(0)
enc = sdfr.GridEncoder(desired_resolution=4096).to(dev)
with torch.no_grad():
    enc.embeddings.uniform_(-1, 1)
S = int(sys.argv[2])
if sys.argv[3] == "tile":
    # the fused renderer's samples in its tile order (16 rays of a row x N depths),
    # S // (64*64*24) faces: pts = o + d z, normalised by 2 / (far - near)
    nb, res, N = max(1, S // (64 * 64 * 24)), 64, 24
    ext, focal, near, far, _ = sdfr.generate_camera_params(res, dev, batch=nb)
    c = torch.arange(res, device=dev, dtype=torch.float32) + 0.5
    yy, xx = torch.meshgrid(c, c, indexing="ij")
    f = focal.view(nb, 1, 1)
    dirs = torch.stack([(xx - res / 2) / f, -(yy - res / 2) / f, -torch.ones_like(xx / f)], -1)
    d = torch.einsum("bhwj,bkj->bhwk", dirs, ext[:, :, :3]).reshape(nb, res * res, 1, 3)
    o = ext[:, :, 3].view(nb, 1, 1, 3)
    t = (torch.arange(N, device=dev) + torch.rand(nb, res * res, N, device=dev)) / N
    z = (near.view(nb, 1, 1) * (1 - t) + far.view(nb, 1, 1) * t)[..., None]
    pts = (o + d * z) * 2 / (far - near).view(nb, 1, 1, 1)
    x = pts.view(nb, res * res // 16, 16, N, 3).permute(0, 1, 3, 2, 4).reshape(-1, 3).contiguous()
    S = x.shape[0]
else:
    x = (torch.rand(S, 3, device=dev) * 1.1 - 0.55)   # normalised points, uniform
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
def t(fn, reps=5):
    ts = []
    for r in range(reps + 2):
        e0.record(); out = fn(); e1.record(); torch.cuda.synchronize()
        if r >= 2: ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), out
with torch.no_grad():
    f_ms, y = t(lambda: enc(x, bound=2))
xr = x.clone().requires_grad_(True)
d_ms, yd = t(lambda: enc(xr, bound=2))
g = torch.randn_like(yd)
b_ms, _ = t(lambda: torch.autograd.grad(yd, [xr, enc.embeddings], g, retain_graph=True))
gx, ge = torch.autograd.grad(yd, [xr, enc.embeddings], g)
ck = lambda v: int(v.contiguous().view(torch.int32).to(torch.int64).sum())
print(f"fwd {f_ms:.3f} ms ({1024 * S / f_ms / 1e6:.0f} GB/s alg)  fwd+dy_dx {d_ms:.3f} ms  "
      f"bwd {b_ms:.3f} ms  ck={ck(y)},{ck(yd)},{ck(gx)}")
'''


def main():
    libs = sys.argv[1:] or ["sdface-gan_amd/lib/libsdfr.so"]
    S = os.environ.get("S", str(32 * 4096 * 24))
    for lib in libs:
        env = dict(os.environ, SDFR_LIB=str(REPO / lib) if not lib.startswith("/") else lib)
        r = subprocess.run([sys.executable, "-c", CHILD, str(REPO), S,
                            os.environ.get("ORDER", "uniform")], env=env,
                           capture_output=True, text=True, timeout=300)
        out = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else \
            f"FAILED rc={r.returncode}: {r.stderr.strip()[-600:]}"
        print(f"{lib}: {out}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
