"""Hash-grid encode stage: median time per launch (32 faces, or SDFR_ENC_B faces) and an
exact checksum of its [L][S][2] output, for each ngp_encode_kernel mode (SDFR_ENC_MODE, one
subprocess per mode).  Profiling aid, not a test; the checksums of all modes must
agree (the modes change scheduling and load width, never arithmetic).
    [SDFR_ENC_B=<faces>] python scripts/encode_time.py [modes...]"""
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
import os
dev = "cuda:0"; B = int(os.environ.get("SDFR_ENC_B", "32"))
opt = sdfr.vol_render_opt()
torch.manual_seed(0)
g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
with torch.no_grad():   # table amplitude of a trained model, not the 1e-4 init
    g.renderer.network.encoder.embeddings.uniform_(-1, 1)
ren = g.renderer; ren.rng_device = "device"
ext, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
tr = torch.rand(B, 64, 64, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
with torch.no_grad():
    lat = g.style(torch.randn(B, 256, device=dev))
    for r in range(7):   # 10 back-to-back launches per event pair: host overhead hidden
        e0.record()
        for _ in range(10):
            ws = ren.fused_forward(ext, focal, near, far, lat, t_rand=tr, encode_only=True)
        e1.record(); torch.cuda.synchronize()
        if r >= 2: ts.append(e0.elapsed_time(e1) / 10)
S = B * 4096 * 24
enc = ws[: 16 * S * 8].view(torch.int32).to(torch.int64)
w = (torch.arange(enc.numel(), device=dev, dtype=torch.int64) % 9973) + 1
ck = int(((enc * w) % (1 << 61)).sum()) , int(enc.sum())
med = statistics.median(ts)
print(f"{med:.4f} ms  {1024 * S / med / 1e6:.0f} GB/s algorithmic  ck={ck}")
'''


def main():
    modes = sys.argv[1:] or ["9", "1", "2", "33", "257", "289", "290"]
    for m in modes:
        env = dict(os.environ, SDFR_ENC_MODE=m)
        r = subprocess.run([sys.executable, "-c", CHILD, str(REPO)], env=env,
                           capture_output=True, text=True, timeout=300)
        out = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-800:]
        print(f"mode {m}: {out}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
