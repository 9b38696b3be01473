"""Median field-stage time of the fused renderer for each libsdfr.so variant given on
the command line (each in its own subprocess; profiling aid, not a test).  NET=siren
(or fc) times the SIREN (FC) renderer instead of ngp.
    python scripts/field_time.py sdface-gan_amd/lib_var/a/libsdfr.so ..."""
import os
import statistics
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]

CHILD = r'''
import statistics, sys, torch
sys.path.insert(0, sys.argv[1])
from sdfr_loader import load
sdfr = load()
dev = "cuda:0"; B = 32
import os
net = os.environ.get("NET", "ngp")
opt = sdfr.vol_render_opt(ngp=net == "ngp", fc=net == "fc")
torch.manual_seed(0)
g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
ren = g.renderer; ren.rng_device = "device"; ren.field_precision = sys.argv[2]
ext, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
evs = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
for e in evs: e.record()
ts = []
with torch.no_grad():
    lat = g.style(torch.randn(B, 256, device=dev))
    for r in range(8):
        ren.stage_events = evs[:4]
        ren.field_event = evs[4]                  # right before the field kernel
        torch.manual_seed(5)
        out = ren(ext, focal, near, far, styles=lat)
        torch.cuda.synchronize()
        if r >= 2: ts.append(evs[4].elapsed_time(evs[3]))
med = statistics.median(ts)
import hashlib
h = hashlib.sha1(b"".join(t.detach().float().cpu().numpy().tobytes() for t in out[:2])).hexdigest()[:12]
flop = {"siren": 1053696, "fc": 1093632}.get(net, 417792)
print(f"out {h}  {med:.3f} ms  {flop * B * 4096 * 24 / med / 1e9:.1f} TFLOP/s")
'''


def main():
    prec = os.environ.get("PREC", "f16x3")
    reps = int(os.environ.get("REPS", "3"))
    libs = sys.argv[1:]
    res = {lib: [] for lib in libs}
    for _ in range(reps):                       # libs interleaved, each in its own process
        for lib in libs:
            env = dict(os.environ, SDFR_LIB=str(REPO / lib) if not lib.startswith("/") else lib)
            out = subprocess.run([sys.executable, "-c", CHILD, str(REPO), prec], env=env,
                                 capture_output=True, text=True, timeout=240)
            if out.returncode:
                print(f"{lib:50s} FAILED rc={out.returncode}: {out.stderr.strip().splitlines()[-1:]}")
                continue
            line = out.stdout.strip().splitlines()[-1]
            res[lib].append(float(line.split()[2]))
            print(f"{lib:50s} {line}", flush=True)
    for lib, v in res.items():
        if v:
            print(f"SUMMARY {lib:50s} median {statistics.median(v):.3f} ms  min {min(v):.3f}  "
                  f"n {len(v)}", flush=True)


if __name__ == "__main__":
    main()
