"""A/B of the field kernels (field_x2_kernel vs field_p_kernel) on the bench workload:
median field time per variant (each in its own subprocess, selected by SDFR_FIELD_X2)
and the max |difference| of their outputs.  Profiling aid, not a test.
    python scripts/pair_ab.py [net] [B] [rounds]"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]

CHILD = r'''
import statistics, sys, torch, numpy as np
sys.path.insert(0, sys.argv[1])
from sdfr_loader import load
sdfr = load()
dev = "cuda:0"; net = sys.argv[2]; B = int(sys.argv[3]); rounds = int(sys.argv[4])
opt = sdfr.vol_render_opt(ngp=(net == "ngp"))
opt.rendering.return_sdf = True
opt.rendering.return_xyz = True
torch.manual_seed(0)
g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
ren = g.renderer; ren.rng_device = "device"
ext, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
for e in evs: e.record()
ts = []; te = []
with torch.no_grad():
    lat = g.style(torch.randn(B, 256, device=dev))
    for r in range(rounds):
        ren.stage_events = evs
        torch.manual_seed(5)
        out = ren(ext, focal, near, far, styles=lat)
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(evs[2].elapsed_time(evs[3])); te.append(evs[1].elapsed_time(evs[2]))
print("encode_ms", statistics.median(te), file=sys.stderr)
np.savez(sys.argv[5], *[t.float().cpu().numpy() for t in out if torch.is_tensor(t)])
print(statistics.median(ts))
'''


def main():
    net = sys.argv[1] if len(sys.argv) > 1 else "ngp"
    B = sys.argv[2] if len(sys.argv) > 2 else "32"
    rounds = sys.argv[3] if len(sys.argv) > 3 else "10"
    res = {}
    outs = {}
    for name in ("x2", "pair", "x2b", "pairb"):
        env = dict(os.environ)
        env.pop("SDFR_FIELD_X2", None)
        if name.startswith("x2"):
            env["SDFR_FIELD_X2"] = "1"
        f = f"/tmp/pair_ab_{name}.npz"
        r = subprocess.run([sys.executable, "-c", CHILD, str(REPO), net, B, rounds, f], env=env,
                           capture_output=True, text=True, timeout=600)
        if r.returncode:
            print(r.stderr[-3000:])
            sys.exit(r.returncode)
        res[name] = float(r.stdout.strip().splitlines()[-1])
        outs[name] = np.load(f)
    diffs = {}
    for k in outs["x2"].files:
        a, b = outs["x2"][k], outs["pair"][k]
        diffs[k] = [list(a.shape), float(np.abs(a - b).max()), float(np.abs(a).max())]
    flop = (550912 if net == "ngp" else 1053696) * int(B) * 4096 * 24
    print(json.dumps({"net": net, "B": int(B), "field_ms": res,
                      "tflops": {k: flop / v / 1e9 for k, v in res.items()},
                      "max_abs_diff_x2_vs_pair": diffs}, indent=1))


if __name__ == "__main__":
    main()
