"""Attribute ngp_field_kernel time by ablation (profiling aid, not a test).

Runs the fused renderer on B faces with each ablated field-kernel build
(sdfr_debug_set_field_variant), interleaved over several rounds in ONE process,
and prints the median field-stage time per variant.  Also probes PyTorch-ROCm's
own fp32 sin / GEMM accuracy against float64 (explains the module-path bound).
"""
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402

VARIANTS = {0: "product", 1: "no barrier", 2: "no LDS A reads", 4: "no staging",
            8: "no activations", 16: "no compositing (f16x3)", 31: "MFMA only"}


def main(B=32, rounds=5, precision="f16x3"):
    sdfr = load()
    dev = "cuda:0"
    opt = sdfr.vol_render_opt()
    torch.manual_seed(0)
    g = sdfr.Generator(opt.model, opt.rendering).to(dev).eval()
    ren = g.renderer
    ren.rng_device = "device"
    ren.field_precision = precision
    print(f"field precision {precision}")
    ext, focal, near, far, _ = sdfr.generate_camera_params(64, dev, batch=B)
    lat = g.style(torch.randn(B, 256, device=dev))
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for e in evs:
        e.record()
    lib = sdfr._lib.lib()
    times = {v: [] for v in VARIANTS}
    with torch.no_grad():
        for r in range(rounds + 1):
            for v in VARIANTS:
                sdfr._lib.check(lib.sdfr_debug_set_field_variant(v), "variant")
                ren.stage_events = evs
                ren(ext, focal, near, far, styles=lat)
                torch.cuda.synchronize()
                if r:
                    times[v].append(evs[2].elapsed_time(evs[3]))
    lib.sdfr_debug_set_field_variant(0)
    ren.stage_events = None
    out = {}
    for v, name in VARIANTS.items():
        med = statistics.median(times[v])
        out[name] = med
        samples = B * 64 * 64 * 24
        print(f"variant {v:2d} {name:16s} field {med:8.3f} ms  "
              f"{550912 * samples / med / 1e9:7.1f} TFLOP/s", flush=True)

    # device sin implementations vs float64 (|x| <= 200, the FiLM argument range)
    xs = ((torch.rand(1 << 22, dtype=torch.float64) - 0.5) * 400).float()
    xd = xs.to(dev)
    cw = torch.empty_like(xd)
    hw = torch.empty_like(xd)
    sdfr._lib.check(lib.sdfr_debug_sin_probe(sdfr._lib.ptr(xd), sdfr._lib.ptr(cw),
                                             sdfr._lib.ptr(hw), xd.numel(), None), "sin probe")
    torch.cuda.synchronize()
    ref = torch.sin(xs.double())
    for name, v in (("sin_cw", cw), ("sin_hw", hw)):
        e = (v.cpu().double() - ref).abs()
        print(f"{name}: max abs err {e.max().item():.3e}, mean {e.mean().item():.3e}", flush=True)
        out[f"{name}_max_err"] = e.max().item()

    # PyTorch-ROCm fp32 accuracy probes (module path)
    x = (torch.rand(1 << 20, dtype=torch.float64) - 0.5) * 200
    s_gpu = torch.sin(x.float().to(dev)).double().cpu()
    err_sin = (s_gpu - torch.sin(x.float().double())).abs().max().item()
    a = torch.randn(4096, 256, dtype=torch.float64)
    w = torch.randn(256, 256, dtype=torch.float64) / 16
    y_gpu = torch.nn.functional.linear(a.float().to(dev), w.float().to(dev)).double().cpu()
    y_ref = torch.nn.functional.linear(a.float().double(), w.float().double())
    err_gemm = ((y_gpu - y_ref).abs().max() / y_ref.abs().max()).item()
    print(f"torch-ROCm fp32: max|sin err| = {err_sin:.3e} (|x|<=100), "
          f"linear max rel err = {err_gemm:.3e}", flush=True)
    out["torch_sin_err"] = err_sin
    out["torch_linear_rel_err"] = err_gemm
    Path("gpurun_out").mkdir(exist_ok=True)
    Path("gpurun_out/field_ablation.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(precision=sys.argv[1] if len(sys.argv) > 1 else "f16x3")
