"""A training step under torch.profiler (profiling aid, not a test): which aten ops
and which Python call sites issue the kernels around the HIP ones.  Stage 2 also
gets a per-phase table (the trainer's record_function ranges: D step incl. R1, G
step, path regularisation) with the device time of the kernels inside each.

    python scripts/train_prof.py [--stage 1|2] [--steps 2] [--miopen-find]
                                 [--out gpurun_out/train_prof.txt]"""
import argparse
import sys
from pathlib import Path

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--out", default="gpurun_out/train_prof.txt")
    p.add_argument("--net", default="ngp", choices=["ngp", "siren"])
    p.add_argument("--stage", type=int, default=1, choices=[1, 2])
    p.add_argument("--miopen-find", action="store_true")
    a = p.parse_args()
    torch.backends.cudnn.benchmark = a.miopen_find
    dev = torch.device("cuda", 0)
    sdfr = load()
    from sdface_gan_amd.training import CoordConv2d, FullPipelineTrainer, RendererTrainer
    CoordConv2d.pad_to = 8
    opt = sdfr.vol_render_opt(ngp=a.net == "ngp", batch=8, chunk=2,
                              train_renderer=a.stage == 1)
    tr = (RendererTrainer if a.stage == 1 else FullPipelineTrainer)(opt, dev, seed=0)
    tr.g_module.renderer.rng_device = "device"
    tr.generator_test.renderer.rng_device = "device"
    size = opt.training.renderer_output_size if a.stage == 1 else opt.model.size
    torch.manual_seed(1000)
    real = [torch.rand(8, 3, size, size, device=dev) * 2 - 1 for _ in range(4)]
    for k in range(4):
        tr.step(real[k % 4])
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for k in range(4):
        tr.step(real[k % 4])
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t0) / 4 * 1e3
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        for k in range(a.steps):
            tr.step(real[k % 4])
        torch.cuda.synchronize()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "w") as f:
        f.write(f"# {a.steps} stage-{a.stage} steps (steps 4-7 of the trainer; 4 unprofiled "
                f"steps before: {wall_ms:.1f} ms per step wall), miopen_find={a.miopen_find}\n")
        ranges = [ev for ev in prof.key_averages() if ev.key.startswith("stage")]
        if ranges:
            f.write("# per phase (record_function ranges): CPU wall ms/step, device ms/step\n")
            for ev in sorted(ranges, key=lambda e: e.key):
                f.write(f"{ev.key:24s} {ev.cpu_time_total / 1e3 / a.steps:9.2f} "
                        f"{ev.device_time_total / 1e3 / a.steps:9.2f}  x{ev.count / a.steps:.2f}\n")
        # (the record_function ranges carry their whole span as self device time: left out)
        names = {ev.key for ev in ranges} if ranges else set()
        tot = sum(ev.self_device_time_total for ev in prof.key_averages()
                  if ev.key not in names) / 1e3 / a.steps
        f.write(f"# device time, all kernels: {tot:.2f} ms per step\n\n")
        f.write(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=70,
                                          max_name_column_width=70))
        f.write("\n\n# by call site (5 frames)\n")
        f.write(prof.key_averages(group_by_stack_n=5).table(
            sort_by="self_cuda_time_total", row_limit=80, max_name_column_width=50,
            max_src_column_width=120))
        f.write("\n\n# call sites of the small torch ops (stack, repo frames only)\n")
        rows = []
        for ev in prof.key_averages(group_by_stack_n=12):
            if not ev.key.startswith("aten::") or ev.key in ("aten::miopen_convolution",
                                                             "aten::convolution_backward"):
                continue
            cuda = ev.self_device_time_total
            if cuda <= 0:
                continue
            frames = [fr for fr in ev.stack if "sdface-gan_amd" in fr or "scripts/" in fr]
            rows.append((cuda, ev.count, ev.key, frames[:4]))
        rows.sort(key=lambda r: -r[0])
        for cuda, cnt, key, frames in rows[:60]:
            f.write(f"{cuda / 1e3 / a.steps:8.3f} ms/step {cnt / a.steps:7.1f} calls/step  {key}\n")
            for fr in frames:
                f.write(f"            {fr}\n")
        f.write("\n\n# small torch ops by input shapes\n")
        rows = []
        for ev in prof.key_averages(group_by_input_shape=True):
            if ev.key in ("aten::copy_", "aten::cat", "aten::mul", "aten::add", "aten::add_",
                          "aten::sum", "aten::div", "aten::fill_", "aten::sub", "aten::mm") \
                    and ev.self_device_time_total > 0:
                rows.append((ev.self_device_time_total, ev.count, ev.key, ev.input_shapes))
        rows.sort(key=lambda r: -r[0])
        for cuda, cnt, key, shp in rows[:70]:
            f.write(f"{cuda / 1e3 / a.steps:8.3f} ms/step {cnt / a.steps:7.1f}/step  {key:12s} {shp}\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
