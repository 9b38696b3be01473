"""BASELINE configs[2] / configs[4]: training throughput, DDP over RCCL.

    python scripts/train_bench.py [--stage 1|2] [--net ngp|siren|fc] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 scripts/train_bench.py ...

Random-init G/D (no checkpoints offline), synthetic real images; per GPU batch 8 in
chunks of 2 (train.py defaults), R1 every 16, path regularisation every 4 steps.
One JSON line: training steps/s and faces/s (all ranks; each step renders
batch D-fakes + batch G-fakes, + batch/2 every 4th step), timed between barriers,
max over ranks.

--stage 1 measures renderer training (training_utils.py:287-451; SURVEY §8(d) "stage 1
reported separately as 64^2 thumbs/s"): the renderer trains through the op-by-op path
with the HIP hash-grid / SH encoder forward and backward (table gradients by fp32
atomics, dy_dx for the eikonal term), VolumeRenderDiscriminator on 64^2 thumbs, the
eikonal + minimal-surface + smoothness losses; one step = one D and one G iteration
over `batch` thumbs (D-fakes + G-fakes).  Stage 1 uses batch 8 in chunks of 2 too
unless --batch/--chunk say otherwise."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


class _NoCache(dict):
    def __setitem__(self, k, v):
        pass


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--stage", type=int, default=2, choices=[1, 2])
    p.add_argument("--net", default="ngp", choices=["ngp", "siren", "fc"])
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--chunk", type=int, default=2)
    p.add_argument("--miopen-find", action="store_true",
                   help="torch.backends.cudnn.benchmark = True (MIOpen find per conv shape "
                        "during warmup instead of its heuristics)")
    p.add_argument("--miopen-db", default=None,
                   help="MIOpen user find / perf database directory (MIOPEN_USER_DB_PATH), "
                        "e.g. sdface-gan_amd/miopen_db: the stage-2 convolutions' find results "
                        "recorded on an MI355X (ROCm 7.2 image), so --miopen-find skips its "
                        "~12 min search")
    p.add_argument("--train-gemm", default="f16x3", choices=["f16x3", "torch"],
                   help="stage 1: renderer-MLP GEMMs on the split-fp16 MFMA kernels or on "
                        "rocBLAS fp32 (linear.py)")
    p.add_argument("--coord-pad", type=int, default=8,
                   help="stage-1 discriminator CoordConv channel padding (training.py; 1 = off)")
    p.add_argument("--no-coord-cache", action="store_true",
                   help="rebuild the CoordConv coordinate planes per call (A/B aid)")
    p.add_argument("--no-skip-identity", action="store_true",
                   help="LinearLayer computes the literal 1 * y + 0 (A/B aid)")
    a = p.parse_args()
    if a.miopen_db:                      # before MIOpen's first handle (the first convolution)
        os.environ["MIOPEN_USER_DB_PATH"] = str(Path(a.miopen_db).resolve())
    torch.backends.cudnn.benchmark = a.miopen_find
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    sdfr = load()
    from sdface_gan_amd.linear import set_train_gemm
    from sdface_gan_amd.training import FullPipelineTrainer, RendererTrainer
    set_train_gemm(a.train_gemm)
    from sdface_gan_amd.training import CoordConv2d
    CoordConv2d.pad_to = a.coord_pad
    if a.no_skip_identity:
        from sdface_gan_amd.renderer import LinearLayer
        LinearLayer.skip_identity = False
    if a.no_coord_cache:
        import sdface_gan_amd.training as training_mod
        training_mod._COORD_PLANES = _NoCache()
    opt = sdfr.vol_render_opt(ngp=a.net == "ngp", fc=a.net == "fc", batch=a.batch, chunk=a.chunk,
                              train_renderer=a.stage == 1)
    if a.stage == 1:
        tr = RendererTrainer(opt, dev, seed=0)
        size = opt.training.renderer_output_size
    else:
        tr = FullPipelineTrainer(opt, dev, seed=0)
        size = opt.model.size
    tr.g_module.renderer.rng_device = "device"
    tr.generator_test.renderer.rng_device = "device"
    torch.manual_seed(1000 + rank)
    real = [torch.rand(a.batch, 3, size, size, device=dev) * 2 - 1 for _ in range(4)]
    if a.miopen_find and rank == 0:
        # MIOpen's find can run for minutes inside one warmup step without a line of
        # output: a heartbeat keeps the run visibly alive (gpurun kills silent runs)
        import threading
        t_start = time.perf_counter()

        def beat():
            while True:
                time.sleep(30)
                print(f"  ... {time.perf_counter() - t_start:.0f} s", flush=True)
        threading.Thread(target=beat, daemon=True).start()
    for k in range(a.warmup):
        t0 = time.perf_counter()
        tr.step(real[k % 4])
        torch.cuda.synchronize()
        if rank == 0:          # progress (MIOpen find spends minutes in the first steps)
            print(f"warmup step {k}: {time.perf_counter() - t0:.2f} s", flush=True)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(a.steps):
        losses = tr.step(real[k % 4])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        metric = ("stage-1 renderer training throughput (HIP encoder forward + backward)"
                  if a.stage == 1 else
                  "stage-2 training throughput (renderer frozen, fused HIP forward)")
        unit = "64^2 thumbs/s (real-batch thumbs)" if a.stage == 1 else \
            "faces/s (real-batch faces)"
        print(json.dumps({
            "metric": metric, "value": world * a.batch * a.steps / el, "unit": unit,
            "steps_per_s": a.steps / el, "ms_per_step": el / a.steps * 1e3, "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "scaling": "weak",
            "config": {"workload": f"train.py stage {a.stage}, {a.net} renderer, random-init G/D",
                       "batch_per_gpu": a.batch, "chunk": a.chunk, "size": size,
                       "miopen_find": a.miopen_find,
                       "parallelism": (f"ddp{world} ({dist.get_backend()} all-reduce of "
                                       f"{'G' if a.stage == 1 else 'decoder'} + D grads)")
                                      if world > 1 else "single process (no all-reduce)"},
            "losses": {k: float(v) for k, v in losses.items()}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
