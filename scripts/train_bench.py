"""BASELINE configs[2] / configs[4]: stage-2 training throughput, DDP over RCCL.

    python scripts/train_bench.py [--net ngp|siren] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 scripts/train_bench.py ...

Random-init G/D (no checkpoints offline), synthetic real images; per GPU batch 8 in
chunks of 2 (train.py defaults), R1 every 16, path regularisation every 4 steps.
One JSON line: training steps/s and faces/s (all ranks; each step renders
batch D-fakes + batch G-fakes, + batch/2 every 4th step), timed between barriers,
max over ranks."""
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--net", default="ngp", choices=["ngp", "siren"])
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--chunk", type=int, default=2)
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    sdfr = load()
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = sdfr.vol_render_opt(ngp=a.net == "ngp", batch=a.batch, chunk=a.chunk)
    tr = FullPipelineTrainer(opt, dev, seed=0)
    tr.g_module.renderer.rng_device = "device"
    tr.generator_test.renderer.rng_device = "device"
    torch.manual_seed(1000 + rank)
    size = opt.model.size
    real = [torch.rand(a.batch, 3, size, size, device=dev) * 2 - 1 for _ in range(4)]
    for k in range(a.warmup):
        tr.step(real[k % 4])
    torch.cuda.synchronize()
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
        print(json.dumps({
            "metric": "stage-2 training throughput (renderer frozen, fused HIP forward)",
            "value": world * a.batch * a.steps / el, "unit": "faces/s (real-batch faces)",
            "steps_per_s": a.steps / el, "ms_per_step": el / a.steps * 1e3, "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "scaling": "weak",
            "config": {"workload": f"train.py stage 2, {a.net} renderer, random-init G/D",
                       "batch_per_gpu": a.batch, "chunk": a.chunk, "size": size,
                       "parallelism": f"ddp{world} (RCCL all-reduce of decoder + D grads)"},
            "losses": {k: float(v) for k, v in losses.items()}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
