"""What data parallelism costs per training step, measured on the one GPU of the box.

    python scripts/ddp_cost.py [--steps 6] [--out gpurun_out/ddp_cost.json]

Forms an RCCL ("nccl") process group at world size 1 (the 8-GPU run's own code path:
training.py wraps in DDP and runs its collectives whenever a group exists) and times,
interleaved, the same trainer steps with the group hidden (``training._dist_on`` ->
False: plain replicas, no DDP wrapper, no collective) and with it (DDP bucket
all-reduce, ``allreduce_grads``, ``reduce_loss_dict``):
  * stage 2 (FullPipelineTrainer, batch 8 in chunks of 2, training_utils.py:654-867),
  * stage 1 (RendererTrainer, batch 8 in chunks of 2, training_utils.py:336-451),
  * the stage-1 sphere-init step (batch 3, training_utils.py:287-327) with its flat
    all-reduce of every generator gradient (``allreduce_grads``),
plus the gradient bytes each step all-reduces.  A world-1 all-reduce moves no bytes
over xGMI, so what the with/without difference shows is the wrapper's own cost
(bucket copies, autograd hooks, the collective launches); the W = 8 communication
time is then predicted from the gradient bytes: a ring all-reduce sends
2 (W - 1) / W x bytes per GPU.
"""
import argparse
import json
import os
import socket
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/ddp_cost.json")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    sdfr = load()
    import sdface_gan_amd.training as T
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    real_on = T._dist_on

    def timed(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    def trainer(stage, ddp):
        T._dist_on = real_on if ddp else (lambda: False)
        opt = sdfr.vol_render_opt(ngp=True, batch=8, chunk=2, train_renderer=stage == 1)
        tr = (T.RendererTrainer if stage == 1 else T.FullPipelineTrainer)(opt, dev, seed=0)
        tr.g_module.renderer.rng_device = "device"
        tr.generator_test.renderer.rng_device = "device"
        size = opt.training.renderer_output_size if stage == 1 else opt.model.size
        return tr, size

    res = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
           "steps": a.steps, "rounds": a.rounds, "rows": []}
    for stage in (2, 1):
        for r in range(a.rounds):
            for ddp in (False, True):
                tr, size = trainer(stage, ddp)
                torch.manual_seed(1000)
                real = torch.rand(8, 3, size, size, device=dev) * 2 - 1
                for _ in range(a.warmup):
                    tr.step(real)
                ms = timed(lambda: tr.step(real), a.steps)
                gparams = ([p for p in tr.g_train] if stage == 2 else
                           list(tr.g_module.parameters()))
                nbytes = 4 * (sum(p.numel() for p in gparams) +
                               sum(p.numel() for p in tr.d_module.parameters()))
                res["rows"].append({"what": f"stage {stage} step (batch 8, chunk 2)",
                                    "ddp": ddp, "round": r, "ms_per_step": ms,
                                    "grad_bytes_per_step": nbytes,
                                    "wrapper": type(tr.generator).__name__})
                print(json.dumps(res["rows"][-1]), flush=True)
                if stage == 1:
                    tr.step(real)           # restore requires_grad on the generator
                    ms = timed(lambda: tr.sphere_init_step(), a.steps * 3)
                    gbytes = 4 * sum(p.numel() for p in tr.g_module.parameters())
                    res["rows"].append({"what": "stage 1 sphere-init step (batch 3)",
                                        "ddp": ddp, "round": r, "ms_per_step": ms,
                                        "grad_bytes_per_step": gbytes})
                    print(json.dumps(res["rows"][-1]), flush=True)
                    if ddp:
                        # the flat all-reduce alone, on the gradients of one more step
                        noise = T.mixing_noise(3, tr.t.style_dim, tr.t.mixing, dev)
                        cam, focal, near, far, _ = tr._cams(3)
                        sdf, target = tr.g_module.init_forward(noise, cam, focal, near, far)
                        torch.nn.functional.l1_loss(sdf, target).backward()
                        ps = list(tr.g_module.parameters())
                        ms = timed(lambda: T.allreduce_grads(ps), 20)
                        res["rows"].append({"what": "allreduce_grads alone (world 1)",
                                            "ms": ms, "grad_bytes": gbytes})
                        print(json.dumps(res["rows"][-1]), flush=True)
                del tr
                torch.cuda.empty_cache()
    T._dist_on = real_on
    dist.destroy_process_group()
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))
    print("wrote", a.out)


if __name__ == "__main__":
    main()
