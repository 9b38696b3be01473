"""GPU: the RCCL ("nccl") backend on the one MI355X of the box, world size 1.

The multi-rank tests elsewhere run gloo (two ranks cannot share one GPU over RCCL);
this puts the 8-GPU run's own calls on the hardware before any 8-GPU run: a
freshly spawned child (nothing touched the GPU in it before) forms an "nccl" process
group with ``device_id=cuda:0`` and runs
  * one stage-2 FullPipelineTrainer step with the generator and discriminator wrapped
    in DDP (RCCL bucket all-reduce of the decoder / discriminator gradients), which
    must equal the same step without a process group BIT FOR BIT (a world-1 average
    is the identity: sum of one, divided by 1);
  * ``allreduce_grads`` (the flat all-reduce of the stage-1 sphere init) and
    ``reduce_loss_dict`` (training.py), likewise bit-identical;
  * bench.py's ``timed_steps`` (barrier + synchronize + MAX all-reduce);
and bench.py itself under torchrun with ``SDFR_BENCH_DIST=1`` (setup_dist's nccl
init).  Reference: sdf_utils.py:344-379 (get_world_size / synchronize /
reduce_loss_dict over NCCL).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _stage2(sdfr, dev, real):
    from sdface_gan_amd.training import FullPipelineTrainer
    opt = sdfr.vol_render_opt(batch=2, chunk=1)
    tr = FullPipelineTrainer(opt, dev, seed=3)
    torch.manual_seed(50)
    losses = tr.step(real.clone())
    out = {"losses": {k: v.detach().clone() for k, v in losses.items()},
           "d": {k: v.detach().clone() for k, v in tr.d_module.state_dict().items()},
           "dec": {k: v.detach().clone() for k, v in tr.g_module.state_dict().items()
                   if k.startswith("decoder.")}}
    ddp = type(tr.generator).__name__
    del tr
    return out, ddp


def _diff(a, b):
    bad = []
    for part in ("losses", "d", "dec"):
        for k, v in a[part].items():
            if not torch.equal(v, b[part][k]):
                bad.append(f"{part}.{k}")
    return bad


def _rccl_worker(rank, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    sys.path.insert(0, str(REPO))
    from sdfr_loader import load
    sdfr = load()
    from sdface_gan_amd.training import allreduce_grads, reduce_loss_dict
    import bench
    res = {}
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    real = torch.rand(2, 3, 256, 256, device=dev, generator=g) * 2 - 1
    # two runs without a process group: the step's own run-to-run determinism
    a, wrap_a = _stage2(sdfr, dev, real)
    b, _ = _stage2(sdfr, dev, real)
    res["plain_runs_equal"] = not _diff(a, b)

    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res["backend"] = dist.get_backend()
    c, wrap_c = _stage2(sdfr, dev, real)
    res["wrapper_plain"], res["wrapper_ddp"] = wrap_a, wrap_c
    res["ddp_vs_plain_diff"] = _diff(a, c)

    # the flat gradient all-reduce and the loss-dict reduction
    params = [torch.nn.Parameter(torch.randn(n, device=dev, generator=g)) for n in (12_658_000, 256, 3)]
    for p in params:
        p.grad = torch.randn(p.shape, device=dev, generator=g)
    before = [p.grad.clone() for p in params]
    allreduce_grads(params)
    res["allreduce_grads_equal"] = all(torch.equal(x, p.grad) for x, p in zip(before, params))
    ld = {"d": torch.tensor(0.25, device=dev), "g": torch.tensor(-1.5, device=dev),
          "r1": torch.tensor(3.0e-3, device=dev)}
    red = reduce_loss_dict(ld)
    res["reduce_loss_dict_equal"] = all(torch.equal(ld[k].float(), red[k]) for k in ld)

    # bench.py's timed region with the group formed (barrier, MAX all-reduce)
    x = torch.randn(1 << 20, device=dev)
    el = bench.timed_steps(lambda: x.mul_(1.0), 3, 1, dev)
    res["timed_steps_s"] = el
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(res, f)


def test_rccl_world1_stage2_collectives(tmp_path):
    out = tmp_path / "rccl.json"
    mp.spawn(_rccl_worker, args=(_free_port(), str(out)), nprocs=1, join=True)
    res = json.loads(out.read_text())
    assert res["backend"] == "nccl"
    assert res["wrapper_plain"] == "Generator"
    assert res["wrapper_ddp"] == "DistributedDataParallel"
    assert res["allreduce_grads_equal"] and res["reduce_loss_dict_equal"]
    assert res["timed_steps_s"] > 0
    # bit for bit when the plain step itself is deterministic (it is on MI355X with the
    # deterministic MIOpen flags; otherwise the DDP run could not be told apart anyway)
    assert res["plain_runs_equal"], "stage-2 step not run-to-run deterministic"
    assert res["ddp_vs_plain_diff"] == [], res["ddp_vs_plain_diff"][:10]


def test_bench_rccl_world1():
    """bench.py under torchrun, one rank, process group over RCCL (SDFR_BENCH_DIST=1)."""
    env = dict(os.environ, SDFR_BENCH_DIST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(REPO / "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--batch", "4",
           "--no-cpu-baseline", "--no-extras"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["value"] > 0
