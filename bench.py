"""Throughput bench: rendered 256^2 faces/s (SDF + ngp Generator), 1..8 GPUs.

Workload (BASELINE.json configs[1], eval.py's 5000-image generation): per step
one Generator forward -- mapping MLP -> fused HIP renderer (64^2 rays x 24
samples, hash grid, FiLM-SIREN on split-fp16 MFMA at fp32 accuracy, compositing)
-> StyleGAN2 decoder to 256^2 (HIP implicit-GEMM convolutions with fused
epilogues) -- on a batch of B random latents with
random cameras, random-init weights (pretrained weights are not available
offline), decoder noise drawn per step as in eval.py.  PNG encoding is not
timed.  One process per GPU (torchrun); faces shard across ranks with no
data-path collective (weak scaling): value = all faces / max-over-ranks time.

Also reported: the dominant kernel's roofline (the fused field kernel, MFMA
bound) from HIP events recorded on the renderer's stream around that kernel
during the timed steps, the hash-grid gather kernel's HBM-roofline fraction,
a CPU baseline (the oracle renderer + PyTorch-CPU decoder) on the host cores
for a bounded sample, and after the timed region, outside
`value`: faces/s at B = 1 (eval.py's own batch) and 8, and at B with every
image copied to pinned host memory ("with host copy").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

METRIC = "rendered faces/sec/GPU at 256² (SDF+ngp path); 1/2/4/8-GPU scaling"
FLOP_PER_SAMPLE = 550912          # renderer MLP as the reference runs it, SURVEY.md §8(d)
# what the fused split-fp16 kernel computes per sample: input_linear and pts_linears.0
# composed into one 32 -> 256 map (no nonlinearity between them), so
# one 256 x 256 GEMM (131,072 FLOP) less, and the views layer at its 272 inputs
# (32 + 256 + 256 + 272 rows of 256 x 2 FLOP); roofline.achieved / frac count these (what the
# hardware runs), roofline.algorithmic_equivalent the reference's
FLOP_PER_SAMPLE_FUSED = 417792
FLOP_PER_SAMPLE_SIREN = 1053696   # SirenGenerator MLP, SURVEY.md §8(d)
# FCGenerator MLP (sdf_model.py:1599-1670): 2 (60 + 7 x 256 + 280) 256 + heads 2 (1 + 3) 256
FLOP_PER_SAMPLE_FC = 1093632
GATHER_BYTES_PER_SAMPLE = 1024    # 16 levels x 8 corners x 2 x fp32
MFMA_F32_PEAK_TFLOPS = 157.3      # MI355X fp32 matrix peak (MI355X_MICROARCH.md)
MFMA_F16_PEAK_TFLOPS = 2500.0     # MI355X dense fp16/bf16 MFMA peak (no sparsity)
HBM_PEAK_GBPS = 8000.0            # MI355X HBM3E peak
MFMA_CLOCK_GHZ = 2.4              # clock the MFMA peaks are quoted at


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=32, help="faces per step per GPU")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--field-precision", default="f16x3", choices=["f16x3", "fp32"],
                   help="field-stage GEMM arithmetic (DESIGN.md section 5)")
    p.add_argument("--net", default="ngp", choices=["ngp", "siren", "fc"],
                   help="renderer network: ngp (headline, configs[1]), fc (FCGenerator, "
                        "rendering.fc = 1: configs[4]'s plain Fourier MLP) or siren "
                        "(rendering.type 'sdf', configs[4]'s generator)")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-extras", action="store_true",
                   help="skip the B=1/8 and host-copy measurements")
    p.add_argument("--traffic-json", default=str(REPO / "profiles" / "field_traffic.json"))
    p.add_argument("--counters-json", default=str(REPO / "profiles" / "round6_counters.json"),
                   help="committed SQ counter summary (scripts/summarize_counters.py) quoted "
                        "as the field kernel's MFMA-busy fraction")
    return p.parse_args()


def setup_dist(args=None):
    """One process per GPU (torchrun's RANK / LOCAL_RANK / WORLD_SIZE): backend "nccl"
    (RCCL over xGMI).  SDFR_BENCH_BACKEND=gloo with SDFR_BENCH_SAME_DEVICE=1 runs the
    same multi-rank path with every rank on cuda:0 (the world-2 test on a one-GPU
    box, tests/test_gpu_train.py); SDFR_BENCH_DIST=1 forms the process group at world
    size 1 too (RCCL init, barriers and the MAX all-reduce on a one-GPU box)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SDFR_BENCH_SAME_DEVICE") == "1":
        local = 0
    if world > 1 or os.environ.get("SDFR_BENCH_DIST") == "1":
        torch.cuda.set_device(local)
        backend = os.environ.get("SDFR_BENCH_BACKEND", "nccl")
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return world, rank, torch.device("cuda", local)


def timed_steps(step, steps, world, device, before_step=None):
    """The timed region: barrier + synchronize on both sides of exactly `steps`
    steps; returns the MAX over ranks of the wall time (seconds)."""
    grouped = dist.is_available() and dist.is_initialized()
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        if before_step is not None:
            before_step(k)
        step()
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if grouped:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def _cgroup_cpus():
    """CPUs granted by the cgroup's CPU quota (cgroup v2 cpu.max / v1 cfs), or None."""
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            return -(-int(quota) // int(period))
    except (OSError, ValueError):
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        p = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        if q > 0:
            return -(-q // p)
    except (OSError, ValueError):
        pass
    return None


def host_info():
    """Host CPU facts for the CPU baseline line: logical CPUs, the affinity mask, the
    physical cores in it (one per SMT sibling group), the cgroup CPU quota, the model
    name, and `cores` = the threads the baseline runs with: every physical core of the
    affinity mask, capped by the quota (threads beyond the quota only time-slice)."""
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = sorted(os.sched_getaffinity(0))
    groups = set()
    for c in aff:
        try:
            groups.add(Path(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list")
                       .read_text().strip())
        except OSError:
            groups.add(str(c))
    quota = _cgroup_cpus()
    cores = len(groups) if quota is None else max(1, min(len(groups), quota))
    return {"nproc": os.cpu_count(), "affinity_cpus": len(aff), "physical_cores_in_affinity":
            len(groups), "cgroup_cpu_quota": quota, "cpu_model": model, "cores": cores}


def build_generator(sdfr, device, seed, ngp=True, fc=False):
    opt = sdfr.vol_render_opt(ngp=ngp, fc=fc)
    torch.manual_seed(seed)
    g = sdfr.Generator(opt.model, opt.rendering).to(device)
    g.eval()
    # per-ray sampling offsets from the device RNG (no host round trip per step)
    g.renderer.rng_device = "device"
    return g, opt


def cpu_baseline(seconds, siren=False, fc=False):
    """Oracle renderer (torch-CPU fp32 + C encoders) + PyTorch-CPU decoder, one face
    per call as eval.py does, on the host cores; bounded to ~`seconds`."""
    from oracle import oracle
    from sdfr_loader import load
    sdfr = load()
    oracle.build()
    host = host_info()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(host["cores"])
    opt = sdfr.vol_render_opt(ngp=not (siren or fc), fc=fc)
    torch.manual_seed(1)
    g = sdfr.Generator(opt.model, opt.rendering).eval()
    render = oracle.render_fc if fc else (oracle.render_siren if siren else oracle.render_ngp)
    sd = {k: v for k, v in g.state_dict().items() if k.startswith("renderer.")}
    faces, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            z = torch.randn(1, 256)
            cam, focal, near, far, _ = sdfr.generate_camera_params(64, "cpu", batch=1)
            lat = g.style(z)
            out = render(sd, cam.numpy(), focal.numpy(), near.numpy(), far.numpy(),
                                    lat.numpy(), N=24, res=64, t_rand=torch.rand(1, 64, 64).numpy())
            img, _ = g.decoder(out["features"], [lat])
            faces += 1
            el = time.perf_counter() - t0
            if el >= seconds and faces >= 2:
                break
    used = torch.get_num_threads()
    torch.set_num_threads(prev_threads)
    return {"value": faces / el, "unit": "faces/s", **host, "cores": used,
            "kind": "port",
            "sample": f"{faces} faces (64^2x24 oracle renderer + CPU decoder to 256^2), "
                      f"1 face per call, {el:.1f}s; cores = torch intra-op threads used "
                      "(physical cores of the affinity mask, capped by the cgroup quota)"}


def extras(step, B, graphed_step, g, steps=10, warm=5):
    """Outside the timed region (this rank only): faces/s at B = 1 and 8 through the
    plain API call (``faces_per_s_b1``: eval.py's unchanged loop, which
    Generator.forward serves from its own graph cache after the first call;
    ``_nocache``: the same with that cache off, every call eager), at B = 1 from
    GraphedGenerator with the draws inside the graph too, and at B with each step's
    images copied to pinned host memory as eval.py's PNG writer needs them (the copy
    of step k overlaps step k+1's kernels).  At least 200 faces per rate, 600 at
    batch 1: ten batch-1 replays (~6 ms) read 4-5 % low against the steady state, and
    200 (~110 ms) still varied by ~5 % between boxes."""
    def rate(nb, host=False, fn=step):
        buf = torch.empty(nb, 3, 256, 256, pin_memory=True) if host else None
        n = max(steps, -(-(600 if nb == 1 else 200) // nb))
        for _ in range(warm):
            fn(nb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            img = fn(nb)
            if host:
                buf.copy_(img, non_blocking=True)
        torch.cuda.synchronize()
        return nb * n / (time.perf_counter() - t0)
    out = {"faces_per_s_b1": rate(1)}
    g.graph_inference = False
    out["faces_per_s_b1_nocache"] = rate(1)
    g.graph_inference = True
    return {**out, "faces_per_s_b1_graph": rate(1, fn=graphed_step),
            "faces_per_s_b8": rate(8),
            f"faces_per_s_b{B}_with_host_copy": rate(B, host=True), "unit": "faces/s (one GPU)"}


def main():
    args = parse()
    world, rank, device = setup_dist(args)
    from sdfr_loader import load
    sdfr = load()
    fc = args.net == "fc"
    siren = args.net == "siren"
    g, opt = build_generator(sdfr, device, args.seed, ngp=args.net == "ngp", fc=fc)
    siren = siren or fc                         # no hash-grid stage
    g.renderer.field_precision = args.field_precision
    B = args.batch
    res = opt.model.renderer_spatial_output_dim
    N = opt.rendering.N_samples
    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + rank)

    def step(nb=B):
        z = torch.randn(nb, opt.model.style_dim, device=device, generator=gen)
        cam, focal, near, far, _ = sdfr.generate_camera_params(
            res, device, batch=nb, azim_range=opt.camera.azim, elev_range=opt.camera.elev,
            fov_ang=opt.camera.fov, dist_radius=opt.camera.dist_radius)
        with torch.no_grad():
            rgb, thumb = g([z], cam, focal, near, far, truncation=1, truncation_latent=None)
        return rgb

    # per-step stage events on the renderer's stream: [0] entry, [1] before / [2] after
    # the hash-grid gather, [3] after the field kernel, [4] right before it (after the
    # FiLM prep, which the renderer enqueues behind the gather: ABI 11)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(args.steps)]
    for e4 in evs:
        for e in e4:
            e.record()              # materialise the event handles before the timed loop
    torch.cuda.synchronize()

    # and around the decoder's fused regular convolutions (conv_h_kernel), on the
    # decoder's stream
    n_pairs = 1 + len(g.decoder.convs)        # at most one pair per regular convolution
    dev_evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(n_pairs)] for _ in range(args.steps)]
    for pairs in dev_evs:
        for a_, b_ in pairs:
            a_.record()
            b_.record()
    torch.cuda.synchronize()
    conv_flops = []

    # the warmup right before the timed region (the event handles above are made first,
    # so the GPU does not idle between the two)
    for _ in range(args.warmup):
        step()

    # every timed step times the field kernel (the roofline kernel); the first n_full
    # also the render, the gather and the decoder's regular convs (each event the
    # library records costs the stream a few microseconds: the other steps carry two)
    n_full = min(args.steps, 5)
    n_conv = 0

    def set_events(k):
        nonlocal n_conv
        if 0 < k <= n_full:                   # step k - 1's decoder FLOPs / launches
            conv_flops.append(g.decoder.conv_flops)
            n_conv = g.decoder._conv_ev
        full = k < n_full
        g.renderer.stage_events = evs[k][:4] if full else [None, None, None, evs[k][3]]
        g.renderer.field_event = evs[k][4]
        g.decoder.profile_convs(dev_evs[k] if full else None)
    elapsed = timed_steps(step, args.steps, world, device, before_step=set_events)
    if args.steps <= n_full:
        conv_flops.append(g.decoder.conv_flops)
        n_conv = g.decoder._conv_ev
    g.renderer.stage_events = None
    g.renderer.field_event = None
    g.decoder.profile_convs(None)

    conv_ms = sum(a_.elapsed_time(b_) for pairs in dev_evs[:n_full]
                  for a_, b_ in pairs[:n_conv]) / n_full
    enc_ms = sum(e[1].elapsed_time(e[2]) for e in evs[:n_full]) / n_full
    field_ms = sum(e[4].elapsed_time(e[3]) for e in evs) / args.steps
    render_ms = sum(e[0].elapsed_time(e[3]) for e in evs[:n_full]) / n_full
    samples = B * res * res * N
    f16x3 = args.field_precision == "f16x3"
    flop = (FLOP_PER_SAMPLE_FC if fc else FLOP_PER_SAMPLE_SIREN) if siren else (
        FLOP_PER_SAMPLE_FUSED if f16x3 else FLOP_PER_SAMPLE)
    field_tflops = flop * samples / (field_ms * 1e-3) / 1e12
    gather_gbps = GATHER_BYTES_PER_SAMPLE * samples / (enc_ms * 1e-3) / 1e9 if not siren else 0.0
    field_kernel = ("field_r_kernel<sdfr::FcNet>" if fc else
                    "field_p_kernel<sdfr::SirenNet>" if siren else
                    "field_r_kernel<sdfr::NgpNet>") if f16x3 else "ngp_field_kernel"
    field_mfma = "v_mfma_f32_16x16x32_f16" if siren and not fc else "v_mfma_f32_32x32x16_f16"
    def traffic_of(kernel):
        """HBM bytes per launch of `kernel` at this batch, from the committed
        rocprofv3 PMC passes (profiles/, scripts/summarize_profiles.py), or None."""
        tj = Path(args.traffic_json)
        try:
            return json.loads(tj.read_text())["kernels"][kernel]["bytes_per_launch_per_face"] * B
        except (OSError, KeyError, ValueError, TypeError):
            return None

    traffic = traffic_of(field_kernel)

    def decoder_roofline():
        """The decoder's fused regular convolutions (conv_h_kernel, now the largest
        kernel of the step): their fp32-equivalent FLOPs (2 B H W 9 Cin Cout per layer)
        over their HIP-event time, against the same fp32-accurate split-fp16 bound."""
        if not conv_ms or not conv_flops or n_conv == 0:
            return None
        flops = sum(conv_flops) / len(conv_flops)
        tf = flops / (conv_ms * 1e-3) / 1e12
        peak = MFMA_F16_PEAK_TFLOPS / 3
        per_launch = traffic_of("conv_h_kernel")
        return {"kernel": "conv_h_kernel (3x3 convs + styled epilogue + ToRGB partials, "
                          "3 split-fp16 v_mfma_f32_16x16x32_f16 terms per fp32 tile)",
                "bound": "mfma", "achieved": tf, "peak": peak, "unit": "TFLOP/s",
                "frac": tf / peak, "launches_per_step": n_conv, "flop_per_step": flops,
                "traffic": None if per_launch is None else per_launch * n_conv,
                "counters": counters_of("conv_h_kernel")}

    def counters_of(kernel):
        """MFMA-busy fraction of `kernel` from the committed SQ counter passes
        (SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / XCDs)), or None."""
        try:
            ks = json.loads(Path(args.counters_json).read_text())["kernels"]
            # the full templated name (field_r_kernel<sdfr::NgpNet> and
            # field_p_kernel<sdfr::SirenNet> are different kernels)
            k = next(v for n, v in ks.items() if kernel in n.replace("sdfr::(anonymous namespace)::", ""))
            return {"mfma_busy_frac": k["mfma_busy_frac"],
                    "effective_clock_GHz": k["effective_clock_GHz"],
                    "source": str(Path(args.counters_json).relative_to(REPO))}
        except (OSError, KeyError, ValueError, TypeError, StopIteration):
            return None
    if f16x3:
        # fp32-accurate GEMMs as 3 fp16 MFMA terms: the attainable fp32-equivalent
        # peak is the dense fp16 MFMA peak / 3.  `achieved` /
        # `frac` count the FLOPs the kernel EXECUTES (ngp: input_linear and
        # pts_linears.0 composed into one layer, 417,792 FLOP/sample) -- the hardware
        # utilisation; `algorithmic_equivalent` prices the same time at SURVEY.md
        # §8(d)'s per-sample FLOPs of the reference's network (550,912)
        ref_flop = flop if siren else FLOP_PER_SAMPLE
        alg_tflops = field_tflops * ref_flop / flop
        peak = MFMA_F16_PEAK_TFLOPS / 3
        roof = {"kernel": f"{field_kernel} (MLP as 3 split-fp16 {field_mfma} "
                          "terms per fp32 tile + compositing)",
                "bound": "mfma", "achieved": field_tflops, "peak": peak,
                "unit": "TFLOP/s", "frac": field_tflops / peak,
                "traffic": traffic, "flop_per_sample": flop,
                "algorithmic_equivalent": {"flop_per_sample": ref_flop, "achieved": alg_tflops,
                                           "frac": alg_tflops / peak},
                "mfma_dtype": "f16 (hi/lo split, fp32 accumulate)",
                "mfma_issued_tflops": 3 * field_tflops, "mfma_peak_dtype": MFMA_F16_PEAK_TFLOPS,
                "counters": counters_of(field_kernel)}
        clk = (roof["counters"] or {}).get("effective_clock_GHz")
        if clk:
            # the same time against the peak at the clock the chip holds under this body
            # (committed GRBM_GUI_ACTIVE pass; the headline frac stays at 2.4 GHz)
            roof["frac_at_measured_clock"] = roof["frac"] * MFMA_CLOCK_GHZ / clk
    else:
        roof = {"kernel": "ngp_field_kernel (MLP on v_mfma_f32_16x16x4_f32 + compositing)",
                "bound": "mfma", "achieved": field_tflops, "peak": MFMA_F32_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": field_tflops / MFMA_F32_PEAK_TFLOPS,
                "traffic": traffic, "mfma_dtype": "f32"}

    faces = world * B * args.steps
    line = {
        "metric": METRIC,
        "value": faces / elapsed,
        "unit": "faces/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (random z, random cameras, random-init weights)",
        "config": {"workload": ("eval.py generation, SirenGenerator renderer (type 'sdf', "
                                "configs[4]'s generator)") if siren and not fc else
                               ("eval.py generation, FCGenerator renderer (rendering.fc = 1, "
                                "configs[4]'s plain Fourier MLP)") if fc else
                               "eval.py 5000-image generation (ffhq_256_sdf_ngp, configs[1])",
                   "faces_per_step_per_gpu": B, "renderer": f"{res}x{res} rays x {N} samples",
                   "output": "256x256 RGB", "parallelism": f"dp{world} (independent faces)",
                   "field_precision": args.field_precision},
        "roofline": roof,
        "roofline_gather": None if siren else {
            "kernel": "ngp_encode_kernel (sampling + 16-level hash-grid gather)",
            "bound": "hbm", "achieved": gather_gbps, "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": gather_gbps / HBM_PEAK_GBPS,
            "traffic": traffic_of("ngp_encode_kernel")},
        "roofline_decoder": decoder_roofline(),
        "stage_ms_per_step": {"renderer_total": render_ms, "hash_grid": enc_ms,
                              "field": field_ms, "decoder_regular_convs": conv_ms},
        "cpu_baseline": None,
    }
    if not args.no_extras:
        gg = sdfr.GraphedGenerator(g)

        def graphed_step(nb):
            # latents, cameras, sampling offsets and noise drawn inside the graph
            return gg.random_faces(nb, res, azim_range=opt.camera.azim,
                                   elev_range=opt.camera.elev, fov_ang=opt.camera.fov,
                                   dist_radius=opt.camera.dist_radius)[0]
        line["extras"] = extras(step, B, graphed_step, g)
        if f16x3 and not siren:
            # the exact-fp32 field (v_mfma_f32_16x16x4_f32) on the same workload: the
            # cost of exact arithmetic, outside the timed region
            g.renderer.field_precision = "fp32"
            for _ in range(2):
                step()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            for e in ev:
                e.record()          # materialise the handles (as for the timed steps)
            torch.cuda.synchronize()
            g.renderer.stage_events = ev[:4]
            g.renderer.field_event = ev[4]
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            g.renderer.stage_events = None
            g.renderer.field_event = None
            g.renderer.field_precision = args.field_precision
            f32_ms = ev[4].elapsed_time(ev[3])
            # ngp_field_kernel runs the uncomposed network (input_linear, then
            # pts_linears.0): the reference's 550,912 FLOP/sample
            line["extras"]["fp32_field"] = {
                "kernel": "ngp_field_kernel (v_mfma_f32_16x16x4_f32)", "faces_per_s": B / dt,
                "field_ms": f32_ms, "flop_per_sample": FLOP_PER_SAMPLE,
                "field_tflops": FLOP_PER_SAMPLE * samples / (f32_ms * 1e-3) / 1e12,
                "peak_tflops": MFMA_F32_PEAK_TFLOPS}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, siren and not fc, fc)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
