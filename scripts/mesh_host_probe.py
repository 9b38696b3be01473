import sys, time, torch
sys.path.insert(0, "/root/repo")
from sdfr_loader import load
sdfr = load()
dev = "cuda:0"
res = 256
opt = sdfr.vol_render_opt()
opt.model.renderer_spatial_output_dim = res
opt.rendering.N_samples = res
opt.rendering.return_sdf = True
opt.rendering.return_xyz = True
torch.manual_seed(0)
g = sdfr.Generator(opt.model, opt.rendering, full_pipeline=False).to(dev).eval()
g.renderer.rng_device = "device"
ext, focal, near, far, _ = sdfr.generate_camera_params(res, dev, batch=1)
z = torch.randn(1, 256, device=dev)
with torch.no_grad():
    for r in range(4):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        out = g([z], ext, focal, near, far, return_sdf=True, return_xyz=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize(); t2 = time.perf_counter()
        vol = sdfr.align_volume(out[3]); torch.cuda.synchronize(); t3 = time.perf_counter()
        print(f"launch {1e3*(t1-t0):.1f} ms, gpu-wait {1e3*(t2-t1):.1f} ms, align {1e3*(t3-t2):.1f} ms", flush=True)
    import cProfile, pstats
    pr = cProfile.Profile(); pr.enable()
    out = g([z], ext, focal, near, far, return_sdf=True, return_xyz=True); torch.cuda.synchronize()
    pr.disable(); pstats.Stats(pr).sort_stats("cumulative").print_stats(18)
