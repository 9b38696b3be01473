"""BASELINE configs[3]: sdf_mesh.py's SDF volume for marching cubes, on 1 GPU.

Times the surface-extraction Generator (full_pipeline=False, return_sdf/xyz;
sdf_mesh.py:244-252) at 128^2 rays x 128 samples (the reference setting) and at
256^2 x 256 (a 256^3 volume, 16.8 M samples), one face per call as sdf_mesh.py
does, plus align_volume ("ms_per_volume"); then the whole mesh step of
sdf_mesh.py:160-182 -- volume, align_volume and extract_mesh_with_marching_cubes
(GPU marching cubes, vertex scaling/flips, mesh copied to the host) --
("ms_per_mesh"; at the volume's median level, since a random-init SDF has no zero
crossing).  Prints one JSON line per resolution."""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402


def main(reps=5):
    sdfr = load()
    dev = "cuda:0"
    for res in (128, 256):
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
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        for e in evs:
            e.record()
        g.renderer.stage_events = evs[:4]
        g.renderer.field_event = evs[4]          # right before the field kernel
        times, field = [], []
        with torch.no_grad():
            for r in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = g([z], ext, focal, near, far, return_sdf=True, return_xyz=True)
                vol = sdfr.align_volume(out[3])
                torch.cuda.synchronize()
                if r:
                    times.append(time.perf_counter() - t0)
                    field.append(evs[4].elapsed_time(evs[3]))
        ms = sorted(times)[len(times) // 2] * 1e3
        fms = sorted(field)[len(field) // 2]
        g.renderer.stage_events = None
        g.renderer.field_event = None
        mtimes = []
        with torch.no_grad():
            for r in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = g([z], ext, focal, near, far, return_sdf=True, return_xyz=True)
                vol = sdfr.align_volume(out[3])
                # extract_mesh_with_marching_cubes's steps at the volume's median level:
                # a random-init SDF (no sphere init) has no zero crossing
                v3 = vol[0, ..., 0].permute(1, 0, 2)
                verts, faces = sdfr.marching_cubes(v3, float(v3.median()))
                for axis, size in enumerate((vol.shape[2], vol.shape[1], vol.shape[3])):
                    verts[:, axis] = (verts[:, axis] / float(size) - 0.5) * 0.24
                verts[:, 1:] *= -1
                mesh = sdfr.Mesh(verts.cpu().numpy(), faces.cpu().numpy())
                if r:
                    mtimes.append(time.perf_counter() - t0)
        mms = sorted(mtimes)[len(mtimes) // 2] * 1e3
        samples = res * res * res
        print(json.dumps({"config": f"sdf_mesh surface extraction {res}^2 rays x {res} samples "
                                    f"({res}^3 SDF volume), 1 face per call",
                          "ms_per_volume": ms, "volumes_per_s": 1e3 / ms,
                          "field_ms": fms, "ms_per_mesh": mms,
                          "mesh_vertices": int(mesh.vertices.shape[0]),
                          "mesh_faces": int(mesh.faces.shape[0]),
                          "field_tflops": 417792 * samples / fms / 1e9,
                          "volume_shape": list(vol.shape)}), flush=True)
        del g, out, vol
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
