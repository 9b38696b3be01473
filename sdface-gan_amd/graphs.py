"""HIP-graph replay of the whole inference forward (no reference counterpart).

eval.py generates one face per ``Generator.forward`` call (``eval.py:92-113``,
batch 1).  At that size the GPU work is ~1.5 ms and the host's per-call launch
cost (mapping MLP, camera-free renderer launch, decoder layers) is comparable,
so ``GraphedGenerator`` captures the complete forward -- mapping, fused renderer,
fused decoder, decoder noise and the per-ray sampling offsets drawn from the
device RNG -- once per batch size into a ``torch.cuda.CUDAGraph`` and replays it
with the caller's latents and cameras copied into static input buffers.
Replays produce bit-identical images to the eager forward on the same inputs
(``tests/test_gpu_render.py::test_graphed_generator_matches_eager``); random
draws inside the graph (noise, sampling offsets) advance the device generator
on every replay as they do eagerly.

Requirements: the generator is on a CUDA device in eval mode, takes the fused
paths (no autograd), and its renderer draws sampling offsets on the device
(``renderer.rng_device = "device"``; the reference-compatible host draw would be
a pageable copy inside the graph).

Weight updates: a graph freezes the kernels' pointer arguments and the decoder's
packed / stacked weight caches.  Every call compares each parameter's and
buffer's (data_ptr, version) with the values at capture -- an EMA step,
``load_state_dict`` or a moved tensor changes them -- and re-captures when they
differ, so a replay never mixes a new renderer with a stale decoder.
"""
from __future__ import annotations

import torch


class GraphedGenerator:
    """``GraphedGenerator(g)(z, cam, focal, near, far) -> (rgb, thumb)``, or
    ``GraphedGenerator(g).random_faces(B) -> (rgb, thumb)`` with the latents and
    cameras drawn inside the graph too.

    Same arguments as ``Generator.forward`` for the eval use (one style tensor,
    truncation / truncation_latent fixed at construction); one graph per batch
    size, captured on first use.  Outputs live in the graph's static buffers and
    are overwritten by the next replay of the same batch size: copy them to keep
    them (eval.py moves each image to the host right away)."""

    def __init__(self, generator, truncation=1, truncation_latent=None, randomize_noise=True):
        p = next(generator.parameters())
        if not p.is_cuda:
            raise RuntimeError("GraphedGenerator needs the generator on a GPU")
        if generator.training:
            raise RuntimeError("GraphedGenerator needs generator.eval()")
        if generator.renderer.rng_device != "device":
            raise RuntimeError("GraphedGenerator needs renderer.rng_device = 'device' "
                               "(sampling offsets drawn inside the graph)")
        self.g = generator
        self.device = p.device
        self.kw = dict(truncation=truncation, truncation_latent=truncation_latent,
                       randomize_noise=randomize_noise)
        self._graphs = {}
        self._tensors = list(generator.parameters()) + list(generator.buffers())
        self._wkey = None

    def _weights_key(self):
        return tuple((t.data_ptr(), t._version) for t in self._tensors)

    def _check_weights(self):
        """Drop every captured graph when a parameter or buffer changed since capture."""
        key = self._weights_key()
        if key != self._wkey:
            self._graphs.clear()
            self._tensors = list(self.g.parameters()) + list(self.g.buffers())
            self._wkey = self._weights_key()

    def _capture(self, B):
        dev = self.device
        static = {"z": torch.zeros(B, self.g.style_dim, device=dev),
                  "cam": torch.zeros(B, 3, 4, device=dev),
                  "focal": torch.ones(B, 1, 1, device=dev),
                  "near": torch.full((B, 1, 1), 0.88, device=dev),
                  "far": torch.full((B, 1, 1), 1.12, device=dev)}
        static["cam"][:, :, :3] = torch.eye(3, device=dev)
        static["cam"][:, 2, 3] = 1.0

        def fwd():
            with torch.no_grad():
                return self.g([static["z"]], static["cam"], static["focal"], static["near"],
                              static["far"], **self.kw)

        graph, out = self._record(fwd)
        return graph, static, out

    def random_faces(self, B, resolution=64, **camera_kw):
        """B faces from fresh latents z ~ N(0, 1) and cameras drawn by
        generate_camera_params(resolution, **camera_kw) -- eval.py's whole
        per-image loop body -- with the draws inside the graph as well."""
        for k, v in camera_kw.items():
            if isinstance(v, torch.Tensor):
                raise TypeError(f"random_faces: camera_kw[{k!r}] is a tensor; a graph freezes "
                                "it -- pass plain numbers (or call the graphed forward with "
                                "explicit cameras)")
        self._check_weights()
        key = ("random", B, resolution, tuple(sorted(camera_kw.items())))
        if key not in self._graphs:
            from .camera import generate_camera_params

            def fwd():
                z = torch.randn(B, self.g.style_dim, device=self.device)
                cam, focal, near, far, _ = generate_camera_params(resolution, self.device,
                                                                  batch=B, **camera_kw)
                with torch.no_grad():
                    return self.g([z], cam, focal, near, far, **self.kw)

            self._graphs[key] = self._record(fwd)
        graph, out = self._graphs[key]
        graph.replay()
        return out

    def _record(self, fwd):
        """Warm up on a side stream (first calls pack decoder weights and pick
        paths), then capture one call of fwd."""
        dev = self.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                fwd()
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = fwd()
        self._wkey = self._weights_key()          # caches as packed by the warm-up calls
        return graph, out

    def __call__(self, z, cam_poses, focals, near, far):
        B = z.shape[0]
        self._check_weights()
        if B not in self._graphs:
            self._graphs[B] = self._capture(B)
        graph, static, out = self._graphs[B]
        static["z"].copy_(z)
        static["cam"].copy_(cam_poses)
        for k, v in (("focal", focals), ("near", near), ("far", far)):
            v = torch.as_tensor(v, dtype=torch.float32, device=self.device)
            static[k].copy_(v.reshape(-1, 1, 1).expand(B, 1, 1))
        graph.replay()
        return out
