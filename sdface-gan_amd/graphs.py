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

import operator
import weakref
from collections import OrderedDict

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


_PLAIN = (bool, int, float, str, type(None))
_VERSION = operator.attrgetter("_version")
_DATA_PTR = torch.Tensor.data_ptr


def _plain_config(m):
    """A module's public plain-valued attributes (flags such as rng_device,
    field_precision, use_fused, N_samples): anything that can change which kernels
    a forward enqueues or with which constants."""
    return tuple([(k, v) for k, v in m.__dict__.items() if k[0] != "_" and isinstance(v, _PLAIN)])


def _arg_key(v):
    """Shape / dtype / device of a tensor argument (its values are copied into the
    graph's static input per call); the value itself of a plain number (baked in)."""
    if isinstance(v, torch.Tensor):
        return ("t", tuple(v.shape), v.dtype, v.device)
    return ("v", v)


class ForwardGraphCache:
    """``Generator.forward``'s own HIP-graph replay of repeated inference calls, so
    that an UNCHANGED caller -- eval.py's loop of one ``model([z], cam, focal, near,
    far, truncation=1, truncation_latent=None)`` per image (eval.py:87-104) -- gets the
    graph rate without wrapping the model in ``GraphedGenerator``.

    A call is served from a graph when the generator is in eval mode, no gradient is
    recorded, the inputs are on the GPU, the call is the plain image forward (one
    style tensor, no explicit noise / inject_index / t_rand, no latents or eikonal
    returned) and the renderer takes its fused path; and only once the same call key
    -- shapes, flags, every module's plain settings and every parameter's and
    buffer's (data_ptr, version) -- was seen on an earlier call, so a training loop
    whose weights change every step (or a one-off call) never pays for a capture.

    Same results, bit for bit, and the same random streams as the uncached path:
    the renderer's per-ray sampling offsets are drawn from the CPU generator per call
    exactly as the eager path draws them (``rng_device == "cpu"``, the reference's
    stream) and copied into the graph's static input through a pinned staging ring,
    or drawn inside the graph from the device generator (``"device"``); the decoder
    noise is drawn inside the graph; the CPU and device generator states are saved
    before the capture's warm-up and restored after it, so capturing consumes no
    random numbers.  Outputs are returned as fresh tensors (one device copy each),
    as the eager forward returns them: a later call never overwrites them.
    ``tests/test_gpu_render.py::test_forward_graph_cache_matches_uncached``."""

    max_graphs = 4

    def __init__(self):
        self.graphs = OrderedDict()
        self.seen = OrderedDict()
        self.wkey = None
        self.tensors = None
        self.ring = {}

    def eligible(self, g, styles, cam_poses, focals, near, far, kw):
        if g.training or torch.is_grad_enabled() or not cam_poses.is_cuda:
            return False
        for v in (focals, near, far):
            if isinstance(v, torch.Tensor) and v.device != cam_poses.device:
                return False                    # a host tensor: a copy the graph cannot hold
        if (kw["noise"] is not None or kw["inject_index"] is not None or kw["return_latents"]
                or kw["return_eikonal"] or kw["project_noise"] or kw["mesh_path"] is not None
                or kw["t_rand"] is not None):
            return False
        if not (isinstance(styles, (list, tuple)) and len(styles) == 1
                and isinstance(styles[0], torch.Tensor) and styles[0].is_cuda):
            return False
        r = g.renderer
        if (r.stage_events is not None or r.field_event is not None
                or (g.full_pipeline and g.decoder.conv_events is not None)):
            return False                        # per-call profiling events: eager
        if torch.cuda.is_current_stream_capturing():
            return False                        # inside a caller's own capture
        z = styles[0]
        # (the renderer's styles are the mapped latent [B, 256]: z stands in for it
        # whenever it has that shape, without an allocation per call)
        lat = z if kw["input_is_latent"] or (z.dim() == 2 and z.shape[1] == 256) else \
            z.new_empty(z.shape[0], 256)
        if not r._fused_ok(cam_poses, lat, False):
            return False
        return not g.full_pipeline or g.decoder.fused_ready(cam_poses.device)

    def _weights(self, g):
        if self.tensors is None:
            self.tensors = list(g.parameters()) + list(g.buffers())
        return tuple(map(_VERSION, self.tensors)), tuple(map(_DATA_PTR, self.tensors))

    def call_key(self, g, z, cam_poses, focals, near, far, kw):
        tl = kw["truncation_latent"]
        tl_key = None if tl is None else tuple(
            (t.data_ptr(), t._version) if isinstance(t, torch.Tensor) else t for t in tl)
        mods = (g, g.renderer) + ((g.decoder,) if g.full_pipeline else ())
        return ((_arg_key(z), _arg_key(cam_poses), _arg_key(focals), _arg_key(near),
                 _arg_key(far), kw["truncation"], tl_key, kw["input_is_latent"],
                 kw["randomize_noise"], kw["return_sdf"], kw["return_xyz"])
                + tuple(_plain_config(m) for m in mods))

    def _t_rand_shape(self, r, B):
        if not r.perturb:
            return None
        H = W = r.out_im_res
        return (B, H, W) if r.offset_sampling else (B, H, W, r.N_samples)

    def __call__(self, g, styles, cam_poses, focals, near, far, kw):
        """Replay (capturing first if due) and return the outputs, or None when this
        call should run eagerly (first sighting of its key)."""
        wkey = self._weights(g)
        if wkey != self.wkey:                   # new weights: every graph is stale
            self.graphs.clear()
            self.seen.clear()
            self.tensors = None
            self.wkey = self._weights(g)
        z = styles[0]
        key = self.call_key(g, z, cam_poses, focals, near, far, kw)
        entry = self.graphs.get(key)
        if entry is None:
            if key not in self.seen:
                self.seen[key] = True
                while len(self.seen) > 4 * self.max_graphs:
                    self.seen.popitem(last=False)
                return None
            entry = self._capture(g, key, z, cam_poses, focals, near, far, kw)
        else:
            self.graphs.move_to_end(key)
        graph, static, outs, shape = entry
        dev = cam_poses.device
        dst, src = [], []
        for name, v in (("z", z), ("cam", cam_poses), ("focal", focals), ("near", near),
                        ("far", far)):
            if name in static:
                dst.append(static[name])
                src.append(v)
        torch._foreach_copy_(dst, src, non_blocking=True)   # (one launch for the five)
        if shape is not None and g.renderer.rng_device == "cpu":
            # the eager path's draw (renderer._draw_t_rand), same CPU stream position;
            # staged through pinned memory so the copy does not block the host
            self._stage_t_rand(static["t_rand"], torch.rand(shape), dev)
        graph.replay()
        return tuple(o.clone() if isinstance(o, torch.Tensor) else o for o in outs)

    def _stage_t_rand(self, dst, host, dev):
        ring = self.ring.get(host.shape)
        if ring is None:
            ring = self.ring[host.shape] = [[[torch.empty(host.shape, pin_memory=True), None]
                                             for _ in range(2)], 0]
        slot = ring[0][ring[1] % 2]
        ring[1] += 1
        if slot[1] is not None:
            slot[1].synchronize()                # its previous copy has been consumed
        slot[0].copy_(host)
        dst.copy_(slot[0], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        slot[1] = ev

    def _capture(self, g, key, z, cam_poses, focals, near, far, kw):
        dev = cam_poses.device
        static = {}
        for name, v in (("z", z), ("cam", cam_poses), ("focal", focals), ("near", near),
                        ("far", far)):
            if isinstance(v, torch.Tensor):
                static[name] = v.detach().clone()
        args = {n: static.get(n, v) for n, v in (("z", z), ("cam", cam_poses),
                                                  ("focal", focals), ("near", near),
                                                  ("far", far))}
        shape = self._t_rand_shape(g.renderer, z.shape[0])
        ekw = dict(kw)
        if shape is not None and g.renderer.rng_device == "cpu":
            static["t_rand"] = torch.zeros(shape, device=dev)
            ekw["t_rand"] = static["t_rand"]

        def fwd():
            return g._forward_eager([args["z"]], args["cam"], args["focal"], args["near"],
                                    args["far"], **ekw)

        cpu_state = torch.get_rng_state()
        dev_state = torch.cuda.get_rng_state(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            fwd()                               # warm-up (caches are warm already)
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            outs = fwd()
        torch.set_rng_state(cpu_state)
        torch.cuda.set_rng_state(dev_state, dev)
        entry = (graph, static, outs, shape)
        self.graphs[key] = entry
        while len(self.graphs) > self.max_graphs:
            self.graphs.popitem(last=False)
        return entry


_FORWARD_CACHES = weakref.WeakKeyDictionary()


def forward_cache(g):
    """The generator's ForwardGraphCache (kept off the module: graphs do not deepcopy)."""
    c = _FORWARD_CACHES.get(g)
    if c is None:
        c = _FORWARD_CACHES[g] = ForwardGraphCache()
    return c
