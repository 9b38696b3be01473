"""The torch.library ops (sdface-gan_amd/ops.py) on the GPU: torch.library.opcheck (schema
/ no input mutation, FakeTensor outputs against the real ones, AOT dispatch), and the
renderer's registered-op path against its direct library call, bit for bit."""
import numpy as np
import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CHECKS = ("test_schema", "test_faketensor", "test_aot_dispatch_dynamic")


class _Record(TorchDispatchMode):
    """Records the arguments of one op call (the renderer builds them)."""

    def __init__(self, op):
        super().__init__()
        self.op, self.args = op, None

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        if func is self.op:
            self.args = args
        return func(*args, **(kwargs or {}))


@pytest.fixture(scope="module")
def grid(sdfr):
    torch.manual_seed(0)
    enc = sdfr.GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                           log2_hashmap_size=19, desired_resolution=4096).to(DEV)
    enc.embeddings.data.uniform_(-1, 1)
    x = torch.rand(3000, 3, device=DEV)
    return enc, x, float(np.log2(enc.per_level_scale))


@pytest.mark.parametrize("dy", [False, True])
def test_opcheck_grid_encode(sdfr, grid, dy):
    enc, x, S = grid
    args = (x, enc.embeddings.detach(), enc.offsets, S, 16, dy, 0, False, 0)
    torch.library.opcheck(torch.ops.sdfr.grid_encode_forward.default, args, test_utils=CHECKS)
    out, dydx = torch.ops.sdfr.grid_encode_forward(*args)
    g = torch.randn_like(out)
    for want_table in (True, False) if dy else (True,):
        bargs = (g, x, enc.embeddings.detach(), enc.offsets, dydx, S, 16, want_table, 0, False, 0)
        torch.library.opcheck(torch.ops.sdfr.grid_encode_backward.default, bargs,
                              test_utils=("test_schema", "test_faketensor"))


def test_grid_encoder_module_through_op(sdfr, grid):
    """GridEncoder.forward / backward go through the registered ops: gradients of the
    table and the inputs match a direct call of those ops."""
    enc, x, S = grid
    xi = x.clone().requires_grad_(True)
    out = enc(xi * 2 - 1, bound=1)
    g = torch.randn_like(out)
    out.backward(g)
    o2, dydx = torch.ops.sdfr.grid_encode_forward(((xi * 2 - 1) + 1) / 2, enc.embeddings.detach(),
                                                  enc.offsets, S, 16, True, 0, False, 0)
    assert torch.equal(out.detach(), o2.permute(1, 0, 2).reshape(out.shape))
    ge, gi = torch.ops.sdfr.grid_encode_backward(
        g.view(-1, 16, 2).permute(1, 0, 2).contiguous(), ((xi.detach() * 2 - 1) + 1) / 2,
        enc.embeddings.detach(), enc.offsets, dydx, S, 16, True, 0, False, 0)
    # (the table gradient is a sum over samples in hardware atomic order, as the
    # reference's atomicAdd: equal up to fp32 reassociation)
    err = (enc.embeddings.grad - ge).abs().max() / ge.abs().max()
    assert err <= 1e-5, err
    assert torch.equal(xi.grad, gi)     # d/dxi of (2 xi - 1 + 1) / 2 is exactly 1


def test_opcheck_sh_encode(sdfr):
    torch.manual_seed(1)
    d = torch.nn.functional.normalize(torch.randn(777, 3, device=DEV), dim=-1)
    torch.library.opcheck(torch.ops.sdfr.sh_encode_forward.default, (d, 4, True),
                          test_utils=CHECKS)
    out, dydx = torch.ops.sdfr.sh_encode_forward(d, 4, True)
    torch.library.opcheck(torch.ops.sdfr.sh_encode_backward.default,
                          (torch.randn_like(out), d, dydx, 4), test_utils=CHECKS)


@pytest.mark.parametrize("net,flags", [("ngp", {}), ("ngp", dict(return_sdf=True, return_xyz=True)),
                                       ("siren", {}), ("fc", {})])
def test_render_op_matches_direct_call(sdfr, net, flags):
    """VolumeFeatureRenderer's plain call (sdfr::render_fused) against the same render
    through the direct library call (taken when stage events are set): identical."""
    opt = sdfr.vol_render_opt(ngp=net == "ngp", fc=net == "fc")
    r = opt.rendering
    for k, v in flags.items():
        r[k] = v
    torch.manual_seed(3)
    ren = sdfr.VolumeFeatureRenderer(r, style_dim=256, out_im_res=16).to(DEV).eval()
    cam, focal, near, far, _ = sdfr.generate_camera_params(16, DEV, batch=2)
    styles = torch.randn(2, 256, device=DEV)
    t_rand = torch.rand(2, 16, 16, device=DEV)
    with torch.no_grad():
        rec = _Record(torch.ops.sdfr.render_fused.default)
        with rec:
            a = ren(cam, focal, near, far, styles=styles, t_rand=t_rand)
        assert rec.args is not None, "the plain call did not go through sdfr::render_fused"
        ren.stage_events = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        b = ren(cam, focal, near, far, styles=styles, t_rand=t_rand)
        ren.stage_events = None
    torch.cuda.synchronize()
    for x, y in zip(a[:5], b[:5]):
        assert (x is None) == (y is None)
        if x is not None:
            assert torch.equal(x, y)
    args = tuple([t.detach() for t in v] if isinstance(v, list) and v and
                 isinstance(v[0], torch.Tensor) else v for v in rec.args)
    torch.library.opcheck(torch.ops.sdfr.render_fused.default, args,
                          test_utils=("test_schema", "test_faketensor"))
