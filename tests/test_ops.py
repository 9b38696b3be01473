"""torch.library registration of the hot-path ops (sdface-gan_amd/ops.py):
schemas, FakeTensor shape propagation and the reference's device errors, on the CPU.
The ops' results are checked on the GPU (tests/test_gpu_ops.py)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode


@pytest.fixture(scope="module")
def ops(sdfr):
    import importlib
    return importlib.import_module(sdfr.__name__ + ".ops")


def test_ops_registered(ops):
    names = {"grid_encode_forward", "grid_encode_backward", "sh_encode_forward",
             "sh_encode_backward", "render_fused"}
    for n in names:
        assert hasattr(torch.ops.sdfr, n), n
    s = str(torch.ops.sdfr.grid_encode_forward.default._schema)
    assert s.startswith("sdfr::grid_encode_forward(Tensor inputs, Tensor embeddings, "
                        "Tensor offsets, float S")
    assert "Tensor? t_rand" in str(torch.ops.sdfr.render_fused.default._schema)


def test_grid_encode_fake_shapes(ops):
    with FakeTensorMode():
        x = torch.empty(100, 3)
        emb = torch.empty(6328848, 2)
        off = torch.empty(17, dtype=torch.int32)
        out, dy = torch.ops.sdfr.grid_encode_forward(x, emb, off, 0.533, 16, True, 0, False, 0)
        assert out.shape == (16, 100, 2) and dy.shape == (100, 96)
        out, dy = torch.ops.sdfr.grid_encode_forward(x, emb, off, 0.533, 16, False, 0, False, 0)
        assert dy.numel() == 0
        g = torch.empty(16, 100, 2)
        ge, gi = torch.ops.sdfr.grid_encode_backward(g, x, emb, off, torch.empty(100, 96), 0.533,
                                                     16, True, 0, False, 0)
        assert ge.shape == emb.shape and gi.shape == x.shape
        ge, gi = torch.ops.sdfr.grid_encode_backward(g, x, emb, off, torch.empty(0), 0.533, 16,
                                                     False, 0, False, 0)
        assert ge.numel() == 0 and gi.numel() == 0


def test_sh_encode_fake_shapes(ops):
    with FakeTensorMode():
        d = torch.empty(50, 3)
        out, dy = torch.ops.sdfr.sh_encode_forward(d, 4, True)
        assert out.shape == (50, 16) and dy.shape == (50, 48)
        gi = torch.ops.sdfr.sh_encode_backward(torch.empty(50, 16), d, dy, 4)
        assert gi.shape == d.shape


@pytest.mark.parametrize("flags,shapes", [
    (dict(output_features=1, return_sdf=1, return_xyz=1),
     [(2, 3, 8, 8), (2, 256, 8, 8), (2, 8, 8, 24, 1), (2, 1, 8, 8), (2, 3, 8, 8)]),
    (dict(output_features=1, return_sdf=0, return_xyz=0),
     [(2, 3, 8, 8), (2, 256, 8, 8), (0,), (0,), (0,)]),
])
def test_render_fused_fake_shapes(ops, sdfr, flags, shapes):
    opt = sdfr.vol_render_opt()
    ren = sdfr.VolumeFeatureRenderer(opt.rendering, style_dim=256, out_im_res=8)
    f = dict.fromkeys(ops.RENDER_FLAGS, 0)
    f.update(flags)
    ts = ren._weight_tensors(0)
    fs, is_ = ren._weight_scalars(0)
    with FakeTensorMode(allow_non_fake_inputs=True) as m:
        fake = [m.from_tensor(t.detach()) for t in ts]
        out = torch.ops.sdfr.render_fused(
            0, fake, torch.empty(2, 3, 4), torch.empty(2), torch.empty(2), torch.empty(2),
            torch.empty(2, 256), None, None, torch.empty(8), torch.empty(8), torch.empty(24),
            None, fs, is_, [f[k] for k in ops.RENDER_FLAGS], 8, 8, 24)
    assert [tuple(o.shape) for o in out] == shapes


def test_weight_tensors_order(sdfr):
    """The flat list feeds ops.weights_struct positionally: its length per network."""
    opt = sdfr.vol_render_opt()
    ren = sdfr.VolumeFeatureRenderer(opt.rendering, style_dim=256, out_im_res=8)
    assert len(ren._weight_tensors(0)) == 4 + 6 * 3 + 6 + 4 + 1
    assert ren._weight_tensors(0)[0] is ren.network.encoder.embeddings
    assert ren._weight_tensors(0)[-1] is ren.sigmoid_beta


def test_ops_raise_on_host_tensors(ops):
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        torch.ops.sdfr.grid_encode_forward(torch.zeros(4, 3), torch.zeros(10, 2),
                                           torch.zeros(17, dtype=torch.int32), 0.5, 16, False,
                                           0, False, 0)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        torch.ops.sdfr.sh_encode_forward(torch.zeros(4, 3), 4, False)
