"""The training GEMMs' autograd structure (sdface-gan_amd/linear.py) on the CPU: the
kernel entry points are replaced by torch restatements of what they compute, so these
tests check the routing, the padding, the first-order backward, the double backward
that the SIREN eikonal loss needs (sdf_model.py:224-229, create_graph=True) and the
per-graph skipping of unused gradients -- against the same network on F.linear /
torch.sin (the reference's ops).  The kernels' numerics are tests/test_gpu_linear.py's.
"""
import importlib

import pytest
import torch

from sdfr_loader import load

sdfr = load()
lin = importlib.import_module(sdfr.__name__ + ".linear")


@pytest.fixture()
def cpu_kernels(monkeypatch):
    L = lin
    calls = {"wgrad": 0, "gemm": 0, "film_fwd": 0, "film_bwd": 0, "film_bwd2": 0, "head_bwd": 0}

    def pack(w, transposed):
        return (w.t() if transposed else w).contiguous()      # B [N, K]

    def gemm(x2, B, bias, N):
        calls["gemm"] += 1
        assert x2.shape[1] == B.shape[1] and B.shape[0] == N
        assert x2.shape[1] % 4 == 0 and N % 16 == 0           # the kernels' shape rules
        out = x2 @ B.t()
        return out + bias if bias is not None else out

    def wgrad(gy2, x2):
        calls["wgrad"] += 1
        assert gy2.shape[1] == 256 and x2.shape[1] % 4 == 0 and x2.shape[1] <= 288
        return gy2.t() @ x2

    def film_fwd(x2, B, bias, g2, b2, N):
        calls["film_fwd"] += 1
        F_ = g2.shape[0]
        y = x2 @ B.t() + bias
        yf = y.view(F_, -1, N)
        return torch.sin(g2[:, None] * yf + b2[:, None]).reshape(-1, N), y

    def film_bwd(ds2, y, g2, b2):
        calls["film_bwd"] += 1
        F_, N = g2.shape
        dsf, yf = ds2.view(F_, -1, N), y.view(F_, -1, N)
        du = dsf * torch.cos(g2[:, None] * yf + b2[:, None])
        dy = du * g2[:, None]
        return dy.reshape(-1, N), (du * yf).sum(1), du.sum(1), dy.sum(1)

    def film_bwd2(ds2, y, g2, b2, gdy, gdg, gdb):
        # sdfr_film_backward_grad's formulas (include/sdfr.h), checked here against
        # autograd of the reference's ops through the whole double backward
        calls["film_bwd2"] += 1
        F_, N = g2.shape
        dsf, yf = ds2.view(F_, -1, N), y.view(F_, -1, N)
        gm, bt = g2[:, None], b2[:, None]
        u = gm * yf + bt
        cu, su = torch.cos(u), torch.sin(u)
        gd = gdy.view(F_, -1, N) if gdy is not None else torch.zeros_like(dsf)
        gg = gdg[:, None] if gdg is not None else torch.zeros_like(gm)
        gb = gdb[:, None] if gdb is not None else torch.zeros_like(gm)
        h = gd * gm + gg * yf + gb
        dU = -h * dsf * su
        d_ds = h * cu
        d_y = dU * gm + gg * dsf * cu
        return (d_ds.reshape(-1, N), d_y.reshape(-1, N), (dU * yf + gd * dsf * cu).sum(1),
                dU.sum(1))

    def head_fwd(x2, w, bias):
        out = x2 @ w.t()
        return out + bias if bias is not None else out

    def head_bwd(gy2, x2, w, nx, nw, nb):
        calls["head_bwd"] += 1
        return (gy2 @ w if nx else None, gy2.t() @ x2 if nw else None,
                gy2.sum(0) if nb else None)

    for k, v in dict(_pack=pack, _gemm=gemm, _wgrad=wgrad, _film_fwd=film_fwd, _film_bwd=film_bwd,
                     _film_bwd2=film_bwd2, _head_fwd=head_fwd, _head_bwd=head_bwd,
                     _on_device=lambda x: True).items():
        monkeypatch.setattr(L, k, v)
    return calls


def _nets(seed=0, D=3):
    torch.manual_seed(seed)
    a = sdfr.SirenGenerator(D=D, W=256, style_dim=256)
    torch.manual_seed(seed)
    b = sdfr.SirenGenerator(D=D, W=256, style_dim=256)
    for m in b.modules():
        if hasattr(m, "train_kernels"):
            m.train_kernels = False                          # the reference's ops
    return a, b


def _loss(net, pts, views, styles, eik_weight):
    """thumb-like mean + surface term + the eikonal loss through create_graph."""
    pts = pts.clone().requires_grad_(True)
    out = net(torch.cat([pts, views], -1), styles)
    rgb, sdf = out[..., :3], out[..., 3:4]
    eik = torch.autograd.grad(sdf, pts, torch.ones_like(sdf), create_graph=True)[0]
    eik_loss = ((eik.norm(dim=-1) - 1) ** 2).mean()
    return rgb.mean() + torch.exp(-10 * sdf.abs()).mean() + eik_weight * eik_loss, eik


def test_siren_double_backward_matches_reference_ops(cpu_kernels):
    a, b = _nets()
    torch.manual_seed(1)
    F_, R, S = 2, 8, 64                                      # 1024 rows: routed
    pts = torch.rand(F_, R, S, 3) * 2 - 1
    views = torch.nn.functional.normalize(torch.randn(F_, R, S, 3), dim=-1)
    styles = torch.randn(F_, 256)
    la, ea = _loss(a, pts, views, styles, 0.1)
    lb, eb = _loss(b, pts, views, styles, 0.1)
    assert cpu_kernels["film_fwd"] > 0 and cpu_kernels["gemm"] > 0
    torch.testing.assert_close(ea, eb, rtol=1e-4, atol=1e-5)
    la.backward()
    lb.backward()
    assert cpu_kernels["film_bwd2"] > 0                      # the second-order FiLM op ran
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=1e-6)
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert pa.grad is not None, n
        scale = pb.grad.abs().max().clamp_min(1e-12)
        err = ((pa.grad - pb.grad).abs().max() / scale).item()
        assert err < 1e-4, f"{n}: {err:.2e}"


def test_eikonal_pass_skips_weight_gradients(cpu_kernels):
    """autograd.grad(sdf, pts) runs no weight-gradient GEMM (per graph task), while the
    following loss.backward() computes all of them."""
    a, _ = _nets(D=2)
    torch.manual_seed(2)
    pts = (torch.rand(2, 8, 64, 3) * 2 - 1).requires_grad_(True)
    views = torch.nn.functional.normalize(torch.randn(2, 8, 64, 3), dim=-1)
    out = a(torch.cat([pts, views], -1), torch.randn(2, 256))
    sdf = out[..., 3:4]
    before = cpu_kernels["wgrad"]
    eik = torch.autograd.grad(sdf, pts, torch.ones_like(sdf), create_graph=True)[0]
    assert cpu_kernels["wgrad"] == before
    ((eik.norm(dim=-1) - 1) ** 2).mean().backward()
    assert cpu_kernels["wgrad"] > before
    assert all(p.grad is not None for n, p in a.named_parameters()
               if n.startswith("pts_linears") and n.endswith("weight") and "gamma" not in n
               and "beta" not in n)


def test_padded_shapes_route_and_match(cpu_kernels):
    """In features 3 (SIREN layer 0), 259 (views), 60 / 280 (FCGenerator x_in / views)
    and 1 (a head's transposed weight) take the kernels with zero padding; gradients
    equal F.linear's."""
    torch.manual_seed(3)
    for K in (3, 60, 259, 268, 272, 280):
        x = torch.randn(1024, K, requires_grad=True)
        w = torch.randn(256, K, requires_grad=True)
        bias = torch.randn(256, requires_grad=True)
        y = lin.linear(x, w, bias)
        y2 = torch.nn.functional.linear(x.detach().requires_grad_(True), w.detach().requires_grad_(True),
                                        bias.detach().requires_grad_(True))
        torch.testing.assert_close(y, y2, rtol=1e-5, atol=1e-5)
        g = torch.randn_like(y)
        gx, gw, gb = torch.autograd.grad(y, (x, w, bias), g)
        assert gx.shape == x.shape and gw.shape == w.shape
        torch.testing.assert_close(gx, g @ w.detach(), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(gw, g.t() @ x.detach(), rtol=1e-4, atol=1e-3)
    w = torch.randn(256, 292)
    assert not lin._routable(torch.randn(1024, 292), w)      # input gradient would exceed 288
    w = torch.randn(256, 100)
    assert not lin._routable(torch.randn(1024, 100), w)      # 64 < K < 256: no such kernel


def test_single_backward_layer_refuses_double_backward(cpu_kernels):
    """A layer routed with twice=False (the ngp network's) computes its backward on the
    kernels; run with create_graph its gradients are marked like once_differentiable's,
    so differentiating them again raises instead of silently dropping the second-order
    term -- while first-order use under create_graph still works."""
    torch.manual_seed(5)
    x = torch.randn(1024, 256, requires_grad=True)
    w = torch.randn(256, 256, requires_grad=True)
    y = lin.linear(x, w, None, True, False)
    assert "LinearF16x3" in type(y.grad_fn).__name__
    gx = torch.autograd.grad(y.square().sum(), x, create_graph=True)[0]
    torch.testing.assert_close(gx.detach(), (2 * y.detach()) @ w.detach(), rtol=1e-4, atol=1e-3)
    with pytest.raises(RuntimeError, match="differentiate twice"):
        gx.sum().backward()
    # the twice=True route stays differentiable
    y2 = lin.linear(x, w, None, True, True)
    gx2 = torch.autograd.grad(y2.square().sum(), x, create_graph=True)[0]
    gx2.sum().backward()
    assert w.grad is not None
