"""GPU: the renderer MLP's training GEMMs on split-fp16 MFMA (csrc/linear_f16x3.hip,
linear.py) against float64 references of the same op, and the stage-1 gradients of a
whole renderer with the kernels on and off.

Accuracy bound, per output element: |got - exact| <= c * 2^-24 * sum_k |x_k w_k|
(the scale of an fp32 dot product's rounding), with c small; the PyTorch fp32
product on the same inputs is measured beside it."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
U = 2.0 ** -24


def _rand(shape, mag, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(*shape, generator=g)
    if mag == "rows":                       # per-row magnitudes 1e-8 .. 1e2
        x = x * 10.0 ** (torch.rand(shape[0], 1, generator=g) * 10 - 8)
    elif mag == "tiny":
        x = x * 1e-6
    return x


def _bound_check(name, got, exact, scale, c=32.0):
    err = (got.double().cpu() - exact).abs()
    bound = c * U * scale + 1e-30
    ratio = float((err / bound).max())
    assert ratio <= 1.0, f"{name}: max err / bound = {ratio:.3f}"
    return ratio


@pytest.mark.parametrize("M,N,K", [(4096, 256, 32), (3000, 256, 256), (2048, 256, 272),
                                   (1001, 256, 256), (2048, 256, 60), (2048, 256, 280)])
@pytest.mark.parametrize("mag", ["unit", "rows", "tiny"])
def test_linear_forward_and_backward_vs_float64(sdfr, M, N, K, mag):
    from sdface_gan_amd.linear import _LinearF16x3
    x = _rand((M, K), mag, 1).to(DEV).requires_grad_(True)
    w = (_rand((N, K), "unit", 2) * 0.05).to(DEV).requires_grad_(True)
    b = (_rand((N,), "unit", 3) * 0.1).to(DEV).requires_grad_(True)
    gy = _rand((M, N), mag, 4).to(DEV)
    y = _LinearF16x3.apply(x, w, b, False)
    y.backward(gy)
    torch.cuda.synchronize()
    xd, wd, bd, gyd = (t.detach().double().cpu() for t in (x, w, b, gy))
    yd = xd @ wd.t() + bd
    # PyTorch's fp32 (rocBLAS) op on the same data, for scale
    x32, w32, b32 = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    y32 = torch.nn.functional.linear(x32, w32, b32)
    y32.backward(gy)
    for name, got, ref32, exact, scale in (
            ("forward", y.detach(), y32.detach(), yd, xd.abs() @ wd.abs().t() + bd.abs()),
            ("input grad", x.grad, x32.grad, gyd @ wd, gyd.abs() @ wd.abs()),
            ("weight grad", w.grad, w32.grad, gyd.t() @ xd, gyd.abs().t() @ xd.abs())):
        # within c u sum|terms| of the exact result, or no worse than 2x rocBLAS fp32
        err = (got.double().cpu() - exact).abs()
        err32 = float(((ref32.double().cpu() - exact).abs() / (U * scale + 1e-30)).max())
        ratio = float((err / (U * scale + 1e-30)).max())
        assert ratio <= max(32.0, 2.0 * err32), f"{name}: {ratio:.1f} u (rocBLAS {err32:.1f} u)"
    np.testing.assert_allclose(b.grad.cpu().numpy(), gyd.sum(0).numpy(),
                               rtol=1e-5, atol=1e-5 * float(gyd.abs().sum(0).max()))


def test_linear_routing_and_deterministic(sdfr):
    """linear() takes the kernels only for the MLP's training shapes; the weight
    gradient's split reduction is deterministic run to run."""
    from sdface_gan_amd import linear as lin
    x = torch.randn(196608 // 16, 256, device=DEV, requires_grad=True)
    w = torch.randn(256, 256, device=DEV, requires_grad=True)
    y = lin.linear(x, w)
    assert y.grad_fn is not None and "LinearF16x3" in type(y.grad_fn).__name__
    with torch.no_grad():
        assert lin.linear(x, w).grad_fn is None             # inference: F.linear
    s = torch.randn(8, 256, device=DEV)
    assert "LinearF16x3" not in type(lin.linear(s.requires_grad_(), w).grad_fn).__name__
    # in features up to 288 take both directions (padded: the FCGenerator's 280-wide views
    # layer); 292 would need a 304-wide input gradient, which the kernels do not take:
    # F.linear
    for K, routed in ((60, True), (259, True), (272, True), (280, True), (292, False)):
        xk = torch.randn(4096, K, device=DEV, requires_grad=True)
        wk = torch.randn(256, K, device=DEV, requires_grad=True)
        yk = lin.linear(xk, wk)
        assert ("LinearF16x3" in type(yk.grad_fn).__name__) == routed, K
        yk.square().sum().backward()
        assert xk.grad.shape == xk.shape and wk.grad.shape == wk.shape
    grads = []
    for _ in range(2):
        w.grad = None
        lin.linear(x, w).square().sum().backward()
        grads.append(w.grad.clone())
    assert torch.equal(grads[0], grads[1])


class _F64Linear:
    """torch.nn.functional with linear evaluated in float64 (a more exact reference for
    the renderer MLP's GEMMs; the rest of the model stays fp32)."""

    def __getattr__(self, name):
        return getattr(torch.nn.functional, name)

    @staticmethod
    def linear(x, w, b=None):
        y = torch.nn.functional.linear(x.double(), w.double(), None if b is None else b.double())
        return y.float()


@pytest.mark.parametrize("ngp", [True, False], ids=["ngp", "siren"])
def test_stage1_gradients_kernels_vs_torch_gemm(sdfr, ngp):
    """One stage-1 generator backward (adversarial + eikonal + minimal-surface +
    smoothness terms, perturb 0) with the renderer MLP's GEMMs on the HIP kernels, on
    rocBLAS fp32, and in float64 (the reference): every gradient of the kernels is
    within 2e-4 of the largest gradient of its tensor, or no further from the float64
    run than the rocBLAS fp32 run is (twice that distance) -- the latter for the
    cancelling scalar sigmoid_beta (a sum over every sample, tests/test_gpu_stage1.py)."""
    from sdface_gan_amd import linear as lin
    from sdface_gan_amd import training
    from sdface_gan_amd.training import RendererTrainer
    from tests.test_train_renderer import stage1_opt
    opt = stage1_opt(sdfr, ngp=ngp, res=32, samples=24, batch=2, chunk=2)
    opt.rendering.perturb = 0
    torch.manual_seed(0)
    noise = [torch.randn(2, 256, device=DEV)]
    cams = sdfr.generate_camera_params(32, DEV, batch=2)
    grads = {}
    orig, orig_f = training.smoothness, lin.F
    for mode in ("torch", "f64", "f16x3"):
        lin.set_train_gemm("f16x3" if mode == "f16x3" else "torch")
        if mode == "f64":
            lin.F = _F64Linear()
        tr = RendererTrainer(opt, DEV, seed=5)

        def smooth(*a, **k):
            torch.manual_seed(7)                       # the same voxel block every time
            return orig(*a, **k)
        training.smoothness = smooth
        try:
            tr.g_backward(iter([(noise, cams)]), 1)
        finally:
            training.smoothness = orig
            lin.F = orig_f
            lin.set_train_gemm("f16x3")
        grads[mode] = {n: p.grad.detach().clone() for n, p in tr.g_module.named_parameters()
                       if p.grad is not None}
    assert set(grads["torch"]) == set(grads["f16x3"]) == set(grads["f64"])
    for k, ref in grads["f64"].items():
        got, t32 = grads["f16x3"][k], grads["torch"][k]
        scale = float(ref.abs().max())
        err = float((got - ref).abs().max())
        err32 = float((t32 - ref).abs().max())
        assert err <= max(2e-4 * scale, 2.0 * err32) + 1e-12, \
            f"{k}: max |diff| {err:.3e} (rocBLAS fp32 {err32:.3e}, max |g| {scale:.3e})"


@pytest.mark.parametrize("F_,R,K", [(2, 1536, 256), (3, 700, 272)])
def test_film_linear_vs_float64(sdfr, F_, R, K):
    """FiLMSiren with the FiLM activation fused into the GEMM epilogue and its backward's
    elementwise part in one kernel: sin(gamma (x W^T + b) + beta) and the gradients of
    x, W, b, gamma, beta against float64 autograd of the reference's ops."""
    from sdface_gan_amd.linear import _FiLMLinearF16x3
    N = 256
    x = (_rand((F_, R, K), "unit", 5) * 0.5).to(DEV).requires_grad_(True)
    w = (_rand((N, K), "unit", 6) * 0.05).to(DEV).requires_grad_(True)
    b = (_rand((N,), "unit", 7) * 0.1).to(DEV).requires_grad_(True)
    gam = (30 + 15 * _rand((F_, 1, N), "unit", 8) * 0.2).to(DEV).requires_grad_(True)
    bet = (0.25 * _rand((F_, 1, N), "unit", 9)).to(DEV).requires_grad_(True)
    ds = _rand((F_, R, N), "unit", 10).to(DEV)
    s = _FiLMLinearF16x3.apply(x, w, b, gam, bet, False)
    s.backward(ds)
    torch.cuda.synchronize()
    xd, wd, bd, gd, btd = (t.detach().double().cpu().requires_grad_(True)
                           for t in (x, w, b, gam, bet))
    y = xd @ wd.t() + bd
    sd = torch.sin(gd * y + btd)
    sd.backward(ds.double().cpu())
    # the sin argument is ~30x the GEMM output: compare through its own scale
    yscale = (xd.detach().abs() @ wd.detach().abs().t() + bd.detach().abs())
    arg_err = 64 * U * (gd.detach().abs() * yscale + btd.detach().abs()) + 1.5e-6
    assert float(((s.detach().cpu().double() - sd.detach()).abs() - arg_err).max()) <= 0
    for name, got, ref in (("x", x.grad, xd.grad), ("W", w.grad, wd.grad), ("b", b.grad, bd.grad),
                           ("gamma", gam.grad, gd.grad), ("beta", bet.grad, btd.grad)):
        ref = ref.detach()
        err = float((got.cpu().double() - ref).abs().max())
        scale = float(ref.abs().max())
        assert err <= 2e-4 * scale, f"{name}: max |diff| {err:.3e} vs max |g| {scale:.3e}"


@pytest.mark.parametrize("J,K", [(1, 256), (3, 256), (4, 36)])
def test_linear_head_vs_float64(sdfr, J, K):
    """The narrow heads (sigma 256 -> 1, rgb 256 -> 3; csrc/linear_head.hip): forward,
    input / weight / bias gradients against float64, fp32 FMA accuracy; deterministic."""
    from sdface_gan_amd.linear import _LinearHead, linear
    M = 70001
    x = _rand((M, K), "unit", 11).to(DEV).requires_grad_(True)
    w = (_rand((J, K), "unit", 12) * 0.05).to(DEV).requires_grad_(True)
    b = (_rand((J,), "unit", 13) * 0.1).to(DEV).requires_grad_(True)
    gy = _rand((M, J), "unit", 14).to(DEV)
    y = linear(x, w, b)
    assert "LinearHead" in type(y.grad_fn).__name__
    y.backward(gy)
    torch.cuda.synchronize()
    xd, wd, bd, gyd = (t.detach().double().cpu() for t in (x, w, b, gy))
    for name, got, exact, scale in (
            ("forward", y.detach(), xd @ wd.t() + bd, xd.abs() @ wd.abs().t() + bd.abs()),
            ("input grad", x.grad, gyd @ wd, gyd.abs() @ wd.abs()),
            ("weight grad", w.grad, gyd.t() @ xd, gyd.abs().t() @ xd.abs()),
            ("bias grad", b.grad, gyd.sum(0), gyd.abs().sum(0))):
        _bound_check(name, got, exact, scale, c=64.0)
    g0 = w.grad.clone()
    w.grad = None
    _LinearHead.apply(x, w, b, False).backward(gy)
    assert torch.equal(g0, w.grad)
