"""GPU parity: the HIP grid / SH encoder kernels against the C oracle.

Index math and the trilinear accumulation follow the oracle's exact operation
order, so forward outputs and dy_dx must be BIT-EXACT.  The table backward
scatters with fp32 atomics (order-dependent), so it is compared with a
tolerance; the input backward is a fixed-order reduction and is bit-exact.
"""
import ctypes

import numpy as np
import pytest
import torch

from tests.golden import weights as W

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _grid_gpu(sdfr, x, emb, offsets, pls, H=16, dydx=False, gridtype=0, align=False, interp=0):
    lib = sdfr._lib
    xt = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    et = torch.from_numpy(np.ascontiguousarray(emb)).to(DEV)
    ot = torch.from_numpy(np.ascontiguousarray(offsets, dtype=np.int32)).to(DEV)
    B, D = x.shape
    L = len(offsets) - 1
    C = emb.shape[1]
    out = torch.empty(L, B, C, device=DEV)
    dd = torch.empty(B, L * D * C, device=DEV) if dydx else None
    lib.check(lib.lib().sdfr_grid_encode_forward(
        lib.ptr(xt), lib.ptr(et), lib.ptr(ot), lib.ptr(out), B, D, C, L,
        float(np.float32(np.log2(pls))), H, lib.ptr(dd), gridtype, int(align), interp,
        lib.stream_of(xt)), "grid fwd")
    torch.cuda.synchronize()
    return out.cpu().numpy(), (dd.cpu().numpy() if dydx else None)


@pytest.fixture(scope="module")
def table(oracle_mod):
    offsets, pls = oracle_mod.grid_offsets()
    return offsets, pls, W.det_table(int(offsets[-1]), 2, seed=7)


def test_grid_forward_bit_exact_golden_inputs(sdfr, oracle_mod, golden_dir, table):
    offsets, pls, emb = table
    g = np.load(golden_dir / "encoders.npz")
    x = g["grid_x"]
    got, _ = _grid_gpu(sdfr, x, emb, offsets, pls)
    ref, _ = oracle_mod.grid_encode_forward(x, emb, offsets, pls, 16)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(got.transpose(1, 0, 2).reshape(len(x), -1), g["grid_out"])


def test_grid_forward_bit_exact_large_and_dydx(sdfr, oracle_mod, table):
    offsets, pls, emb = table
    rng = np.random.default_rng(11)
    x = rng.uniform(-0.05, 1.05, size=(200_003, 3)).astype(np.float32)   # ragged, some OOB
    got, gd = _grid_gpu(sdfr, x, emb, offsets, pls, dydx=True)
    ref, rd = oracle_mod.grid_encode_forward(x, emb, offsets, pls, 16, calc_dy_dx=True)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(gd, rd)


@pytest.mark.parametrize("D,C,gridtype,align,interp,log2h", [
    (2, 4, 0, False, 0, 14),
    (3, 1, 1, False, 0, 12),
    (3, 8, 0, True, 1, 15),
    (4, 2, 0, False, 0, 16),
])
def test_grid_forward_variants(sdfr, oracle_mod, D, C, gridtype, align, interp, log2h):
    from oracle.oracle import grid_offsets
    offsets, pls = grid_offsets(num_levels=8, level_dim=C, base_resolution=8,
                                log2_hashmap_size=log2h, desired_resolution=256, input_dim=D,
                                align_corners=align)
    emb = W.det_uniform((int(offsets[-1]), C), -1, 1, 17)
    rng = np.random.default_rng(D * 10 + C)
    x = rng.uniform(0, 1, size=(5000, D)).astype(np.float32)
    got, gd = _grid_gpu(sdfr, x, emb, offsets, pls, H=8, dydx=True, gridtype=gridtype,
                        align=align, interp=interp)
    ref, rd = oracle_mod.grid_encode_forward(x, emb, offsets, pls, 8, calc_dy_dx=True,
                                             gridtype=gridtype, align_corners=align,
                                             interp=interp)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(gd, rd)


def test_grid_backward(sdfr, oracle_mod, table):
    offsets, pls, emb = table
    rng = np.random.default_rng(5)
    x = rng.uniform(0.2, 0.8, size=(4096, 3)).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    et = torch.nn.Parameter(torch.from_numpy(emb).to(DEV))
    ot = torch.from_numpy(offsets).to(DEV)
    out = sdfr.grid_encode(xt, et, ot, pls, 16, True, 0, False, 0)
    grad = torch.from_numpy(rng.normal(size=out.shape).astype(np.float32)).to(DEV)
    out.backward(grad)
    _, dydx = oracle_mod.grid_encode_forward(x, emb, offsets, pls, 16, calc_dy_dx=True)
    g_lbc = grad.view(4096, 16, 2).permute(1, 0, 2).contiguous().cpu().numpy()
    ge, gi = oracle_mod.grid_encode_backward(g_lbc, x, emb, offsets, pls, 16, dy_dx=dydx)
    # atomics: order-dependent fp32 sums; |sum| of a few dozen O(1) terms
    np.testing.assert_allclose(et.grad.cpu().numpy(), ge, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(xt.grad.cpu().numpy(), gi)


def test_grid_module_and_empty_batch(sdfr, table):
    offsets, pls, emb = table
    enc = sdfr.GridEncoder(desired_resolution=4096).to(DEV)
    with torch.no_grad():
        enc.embeddings.copy_(torch.from_numpy(emb))
    x = torch.rand(2, 5, 3, device=DEV) * 2 - 1
    assert enc(x, bound=2).shape == (2, 5, 32)
    assert enc(torch.zeros(0, 3, device=DEV), bound=2).shape == (0, 32)


def test_sh_forward_backward_bit_exact(sdfr, oracle_mod, golden_dir):
    g = np.load(golden_dir / "encoders.npz")
    rng = np.random.default_rng(9)
    x = np.concatenate([g["sh_dirs"], rng.normal(size=(3001, 3)).astype(np.float32)])
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    out = sdfr.sh_encode(xt, 4, True)
    ref, dref = oracle_mod.sh_encode_forward(x, 4, calc_dy_dx=True)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ref)
    np.testing.assert_array_equal(out.detach().cpu().numpy()[:1024], g["sh_out"])
    grad = rng.normal(size=ref.shape).astype(np.float32)
    out.backward(torch.from_numpy(grad).to(DEV))
    np.testing.assert_array_equal(xt.grad.cpu().numpy(),
                                  oracle_mod.sh_encode_backward(grad, x, 4, dref))
    for deg in (1, 2, 3):
        o = sdfr.sh_encode(torch.from_numpy(x).to(DEV), deg, False)
        np.testing.assert_array_equal(o.cpu().numpy(), oracle_mod.sh_encode_forward(x, deg)[0])


@pytest.mark.parametrize("deg", [5, 6, 7, 8])
def test_sh_degrees_5_to_8_bit_exact(sdfr, oracle_mod, golden_dir, deg):
    """The reference's _shencoder accepts degrees 1..8 (sphere_harmonics.py:62-86):
    the HIP kernel's bands 4..7 equal the oracle bit for bit (forward, dy_dx, input
    backward), and the reference's own degree-8 formulas to fp32 rounding."""
    g = np.load(golden_dir / "sh_deg8.npz")
    x = g["dirs"]
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    out = sdfr.sh_encode(xt, deg, True)
    ref, dref = oracle_mod.sh_encode_forward(x, deg, calc_dy_dx=True)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ref)
    c2 = deg * deg
    scale = np.abs(g["sh_out"][:, :c2]).max(0) + 1e-30
    assert (np.abs(out.detach().cpu().numpy() - g["sh_out"][:, :c2]) / scale).max() < 1e-5
    grad = np.random.default_rng(deg).normal(size=ref.shape).astype(np.float32)
    out.backward(torch.from_numpy(grad).to(DEV))
    np.testing.assert_array_equal(xt.grad.cpu().numpy(),
                                  oracle_mod.sh_encode_backward(grad, x, deg, dref))


def test_device_sin_accuracy(sdfr):
    """The field kernel's sin (hardware v_sin_f32 after an fma 2pi reduction) and
    the polynomial alternative, against float64 over the FiLM argument range."""
    lib = sdfr._lib
    xs = ((torch.rand(1 << 20, dtype=torch.float64, generator=torch.Generator().manual_seed(0))
           - 0.5) * 400).float()
    xd = xs.to(DEV)
    cw, hw = torch.empty_like(xd), torch.empty_like(xd)
    lib.check(lib.lib().sdfr_debug_sin_probe(lib.ptr(xd), lib.ptr(cw), lib.ptr(hw), xd.numel(),
                                             lib.stream_of(xd)), "sin probe")
    ref = torch.sin(xs.double())
    assert (cw.cpu().double() - ref).abs().max() < 2e-7
    assert (hw.cpu().double() - ref).abs().max() < 1e-6


def test_device_sin_rev_accuracy(sdfr):
    """The split-fp16 field kernel's FiLM sin: argument in revolutions (1/(2 pi) folded
    into gamma / beta), v_sin_f32 alone (its own range reduction).  Against float64
    sin(2 pi u) over the FiLM range (|gamma x + beta| <= 200 rad, i.e. |u| <= 32) and
    far beyond it (|u| up to 4096)."""
    lib = sdfr._lib
    gen = torch.Generator().manual_seed(1)
    for span, tol in ((64.0, 1e-6), (8192.0, 1e-6)):
        us = ((torch.rand(1 << 20, dtype=torch.float64, generator=gen) - 0.5) * span).float()
        ud = us.to(DEV)
        out = torch.empty_like(ud)
        lib.check(lib.lib().sdfr_debug_sin_rev_probe(lib.ptr(ud), lib.ptr(out), ud.numel(),
                                                     lib.stream_of(ud)), "sin_rev probe")
        ref = torch.sin(2 * np.pi * us.double())
        assert (out.cpu().double() - ref).abs().max() < tol, span


def test_grid_backward_large_privatised_levels(sdfr, oracle_mod, table):
    """200 k samples in the renderer's coordinate range through the module path
    (GridEncoder's workspace: every level binned, summed in LDS); order-dependent
    fp32 sums of the oracle's per-sample products."""
    offsets, pls, emb = table
    rng = np.random.default_rng(9)
    n = 200_000
    x = rng.uniform(0.23, 0.78, size=(n, 3)).astype(np.float32)
    x[:7] = [[-0.1, 0.5, 0.5], [1.2, 0.5, 0.5], [0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.5],
             [0.999, 0.001, 0.5], [0.25, 0.75, 1.0]]                 # OOB and edges
    xt = torch.from_numpy(x).to(DEV)
    et = torch.nn.Parameter(torch.from_numpy(emb).to(DEV))
    ot = torch.from_numpy(offsets).to(DEV)
    out = sdfr.grid_encode(xt, et, ot, pls, 16, True, 0, False, 0)
    grad = torch.from_numpy(rng.normal(size=out.shape).astype(np.float32)).to(DEV)
    out.backward(grad)
    g_lbc = grad.view(n, 16, 2).permute(1, 0, 2).contiguous().cpu().numpy()
    ge, _ = oracle_mod.grid_encode_backward(g_lbc, x, emb, offsets, pls, 16)
    got = et.grad.cpu().numpy()
    np.testing.assert_allclose(got, ge, rtol=1e-4, atol=2e-5 * float(np.abs(ge).max()))
    assert np.count_nonzero(got) == np.count_nonzero(ge)


def _grid_bwd_ws(sdfr, g_lbc, x, emb, offsets, pls, binned):
    """sdfr_grid_encode_backward_ws with (binned) or without (direct atomics) a workspace."""
    lib = sdfr._lib
    L_ = lib.lib()
    gt = torch.from_numpy(np.ascontiguousarray(g_lbc)).to(DEV)
    xt = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    ot = torch.from_numpy(np.ascontiguousarray(offsets, dtype=np.int32)).to(DEV)
    L, B, C = g_lbc.shape
    S = float(np.float32(np.log2(pls)))
    ge = torch.zeros(emb.shape, device=DEV)
    wsb = L_.sdfr_grid_encode_backward_ws_bytes(B, 3, C, L, S, 16, 0) if binned else 0
    ws = torch.empty(wsb, dtype=torch.uint8, device=DEV) if wsb else None
    assert (wsb > 0) == binned
    lib.check(L_.sdfr_grid_encode_backward_ws(
        lib.ptr(gt), lib.ptr(xt), None, lib.ptr(ot), lib.ptr(ge), B, 3, C, L, S, 16, None, None,
        0, 0, 0, lib.ptr(ws), wsb, lib.stream_of(gt)), "grid bwd ws")
    torch.cuda.synchronize()
    return ge.cpu().numpy()


@pytest.mark.parametrize("C,log2_hash", [(2, 19), (2, 20), (1, 19), (4, 18), (8, 17)])
def test_grid_backward_binned_vs_direct_and_oracle(sdfr, oracle_mod, C, log2_hash):
    """The binned table gradient (count, scan, LDS counting sort, work items, LDS sums)
    against the workspace-less path (LDS windows for the coarse levels, direct atomics
    for the rest) and the oracle, for every C and for tables larger than 32 LDS windows
    per level (log2_hash 20 at C = 2: two sweeps per bin).  Order-dependent fp32 sums
    on all three sides."""
    offsets, pls = oracle_mod.grid_offsets(level_dim=C, log2_hashmap_size=log2_hash)
    emb = W.det_table(int(offsets[-1]), C, seed=11)
    rng = np.random.default_rng(C + log2_hash)
    n = 65_536
    x = rng.uniform(0.05, 0.95, size=(n, 3)).astype(np.float32)
    x[:3] = [[-0.1, 0.5, 0.5], [1.0, 1.0, 1.0], [0.0, 0.0, 0.0]]
    g_lbc = rng.normal(size=(16, n, C)).astype(np.float32)
    ref, _ = oracle_mod.grid_encode_backward(g_lbc, x, emb, offsets, pls, 16)
    tol = dict(rtol=1e-4, atol=2e-5 * float(np.abs(ref).max()))
    binned = _grid_bwd_ws(sdfr, g_lbc, x, emb, offsets, pls, True)
    direct = _grid_bwd_ws(sdfr, g_lbc, x, emb, offsets, pls, False)
    np.testing.assert_allclose(binned, ref, **tol)
    np.testing.assert_allclose(direct, ref, **tol)
    assert np.count_nonzero(binned) == np.count_nonzero(ref)


def test_grid_backward_accumulates_into_existing(sdfr, oracle_mod, table):
    """grad_embeddings is added to, not overwritten (the reference atomically adds into
    the caller's zeros): two binned calls give twice one call."""
    offsets, pls, emb = table
    rng = np.random.default_rng(3)
    n = 8192
    x = rng.uniform(0.1, 0.9, size=(n, 3)).astype(np.float32)
    g_lbc = rng.normal(size=(16, n, 2)).astype(np.float32)
    lib = sdfr._lib
    L_ = lib.lib()
    S = float(np.float32(np.log2(pls)))
    gt, xt = torch.from_numpy(g_lbc).to(DEV), torch.from_numpy(x).to(DEV)
    ot = torch.from_numpy(np.asarray(offsets, np.int32)).to(DEV)
    ge = torch.zeros(emb.shape, device=DEV)
    for _ in range(2):
        lib.check(L_.sdfr_grid_encode_backward(lib.ptr(gt), lib.ptr(xt), None, lib.ptr(ot),
                                               lib.ptr(ge), n, 3, 2, 16, S, 16, None, None, 0, 0,
                                               0, lib.stream_of(gt)), "grid bwd")
    ref, _ = oracle_mod.grid_encode_backward(g_lbc, x, emb, offsets, pls, 16)
    np.testing.assert_allclose(ge.cpu().numpy(), 2 * ref, rtol=1e-4,
                               atol=4e-5 * float(np.abs(ref).max()))


def test_grid_backward_captured_in_hip_graph(sdfr):
    """The hash-grid forward + backward (binned table gradient in a torch-allocated
    workspace) captured in a HIP graph replays to the eager gradients: no hidden
    allocation or host sync in the stream-ordered calls (grid.py:65-89)."""
    import torch
    from sdface_gan_amd.encoders import GridEncoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    enc = GridEncoder(input_dim=3, num_levels=16, level_dim=2, base_resolution=16,
                      log2_hashmap_size=19, desired_resolution=4096).to(dev)
    with torch.no_grad():
        enc.embeddings.uniform_(-1, 1)
    x = (torch.rand(8192, 3, device=dev) * 2 - 1) * 1.1
    gout = torch.randn(8192, 32, device=dev)

    def run():
        enc.embeddings.grad = None
        y = enc(x, bound=2)
        y.backward(gout)
        return enc.embeddings.grad
    ref = run().clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            run()                                   # warm the allocator on the side stream
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    enc.embeddings.grad = None
    with torch.cuda.graph(graph):
        y = enc(x, bound=2)
        y.backward(gout)
    graph.replay()
    torch.cuda.synchronize()
    got = enc.embeddings.grad
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))
