"""Training-path linear layers of the renderer MLP on split-fp16 MFMA.

When the renderer needs gradients (stage-1 training, training_utils.py:396-451)
its networks run op by op as the reference does (FiLMSiren / LinearLayer,
sdf_model.py:23-69, NGPSIRENGenerator :1566-1592): F.linear over ~196 K samples
per chunk, forward and backward.  ``linear`` routes those products to the HIP
kernels of ``csrc/linear_f16x3.hip`` (three fp16 MFMA terms per fp32 product,
fp32 accumulation, power-of-two row / column scaling: fp32-level accuracy):

  FiLM forward     s = sin(g (x W^T + b) + be) sdfr_film_linear_f16x3 (GEMM + epilogue)
  FiLM backward    dy, dg, dbe, db             sdfr_film_backward (one elementwise pass)
  forward          out = x W^T + b             sdfr_linear_f16x3 (B = W)
  input gradient   gx  = gy W                  sdfr_linear_f16x3 (B = W^T)
  weight gradient  gW  = gy^T x                sdfr_linear_wgrad_f16x3
  bias gradient    gb  = gy.sum(0)             (torch reduction)
  narrow heads     J <= 4 outputs (sigma 1, rgb 3): sdfr_linear_head_forward / _backward
                   (HBM-streaming fp32 FMA kernels in place of rocBLAS's N = 1..3 GEMMs)

Shapes the kernels take: out features 256 with in features <= 64, 256 or 257..288
(the networks' input / first layers, dense and views layers, the FCGenerator's 60-wide
x_in and 280-wide views; in features padded with zero columns to a multiple of 4 and the
input gradient's width to 32 / 64 / 256 / 272 / 288), and J <= 4 outputs with K <= 256
(the 3- and 1-wide heads).  Everything else (the per-face
gamma / beta layers on the styles, CPU tensors, inference) stays on F.linear.
``set_train_gemm("torch")`` turns the routing off.

Both networks route here (their layers carry ``train_kernels = True``).  The SIREN
network's eikonal term is an ``autograd.grad(..., create_graph=True)`` through the MLP
(sdf_model.py:224-229), so its loss reaches the weights through a double backward: its
layers also carry ``double_backward = True``, and their backward, when it runs with grad
enabled (create_graph), computes the same gradients as differentiable ops -- ``linear()``
of these kernels again, ``_WGradF16x3``, the FiLM elementwise part in torch ops around
``_LinearGiven`` (the saved pre-activation put on the graph without recomputing it).
Every other backward (and the ngp network's, whose eikonal term leaves autograd in the
grid encoder, grid.py:65-89) runs straight on the kernels.  A backward also skips the
gradients the running backward pass does not use (``_wanted``: the eikonal pass wants
d/d pts only), per graph task.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch.autograd.graph import get_gradient_edge

from . import _lib

_MODE = {"gemm": "f16x3"}


def set_train_gemm(mode: str) -> None:
    """'f16x3' (default): renderer-MLP training GEMMs on the HIP kernels; 'torch':
    F.linear (rocBLAS fp32)."""
    if mode not in ("f16x3", "torch"):
        raise ValueError(f"train gemm must be 'f16x3' or 'torch', got {mode!r}")
    _MODE["gemm"] = mode


def train_gemm() -> str:
    return _MODE["gemm"]


def _pack(w: torch.Tensor, transposed: bool) -> torch.Tensor:
    """Split-fp16 fragments + row scales of B = w (or w^T) for sdfr_linear_f16x3."""
    L = _lib.lib()
    N, K = (w.shape[1], w.shape[0]) if transposed else (w.shape[0], w.shape[1])
    buf = torch.empty(L.sdfr_linear_pack_bytes(N, K), dtype=torch.uint8, device=w.device)
    _lib.check(L.sdfr_linear_pack(_lib.ptr(w), N, K, int(transposed), _lib.ptr(buf),
                                  _lib.stream_of(w)), "sdfr_linear_pack")
    return buf


def _a16(t):
    """t, or a 16-B aligned copy (the kernels read bias / gamma / beta as 16-B vectors)."""
    if t is None:
        return None
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _gemm(x2: torch.Tensor, packed: torch.Tensor, bias, N: int) -> torch.Tensor:
    M, K = x2.shape
    out = torch.empty(M, N, device=x2.device, dtype=torch.float32)
    _lib.check(_lib.lib().sdfr_linear_f16x3(_lib.ptr(out), _lib.ptr(x2), _lib.ptr(packed),
                                            _lib.ptr(bias), M, N, K, _lib.stream_of(x2)),
               "sdfr_linear_f16x3")
    return out


def _wgrad(gy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    L = _lib.lib()
    M, N = gy2.shape
    K = x2.shape[1]
    nws = L.sdfr_linear_wgrad_ws_bytes(M, N, K)
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=gy2.device)
    gw = torch.empty(N, K, device=gy2.device, dtype=torch.float32)
    _lib.check(L.sdfr_linear_wgrad_f16x3(_lib.ptr(gw), _lib.ptr(gy2), _lib.ptr(x2), M, N, K,
                                         _lib.ptr(ws), nws, _lib.stream_of(gy2)),
               "sdfr_linear_wgrad_f16x3")
    return gw


def _film_fwd(x2, packed, bias, g2, b2, N):
    """(sin(gamma[f] y + beta[f]), y = x2 . B^T + bias) over F = g2.shape[0] faces of
    equal row count (sdfr_film_linear_f16x3)."""
    M = x2.shape[0]
    F_ = g2.shape[0]
    out = torch.empty(M, N, device=x2.device, dtype=torch.float32)
    y = torch.empty(M, N, device=x2.device, dtype=torch.float32)
    _lib.check(_lib.lib().sdfr_film_linear_f16x3(
        _lib.ptr(out), _lib.ptr(y), _lib.ptr(x2), _lib.ptr(packed), _lib.ptr(bias), _lib.ptr(g2),
        _lib.ptr(b2), M, N, x2.shape[1], M // F_, _lib.stream_of(x2)), "sdfr_film_linear_f16x3")
    return out, y


def _film_bwd(ds2, y, g2, b2):
    """The FiLM backward's elementwise part (sdfr_film_backward): dy [M,N] and the
    per-face dgamma, dbeta, bias-gradient partials [F,N]."""
    M, N = ds2.shape
    F_ = g2.shape[0]
    L = _lib.lib()
    dy = torch.empty(M, N, device=ds2.device, dtype=torch.float32)
    dg = torch.empty(F_, N, device=ds2.device, dtype=torch.float32)
    db_ = torch.empty(F_, N, device=ds2.device, dtype=torch.float32)
    dbf = torch.empty(F_, N, device=ds2.device, dtype=torch.float32)
    nws = L.sdfr_film_backward_ws_bytes(M, N, M // F_)
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=ds2.device)
    _lib.check(L.sdfr_film_backward(
        _lib.ptr(dy), _lib.ptr(dg), _lib.ptr(db_), _lib.ptr(dbf), _lib.ptr(ds2), _lib.ptr(y),
        _lib.ptr(g2), _lib.ptr(b2), M, N, M // F_, _lib.ptr(ws), nws, _lib.stream_of(ds2)),
        "sdfr_film_backward")
    return dy, dg, db_, dbf


def _film_bwd2(ds2, y, g2, b2, gdy, gdg, gdb):
    """The derivative of _film_bwd's (dy, dgamma, dbeta) w.r.t. (ds, y, gamma, beta)
    given their upstream gradients (each may be None) (sdfr_film_backward_grad)."""
    M, N = ds2.shape
    F_ = g2.shape[0]
    L = _lib.lib()
    d_ds = torch.empty(M, N, device=ds2.device, dtype=torch.float32)
    d_y = torch.empty(M, N, device=ds2.device, dtype=torch.float32)
    d_g = torch.empty(F_, N, device=ds2.device, dtype=torch.float32)
    d_b = torch.empty(F_, N, device=ds2.device, dtype=torch.float32)
    nws = L.sdfr_film_backward_grad_ws_bytes(M, N, M // F_)
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=ds2.device)
    opt = [None if t is None else _a16(t.contiguous()) for t in (gdy, gdg, gdb)]
    _lib.check(L.sdfr_film_backward_grad(
        _lib.ptr(d_ds), _lib.ptr(d_y), _lib.ptr(d_g), _lib.ptr(d_b), _lib.ptr(ds2), _lib.ptr(y),
        _lib.ptr(g2), _lib.ptr(b2), *[None if t is None else _lib.ptr(t) for t in opt],
        M, N, M // F_, _lib.ptr(ws), nws, _lib.stream_of(ds2)), "sdfr_film_backward_grad")
    return d_ds, d_y, d_g, d_b


class _FiLMGrad(torch.autograd.Function):
    """The FiLM backward's elementwise part as ONE differentiable op, for graphs built
    with create_graph (the SIREN eikonal term): forward = sdfr_film_backward
    (du = ds cos(gamma y + beta); dy = du gamma, dgamma = sum du y, dbeta = sum du),
    backward = sdfr_film_backward_grad.  Autograd of the same math as torch ops ran
    ~18 elementwise / reduction passes over the [rows, 256] activation per layer (the
    SIREN stage-1 step's largest cost).  Not differentiable a third time."""

    @staticmethod
    def forward(ctx, ds, y, gamma, beta):
        N = y.shape[-1]
        F_ = gamma.shape[0]
        ds2 = _a16(ds.reshape(-1, N).contiguous())
        y2 = _a16(y.reshape(-1, N).contiguous())
        g2, b2 = _a16(gamma.reshape(F_, N).contiguous()), _a16(beta.reshape(F_, N).contiguous())
        dy, dg, db_, _ = _film_bwd(ds2, y2, g2, b2)
        ctx.save_for_backward(ds2, y2, g2, b2)
        ctx.shapes = (ds.shape, y.shape, gamma.shape, beta.shape)
        return dy.view(y.shape), dg.view(gamma.shape), db_.view(beta.shape)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gdy, gdg, gdb):
        ds2, y2, g2, b2 = ctx.saved_tensors
        sh_ds, sh_y, sh_g, sh_b = ctx.shapes
        N, F_ = y2.shape[1], g2.shape[0]
        d_ds, d_y, d_g, d_b = _film_bwd2(
            ds2, y2, g2, b2, None if gdy is None else gdy.reshape(-1, N),
            None if gdg is None else gdg.reshape(F_, N), None if gdb is None else gdb.reshape(F_, N))
        return d_ds.view(sh_ds), d_y.view(sh_y), d_g.view(sh_g), d_b.view(sh_b)


def _kp(K: int) -> int:
    """In features padded to the GEMM's multiple of 4 (zero columns: the product is
    unchanged)."""
    return -(-K // 4) * 4


def _np_t(K: int) -> int:
    """Output width of the input-gradient GEMM (B = W^T [K, N]): the kernels take 32,
    64, 256, 272 or 288 (a multiple of 16), so W^T gets zero rows up to that."""
    for n in (32, 64, 256, 272, 288):
        if K <= n:
            return n
    raise ValueError(f"no input-gradient GEMM for {K} in features")


def _xk(x: torch.Tensor, K: int) -> torch.Tensor:
    """x [..., K] as a 16-B aligned [M, _kp(K)] matrix (zero-padded copy when K % 4)."""
    x2 = x.reshape(-1, K)
    Kp = _kp(K)
    return F.pad(x2, (0, Kp - K)) if Kp != K else _a16(x2)


def _wk(w: torch.Tensor) -> torch.Tensor:
    N, K = w.shape
    Kp = _kp(K)
    return F.pad(w, (0, Kp - K)) if Kp != K else w.contiguous()


def _gx(gy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """gy2 [M, N] . w [N, K] -> [M, K] on the split-fp16 GEMM (B = W^T, zero rows up to
    _np_t(K))."""
    K = w.shape[1]
    Np = _np_t(K)
    wp = F.pad(w, (0, Np - K)) if Np != K else w.contiguous()
    out = _gemm(gy2, _pack(wp, True), None, Np)
    return out[:, :K] if Np != K else out


def _gw(gy2: torch.Tensor, x: torch.Tensor, K: int) -> torch.Tensor:
    """Weight gradient gy2^T . x [N, K] (x [..., K] zero-padded to the kernel's K)."""
    gw = _wgrad(gy2, _xk(x, K))
    return gw[:, :K].contiguous() if gw.shape[1] != K else gw


def _edge(t):
    """The autograd node a gradient for t goes to (its AccumulateGrad for a leaf), or
    None: kept by the forwards so a backward can tell which of its outputs the running
    backward pass actually uses (_wanted)."""
    if t is None or not t.requires_grad:
        return None
    return get_gradient_edge(t)


def _wanted(need: bool, edge) -> bool:
    """Whether the running backward pass uses this gradient: it may be an
    autograd.grad over other inputs -- the eikonal term's d sdf / d pts -- whose graph
    reaches a weight's node without running it (then the GEMM is skipped).  Scoped to
    the one graph task, unlike a process-global switch."""
    if not need or edge is None:
        return need
    try:
        return bool(torch._C._will_engine_execute_node(edge.node))
    except RuntimeError:                   # not inside a backward pass
        return True


def _once(grads, inputs):
    """The gradients a kernel backward computed outside autograd, returned from a
    backward that runs with grad enabled (create_graph) for a layer not marked
    ``twice``: marked like torch.autograd.function.once_differentiable's outputs, so a
    double backward through them raises instead of silently dropping its second-order
    term.  The ngp network's eikonal pass never differentiates them again:
    the grid encoder's backward ends that graph."""
    if not torch.is_grad_enabled() or not any(
            isinstance(t, torch.Tensor) and t.requires_grad for t in inputs):
        return grads
    from torch._C import _functions
    live = [g for g in grads if g is not None]
    if not live:
        return grads
    err = _functions.DelayedError(
        b"trying to differentiate twice a split-fp16 linear layer built without "
        b"double_backward (linear(..., twice=True))", len(live))

    def fake(v):
        v = v.detach()
        v.requires_grad = True
        return v
    out = err(*[fake(g) for g in live])
    out = list(out) if isinstance(out, tuple) else [out]
    it = iter(out)
    return tuple(next(it) if g is not None else None for g in grads)


def _linear_backward(gy, x, w, has_bias, needs, edges, twice=True):
    """Gradients of y = x W^T + b.  Inside a backward that builds a graph
    (autograd.grad(..., create_graph=True): the SIREN eikonal term) as differentiable
    ops -- linear() (these kernels again), _WGradF16x3, a sum -- so the eikonal loss
    reaches the weights through a double backward; otherwise straight on the kernels."""
    N, K = w.shape
    lead = x.shape[:-1]
    nx = needs[0]
    nw = _wanted(needs[1], edges[0])
    nb = has_bias and _wanted(needs[2], edges[1])
    gx = gw = gb = None
    if twice and torch.is_grad_enabled():
        gy2 = gy.reshape(-1, N)
        if nx:
            gx = linear(gy, w.t(), twice=True)
        if nw:
            gw = _WGradF16x3.apply(gy2, x.reshape(-1, K))
        if nb:
            gb = gy2.sum(0)
        return gx, gw, gb
    gy2 = _a16(gy.reshape(-1, N).contiguous())
    if nx:
        gx = _gx(gy2, w).reshape(*lead, K)
    if nw:
        gw = _gw(gy2, x, K)
    if nb:
        gb = gy2.sum(0)
    return _once((gx, gw, gb), (gy, x, w))


class _LinearF16x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, twice):
        N, K = weight.shape
        lead = x.shape[:-1]
        out = _gemm(_xk(x, K), _pack(_wk(weight), False), _a16(bias), N)
        ctx.save_for_backward(x, weight)        # the inputs themselves: double backward
        ctx.has_bias = bias is not None
        ctx.edges = (_edge(weight), _edge(bias))
        ctx.twice = twice
        return out.view(*lead, N)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        return (*_linear_backward(gy, x, w, ctx.has_bias, ctx.needs_input_grad, ctx.edges,
                                  ctx.twice), None)


class _LinearGiven(torch.autograd.Function):
    """y = x W^T + b whose value the caller already has (the fused FiLM forward saved
    it): returns y, differentiates as the linear layer.  The FiLM double backward uses
    it to put y on the graph without recomputing the GEMM."""

    @staticmethod
    def forward(ctx, x, weight, bias, y):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.edges = (_edge(weight), _edge(bias))
        return y.view_as(y)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        return (*_linear_backward(gy, x, w, ctx.has_bias, ctx.needs_input_grad, ctx.edges), None)


class _WGradF16x3(torch.autograd.Function):
    """gw = gy^T x [N, K] (the weight gradient) as a differentiable op: its own
    backward is two linear() products, so a graph built through a linear backward
    (create_graph) can be differentiated again."""

    @staticmethod
    def forward(ctx, gy2, x2):
        K = x2.shape[1]
        ctx.save_for_backward(gy2, x2)
        ctx.edges = (_edge(gy2), _edge(x2))
        return _gw(_a16(gy2.contiguous()), x2, K)

    @staticmethod
    def backward(ctx, G):
        gy2, x2 = ctx.saved_tensors
        dgy = dx = None
        if _wanted(ctx.needs_input_grad[0], ctx.edges[0]):
            dgy = linear(x2, G, twice=True)     # d/dgy [m, n] = sum_k G[n, k] x[m, k]
        if _wanted(ctx.needs_input_grad[1], ctx.edges[1]):
            dx = linear(gy2, G.t(), twice=True)  # d/dx [m, k] = sum_n G[n, k] gy[m, n]
        return dgy, dx


class _FiLMLinearF16x3(torch.autograd.Function):
    """sin(gamma[f] * (x W^T + b) + beta[f]) over F faces of equal row count: the GEMM
    with the FiLM activation in its epilogue (y = x W^T + b saved), and a backward whose
    elementwise part is one HIP kernel (dy, dgamma, dbeta, db) before the two GEMMs."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, twice):
        N, K = weight.shape
        F_ = gamma.shape[0]
        lead = x.shape[:-1]
        g2, b2 = _a16(gamma.reshape(F_, N)), _a16(beta.reshape(F_, N))
        out, y = _film_fwd(_xk(x, K), _pack(_wk(weight), False), _a16(bias), g2, b2, N)
        ctx.save_for_backward(x, weight, bias, gamma, beta, y)
        ctx.meta = (lead, bias is not None)
        ctx.edges = (_edge(weight), _edge(bias), _edge(gamma), _edge(beta))
        ctx.twice = twice
        return out.view(*lead, N)

    @staticmethod
    def backward(ctx, ds):
        x, w, bias, gamma, beta, y = ctx.saved_tensors
        lead, has_bias = ctx.meta
        N, K = w.shape
        F_ = gamma.shape[0]
        nx = ctx.needs_input_grad[0]
        nw = _wanted(ctx.needs_input_grad[1], ctx.edges[0])
        nb = has_bias and _wanted(ctx.needs_input_grad[2], ctx.edges[1])
        ng = _wanted(ctx.needs_input_grad[3], ctx.edges[2])
        nbe = _wanted(ctx.needs_input_grad[4], ctx.edges[3])
        if ctx.twice and torch.is_grad_enabled():
            # create_graph (the SIREN eikonal term): the same gradients as differentiable
            # ops, y put on the graph as the linear layer's output (_LinearGiven)
            yl = _LinearGiven.apply(x, w, bias, y.view(*lead, N))
            dyl, gg, gbt = _FiLMGrad.apply(ds, yl, gamma, beta)
            gx, gw, gb = _linear_backward(dyl, x, w, has_bias, (nx, nw, nb),
                                          (None, None))
            return gx, gw, gb, (gg if ng else None), (gbt if nbe else None), None
        ds2 = _a16(ds.reshape(-1, N).contiguous())
        g2, b2 = _a16(gamma.reshape(F_, N)), _a16(beta.reshape(F_, N))
        dy, dg, db_, dbf = _film_bwd(ds2, y, g2, b2)
        gx = gw = gb = None
        if nx:
            gx = _gx(dy, w).reshape(*lead, K)
        if nw:
            gw = _gw(dy, x, K)
        if nb:
            gb = dbf.sum(0)
        gg = dg.view(gamma.shape) if ng else None
        gbt = db_.view(beta.shape) if nbe else None
        return (*_once((gx, gw, gb, gg, gbt), (ds, x, w, gamma, beta)), None)


def _head_fwd(x2, w, bias):
    """x2 [M,K] . w [J,K]^T (+ bias) on the narrow-head kernel."""
    M, K = x2.shape
    J = w.shape[0]
    out = torch.empty(M, J, device=x2.device, dtype=torch.float32)
    _lib.check(_lib.lib().sdfr_linear_head_forward(
        _lib.ptr(out), _lib.ptr(x2), _lib.ptr(w), _lib.ptr(bias.contiguous() if bias is not None
                                                           else None),
        M, J, K, _lib.stream_of(x2)), "sdfr_linear_head_forward")
    return out


def _head_bwd(gy2, x2, w, need_x, need_w, need_b):
    """(gx [M,K], gw [J,K], gb [J]) of the narrow head, each None unless needed."""
    M, K = x2.shape
    J = w.shape[0]
    L = _lib.lib()
    gx = torch.empty(M, K, device=gy2.device, dtype=torch.float32) if need_x else None
    gw = torch.empty(J, K, device=gy2.device, dtype=torch.float32) if need_w else None
    gb = torch.empty(J, device=gy2.device, dtype=torch.float32) if need_b else None
    nws = L.sdfr_linear_head_ws_bytes(M, J, K) if (need_w or need_b) else 0
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=gy2.device)
    _lib.check(L.sdfr_linear_head_backward(
        _lib.ptr(gx), _lib.ptr(gw), _lib.ptr(gb), _lib.ptr(gy2), _lib.ptr(x2), _lib.ptr(w),
        M, J, K, _lib.ptr(ws), nws, _lib.stream_of(gy2)), "sdfr_linear_head_backward")
    return gx, gw, gb


class _LinearHead(torch.autograd.Function):
    """x W^T + b for the narrow heads (J <= 4 outputs): HBM-streaming HIP kernels."""

    @staticmethod
    def forward(ctx, x, weight, bias, twice):
        J, K = weight.shape
        lead = x.shape[:-1]
        out = _head_fwd(_a16(x.reshape(-1, K)), _a16(weight), bias)
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.edges = (_edge(weight), _edge(bias))
        ctx.twice = twice
        return out.view(*lead, J)

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        J, K = weight.shape
        lead = x.shape[:-1]
        need_x = ctx.needs_input_grad[0]
        need_w = _wanted(ctx.needs_input_grad[1], ctx.edges[0])
        need_b = ctx.has_bias and _wanted(ctx.needs_input_grad[2], ctx.edges[1])
        if ctx.twice and torch.is_grad_enabled():
            # create_graph (the SIREN eikonal term runs through sigma_linear): differentiable
            gy2 = gy.reshape(-1, J)
            gx = linear(gy, weight.t(), twice=True) if need_x else None
            gw = gy2.t().mm(x.reshape(-1, K)) if need_w else None
            gb = gy2.sum(0) if need_b else None
            return gx, gw, gb, None
        gx, gw, gb = _head_bwd(gy.reshape(-1, J).contiguous(), _a16(x.reshape(-1, K)),
                               _a16(weight), need_x, need_w, need_b)
        return (*_once(((gx.view(*lead, K) if gx is not None else None), gw, gb),
                       (gy, x, weight)), None)


def film_linear(x, weight, bias, gamma, beta, kernels=True, twice=False):
    """FiLMSiren's ``sin(gamma * F.linear(x, weight, bias) + beta)`` (sdf_model.py:62-67),
    gamma / beta [F, 1, ..., 1, N] broadcast over each face's samples: fused on the HIP
    kernels for the renderer MLP's training shapes (and ``kernels``), the reference's
    ops otherwise."""
    F_ = gamma.shape[0]
    if (kernels and _routable(x, weight) and x.shape[0] == F_ and gamma.shape[-1] == weight.shape[0]
            and gamma.numel() == F_ * weight.shape[0] and beta.shape == gamma.shape
            and weight.shape[1] > 32):
        return _FiLMLinearF16x3.apply(x, weight, bias, gamma, beta, twice)
    return torch.sin(gamma * linear(x, weight, bias, kernels, twice) + beta)


def _on_device(x: torch.Tensor) -> bool:
    return x.is_cuda


def _routable(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if _MODE["gemm"] != "f16x3" or not _on_device(x) or not torch.is_grad_enabled():
        return False
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() < 2:
        return False
    N, K = weight.shape
    # in features padded to a multiple of 4 (forward) and the input gradient's output
    # to 32 / 64 / 256 / 272 / 288 (_np_t): the shapes both directions take (ngp, siren,
    # and the FCGenerator's 60-wide x_in and 280-wide views layers)
    if N != 256 or not (K <= 64 or K == 256 or 256 < K <= 288):
        return False
    return x.numel() // K >= 1024            # the per-face gamma / beta layers stay on F.linear


def _head_routable(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if _MODE["gemm"] != "f16x3" or not _on_device(x) or not torch.is_grad_enabled():
        return False
    if x.dtype != torch.float32 or weight.dtype != torch.float32 or x.dim() < 2:
        return False
    J, K = weight.shape
    return J <= 4 and K % 4 == 0 and K <= 256 and x.numel() // K >= 1024


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None, kernels=True,
           twice=False) -> torch.Tensor:
    """F.linear(x, weight, bias), on the split-fp16 MFMA kernels for the renderer MLP's
    training shapes (module docstring) or the narrow-head kernels when ``kernels``, on
    F.linear otherwise.  ``twice``: the backward may itself be differentiated (a graph
    built by autograd.grad(create_graph=True) through this layer must reach its
    parameters: the SIREN eikonal term); otherwise it runs straight on the kernels."""
    if kernels and _routable(x, weight):
        return _LinearF16x3.apply(x, weight, bias, twice)
    if kernels and _head_routable(x, weight):
        return _LinearHead.apply(x, weight, bias, twice)
    return F.linear(x, weight, bias)
