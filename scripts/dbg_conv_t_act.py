"""Debug aid: sdfr_conv_t_act vs conv3x3_f16x3 + styled_epilogue, error breakdown."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from sdfr_loader import load  # noqa: E402

sdfr = load()
ops = sdfr.decoder_ops
DEV = "cuda:0"
L = sdfr._lib.lib()
L.sdfr_set_conv_t_mode(2)
B, Cin, Cout, H, W = 1, 64, 128, 16, 16
g = torch.Generator().manual_seed(5)
x = torch.randn(B, Cin, H, W, generator=g)
w = torch.randn(Cout, Cin, 3, 3, generator=g)
packed, su = ops.conv_pack_weights(w.to(DEV), 1 / math.sqrt(Cin * 9))
xs = ops.split_nhwc(x.to(DEV))
demod = (torch.rand(B, Cout, generator=g) + 0.5).to(DEV) / su
bias = (torch.randn(Cout, generator=g) * 0.1).to(DEV)
nw = torch.tensor([0.3]).to(DEV)
nz = torch.randn(B, 1, 2 * H, 2 * W, generator=g).to(DEV)
sn = (torch.rand(B, Cout, generator=g) + 0.5).to(DEV)
fir = [0.25, 0.75, 0.75, 0.25]
ys = torch.full((B, 2 * H, 2 * W, Cout // 8, 2, 8), 7.0, device=DEV, dtype=torch.float16)
raw = torch.full((B, 2 * H + 1, 2 * W + 1, Cout), 5.0, device=DEV)
a = sdfr._lib.ConvTActArgs()
P = sdfr._lib.ptr
a.x_split, a.packed = P(xs), P(packed)
a.B, a.H, a.W, a.Cin, a.Cout = B, H, W, Cin, Cout
for i in range(4):
    a.fir[i] = fir[i]
a.demod, a.noise, a.noise_weight, a.bias = P(demod), P(nz.contiguous()), P(nw), P(bias)
a.negative_slope, a.act_scale = 0.2, math.sqrt(2)
a.s_next, a.y_split, a.raw = P(sn), P(ys), P(raw)
sdfr._lib.check(L.sdfr_conv_t_act(a, sdfr._lib.stream_of(xs)), "conv_t_act")
ref_raw = ops.conv3x3_f16x3(xs, packed, Cout, transposed=True, split_k=False)
ref, _ = ops.styled_epilogue(ref_raw, fir=fir, bias=bias, noise_weight=nw, noise=nz, demod=demod,
                             blur_up=True, s_next=sn, store_y=True, split_y=True)
torch.cuda.synchronize()
rr = ref_raw.permute(0, 2, 3, 1)          # NHWC view [B, 2H+1, 2W+1, C]
band = (raw != 5.0).any(-1)[0]
print("raw written rows x cols:", band.sum().item())
print("raw rows written:", band.any(1).nonzero().flatten().tolist())
ok = (raw == rr)
print("raw band equal:", bool(ok[0][band].all()))
def unsplit(t):
    return (t[..., 0, :].float() + t[..., 1, :].float()).reshape(B, 2 * H, 2 * W, Cout)
yv, rv = unsplit(ys), unsplit(ref)
d = (yv - rv).abs()
print("untouched y (7.0):", int((ys[..., 0, :] == 7.0).all(-1).all(-1).sum()))
print("max diff", d.max().item(), "mean", d.mean().item())
print("row-wise max diff:", [round(v, 4) for v in d.amax(dim=(0, 2, 3)).tolist()])
print("col-wise max diff:", [round(v, 4) for v in d.amax(dim=(0, 1, 3)).tolist()])
print("chan-wise max diff (first 32):", [round(v, 4) for v in d.amax(dim=(0, 1, 2)).tolist()[:32]])
print("sample y vs ref at (5,5):", yv[0, 5, 5, :8].tolist(), rv[0, 5, 5, :8].tolist())

# --- diagnosis: demod 1, no bias / noise / s_next: y = lrelu(s) sqrt 2 -> recover s
print("---- recover s")
one = torch.ones(B, Cout, device=DEV)
zb = torch.zeros(Cout, device=DEV)
ys2 = torch.full_like(ys, 7.0)
a.demod, a.noise, a.bias, a.s_next, a.y_split = P(one), None, P(zb), None, P(ys2)
sdfr._lib.check(L.sdfr_conv_t_act(a, sdfr._lib.stream_of(xs)), "conv_t_act")
torch.cuda.synchronize()
v = unsplit(ys2) / math.sqrt(2)
s_got = torch.where(v > 0, v, v / 0.2)                        # [B, 2H, 2W, C]
rawc = rr[0].permute(2, 0, 1)                                 # [C, 2H+1, 2W+1]
f = torch.tensor(fir, device=DEV)
k2 = torch.outer(f, f).flip(0, 1)
pad = torch.nn.functional.pad(rawc[None], (1, 1, 1, 1))       # rows/cols -1 .. 2H+1
s_ref = torch.nn.functional.conv2d(pad.permute(1, 0, 2, 3), k2[None, None])[:, 0]  # [C, 2H, 2W]
s_ref = s_ref[:, :2 * H, :2 * W].permute(1, 2, 0)
d = (s_got[0] - s_ref).abs()
print("s err interior max", d[1:30, 1:30].max().item(), " border max", d[0].max().item())
for name, cand in [("h-only(rows Y)", None)]:
    pass
# candidates: vertical only (no horizontal), horizontal only
fh = torch.nn.functional.conv2d(pad.permute(1, 0, 2, 3), torch.outer(torch.tensor([0., 1, 0, 0], device=DEV), f.flip(0))[None, None])[:, 0][:, :2*H, :2*W].permute(1, 2, 0)
fv = torch.nn.functional.conv2d(pad.permute(1, 0, 2, 3), torch.outer(f.flip(0), torch.tensor([0., 1, 0, 0], device=DEV))[None, None])[:, 0][:, :2*H, :2*W].permute(1, 2, 0)
print("vs horizontal-only", (s_got[0] - fh).abs()[1:30, 1:30].max().item())
print("vs vertical-only", (s_got[0] - fv).abs()[1:30, 1:30].max().item())
print("s_got (5,5,:4)", s_got[0, 5, 5, :4].tolist(), "s_ref", s_ref[5, 5, :4].tolist())
print("raw (4..7, 4..7, ch0):", rawc[0, 4:8, 4:8].tolist())

# emulations (interior pixels): own raw class value, horizontal-only (both DPP senses)
print("---- emulations")
rc = rawc                                                   # [C, 2H+1, 2W+1]
own = rc[:, :2 * H, :2 * W].permute(1, 2, 0)
def hpass(sense):
    # horizontal filter at column X from cols X-1..X+2 (sense 1) or mirrored (sense -1)
    p_ = torch.nn.functional.pad(rc, (1, 2))
    cols = [p_[:, :, k:k + 2 * W + 1] for k in range(4)]
    if sense < 0:
        cols = cols[::-1]
    ff = fir[::-1]
    h = cols[0] * ff[0] + cols[1] * ff[1] + cols[2] * ff[2] + cols[3] * ff[3]
    return h[:, :2 * H, :2 * W].permute(1, 2, 0)
for name, e in (("own raw", own), ("horiz +", hpass(1)), ("horiz -", hpass(-1)), ("full", s_ref)):
    print(name, (s_got[0] - e).abs()[1:30, 1:30].max().item())
