"""Kernel-level parity of libmiattack against plain PyTorch fp32/fp64 references (GPU)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gfa_amd import _lib, layouts, ops
from oracle import attack_ref, stylegan2_ref

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 2e-5, torch.float16: 2e-2, torch.bfloat16: 8e-2}  # rel. to max |ref|


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def nhwc(x, dtype):
    return x.permute(0, 2, 3, 1).contiguous().to(dtype)


def nchw(y):
    return y.permute(0, 3, 1, 2).double()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,Cin,Cout", [(2, 8, 8, 64), (3, 17, 64, 128), (1, 16, 128, 192),
                                          (4, 4, 512, 512), (2, 33, 32, 8)])
def test_conv3x3_bias_relu(cuda, dtype, N, H, Cin, Cout):
    g = torch.Generator().manual_seed(N * 1000 + H * 10 + Cin)
    x = torch.randn(N, Cin, H, H + 1, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    b = torch.randn(Cout, generator=g) * 0.1
    xq = x.to(dtype).double()
    wq = w.to(dtype).double()
    ref = F.relu(F.conv2d(xq, wq, b.double(), padding=1))
    y = torch.empty(N, H, H + 1, Cout, dtype=dtype, device=cuda)
    ops.conv3x3(nhwc(x, dtype).to(cuda), layouts.fwd_matrix(w, dtype).to(cuda), y, cout=Cout,
                bias=b.to(cuda), act_out=ops.ACT_RELU)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,W,Cin,Cout", [(2, 16, 16, 64, 64), (1, 32, 48, 128, 192),
                                            (2, 16, 32, 256, 128), (1, 48, 16, 64, 128),
                                            (2, 32, 16, 64, 8), (1, 16, 16, 128, 24)])
@pytest.mark.parametrize("mode", ["bias_relu", "modconv", "dgrad_sdot", "tap_mask"])
@pytest.mark.parametrize("halo", ["1", "0"])
def test_conv3x3_halo_and_generic_paths(cuda, tune, dtype, N, H, W, Cin, Cout, mode, halo):
    """Stride-1 3×3 layers on 16-divisible maps take the halo-tiled kernel (conv_halo.hip) unless
    MIA_CONV_HALO=0; both paths, with every epilogue feature the attack uses, against torch."""
    tune("MIA_CONV_HALO", halo)
    g = torch.Generator().manual_seed(N * 7 + H + W + Cin + Cout)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    xd = nhwc(x, dtype).to(cuda)
    wf = layouts.fwd_matrix(w, dtype).to(cuda)
    y = torch.empty(N, H, W, Cout, dtype=dtype, device=cuda)
    tol = 2 * TOL[dtype]
    if mode == "bias_relu":
        b = torch.randn(Cout, generator=g) * 0.1
        ref = F.relu(F.conv2d(xq, wq, b.double(), padding=1))
        ops.conv3x3(xd, wf, y, cout=Cout, bias=b.to(cuda), act_out=ops.ACT_RELU)
    elif mode == "modconv":
        s = torch.rand(N, Cin, generator=g) + 0.5
        d = torch.rand(N, Cout, generator=g) + 0.5
        nz = torch.randn(H * W, generator=g)
        b = torch.randn(Cout, generator=g) * 0.1
        pre = F.conv2d(xq * s.double().view(N, Cin, 1, 1), wq, padding=1) * d.double().view(
            N, Cout, 1, 1) + 0.3 * nz.double().view(1, 1, H, W) + b.double().view(1, -1, 1, 1)
        ref = F.leaky_relu(pre, 0.2) * math.sqrt(2)
        ops.conv3x3(xd, wf, y, cout=Cout, in_scale=s.to(cuda), out_scale=d.to(cuda),
                    noise=nz.to(cuda), noise_w=0.3, bias=b.to(cuda), act_out=ops.ACT_LRELU_S2)
    elif mode == "dgrad_sdot":
        s = torch.rand(N, Cout, generator=g) + 0.5
        aux = torch.randn(N, Cout, H, W, generator=g)
        conv = F.conv2d(xq, wq, padding=1)
        ref = conv * s.double().view(N, Cout, 1, 1)
        sd_ref = (conv * aux.to(dtype).double()).sum((2, 3))
        sd = torch.zeros(N, Cout, device=cuda)
        ops.conv3x3(xd, wf, y, cout=Cout, out_scale=s.to(cuda), aux_x=nhwc(aux, dtype).to(cuda),
                    sdot=sd)
    else:
        a = torch.randn(N, Cout, H, W, generator=g).relu()
        t = torch.randn(N, Cout, H, W, generator=g)
        aq, tq = a.to(dtype).double(), t.to(dtype).double()
        ref = (F.conv2d(xq, wq, padding=1) + 0.37 * (aq - tq)) * (aq > 0)
        ops.conv3x3(xd, wf, y, cout=Cout, tap_a=nhwc(a, dtype).to(cuda),
                    tap_t=nhwc(t, dtype).to(cuda), tap_coef=0.37, mask_a=nhwc(a, dtype).to(cuda))
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < tol
    if mode == "dgrad_sdot":
        assert rel_err(sd, sd_ref) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_conv3x3_dgrad_tap_mask(cuda, dtype):
    g = torch.Generator().manual_seed(7)
    N, H, Cin, Cout = 2, 12, 64, 128
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    gout = torch.randn(N, Cout, H, H, generator=g)
    a = torch.randn(N, Cin, H, H, generator=g).relu()
    t = torch.randn(N, Cin, H, H, generator=g)
    coef = 0.37
    wq, gq = w.to(dtype).double(), gout.to(dtype).double()
    aq, tq = a.to(dtype).double(), t.to(dtype).double()
    xx = torch.zeros(N, Cin, H, H, dtype=torch.float64, requires_grad=True)
    (gx,) = torch.autograd.grad((F.conv2d(xx, wq, padding=1) * gq).sum(), xx)
    ref = (gx + coef * (aq - tq)) * (aq > 0)
    y = torch.empty(N, H, H, Cin, dtype=dtype, device=cuda)
    ops.conv3x3(nhwc(gout, dtype).to(cuda), layouts.dgrad_matrix(w, dtype).to(cuda), y, cout=Cin,
                tap_a=nhwc(a, dtype).to(cuda), tap_t=nhwc(t, dtype).to(cuda), tap_coef=coef,
                mask_a=nhwc(a, dtype).to(cuda))
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < TOL[dtype]


def _modconv_setup(seed, N, cin, cout, R):
    g = torch.Generator().manual_seed(seed)
    p = {
        "m.weight": torch.randn(1, cout, cin, 3, 3, generator=g),
        "m.modulation.weight": torch.randn(cin, 512, generator=g),
        "m.modulation.bias": torch.ones(cin),
    }
    wlat = torch.randn(N, 512, generator=g)
    x = torch.randn(N, cin, R, R, generator=g)
    noise = torch.randn(1, 1, 2 * R, 2 * R, generator=g)
    bias = 0.1 * torch.randn(cout, generator=g)
    return p, wlat, x, noise, bias


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("up", [False, True])
def test_modconv_fwd(cuda, dtype, up):
    N, cin, cout, R = 3, 64, 128, 8
    p, wlat, x, noise, bias = _modconv_setup(11, N, cin, cout, R)
    Ro = 2 * R if up else R
    noise = noise[..., :Ro, :Ro].contiguous()
    # reference: the oracle's per-sample formulation on lrelu·√2(x) (stored pre-activations)
    xa = F.leaky_relu(x.double(), 0.2) * math.sqrt(2)
    ref = stylegan2_ref.modulated_conv2d({k: v.double() for k, v in p.items()}, "m", xa,
                                         wlat.double(), demodulate=True, upsample=up)
    ref = ref + 0.1 * noise.double() + bias.double().view(1, -1, 1, 1)
    # device path
    scale = 1.0 / math.sqrt(cin * 9)
    ws = p["m.weight"][0].double() * scale
    wm = layouts.upconv_phases(ws) if up else ws
    s = F.linear(wlat.double(), p["m.modulation.weight"].double() / math.sqrt(512),
                 p["m.modulation.bias"].double()).float().to(cuda)
    wsq = (ws ** 2).sum((2, 3)).float().to(cuda)
    demod = torch.empty(N, cout, device=cuda)
    ops.style_demod(s, wsq, demod)
    y = torch.empty(N, Ro, Ro, cout, dtype=dtype, device=cuda)
    ops.conv3x3(nhwc(x, dtype).to(cuda), layouts.fwd_matrix(wm, dtype).to(cuda), y,
                cout=4 * cout if up else cout, act_in=ops.ACT_LRELU_S2, in_scale=s,
                out_scale=demod, noise=noise.reshape(-1).to(cuda), noise_w=0.1,
                bias=bias.to(cuda), shuffle_out=up)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,cin,cout,R", [(3, 128, 128, 32), (2, 256, 256, 16), (2, 64, 128, 48)])
def test_modconv_fwd_per_image_weights(cuda, dtype, N, cin, cout, R):
    """The StyledConv forward on per-image modulated + demodulated weights (mia_modulate_weights
    + mia_conv3x3_wmod, the fp16 / bf16 synthesis at ≥ 128²) against the fp64 oracle's
    per-sample modulated_conv2d (rosinality's weight path) and the halo kernel's LDS-modulated
    form of the same layer; the epilogue (noise, bias, lrelu·√2) as the generator stores it."""
    p, wlat, x, noise, bias = _modconv_setup(13, N, cin, cout, R)
    noise = noise[..., :R, :R].contiguous()
    xa = F.leaky_relu(x.double(), 0.2) * math.sqrt(2)  # the stored activation of the layer below
    pre = stylegan2_ref.modulated_conv2d({k: v.double() for k, v in p.items()}, "m", xa,
                                         wlat.double(), demodulate=True)
    ref = F.leaky_relu(pre + 0.1 * noise.double() + bias.double().view(1, -1, 1, 1),
                       0.2) * math.sqrt(2)
    scale = 1.0 / math.sqrt(cin * 9)
    ws = p["m.weight"][0].double() * scale
    s = F.linear(wlat.double(), p["m.modulation.weight"].double() / math.sqrt(512),
                 p["m.modulation.bias"].double()).float().to(cuda)
    wsq = (ws ** 2).sum((2, 3)).float().to(cuda)
    demod = torch.empty(N, cout, device=cuda)
    ops.style_demod(s, wsq, demod)
    wf = layouts.fwd_matrix(ws, dtype).to(cuda)
    xd = nhwc(xa, dtype).to(cuda)
    kw = dict(cout=cout, in_scale=s, out_scale=demod, noise=noise.reshape(-1).to(cuda),
              noise_w=0.1, bias=bias.to(cuda), act_out=ops.ACT_LRELU_S2)
    y = torch.empty(N, R, R, cout, dtype=dtype, device=cuda)
    wm = torch.empty((N,) + tuple(wf.shape), dtype=dtype, device=cuda)
    ops.conv3x3_modw(xd, wf, y, wm, **kw)
    y_lds = torch.empty_like(y)
    ops.conv3x3(xd, wf, y_lds, **kw)
    torch.cuda.synchronize()
    # the weights themselves: (w·s)·demod in fp32, rounded once to the dtype (within 1 ulp of
    # torch's rounding of the same fp32 product); exactly 0 in the padding
    K = 9 * cin
    wref = torch.zeros(wm.shape, dtype=torch.float32, device=cuda)
    wref[:, :, :K] = wf[:, :K].float()[None] * s.repeat(1, 9)[:, None, :] * demod[:, :, None]
    ulp = 2.0 ** (-10 if dtype == torch.float16 else -7)
    dw = (wm.float() - wref.to(dtype).float()).abs()
    n_ne = int((wm != wref.to(dtype)).sum())
    print(f"per-image weights {dtype}: {n_ne} of {wm.numel()} differ from torch's rounding")
    assert (dw <= wref.abs() * ulp + 2.0 ** -24).all()
    assert (wm[:, :, K:] == 0).all()
    e_w, e_lds = rel_err(nchw(y), ref), rel_err(nchw(y_lds), ref)
    print(f"per-image weights {dtype} {N}x{R}² {cin}->{cout}: rel err {e_w:.2e} "
          f"(LDS-modulated {e_lds:.2e})")
    assert e_w < 2 * TOL[dtype] and e_w < 2 * e_lds + 1e-3
    with pytest.raises(_lib.MiaError):  # not a halo-kernel shape: refused, no fallback
        ops.conv3x3_modw(xd[:, :R - 8, :R - 8].contiguous(), wf,
                         torch.empty(N, R - 8, R - 8, cout, dtype=dtype, device=cuda), wm,
                         **dict(kw, noise=None))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,R,W,C", [(20, 64, 64, 128), (3, 256, 256, 128), (5, 40, 48, 128),
                                     (1, 8, 16, 128), (2, 16, 32, 128)])
def test_wres128_modconv_fwd(cuda, tune, dtype, N, R, W, C):
    """The weights-resident StyledConv forward (conv_wres128.hip: 128 → 128, the 256² layer of the
    fp16 / bf16 synthesis) on per-image weights: persistent runs that cross image boundaries
    (weights reloaded mid-run), patches on a map that is not a halo shape (R = 40), against (a) a torch fp32 GPU conv of the same
    rounded operands and per-image weights + the same epilogue, and (b) the halo tile
    (MIA_CONV_WRES128=0) on the same weights: both accumulate in fp32 in different orders, so the
    outputs agree to the output rounding."""
    cin = cout = C
    g = torch.Generator().manual_seed(N * 31 + R)
    x = torch.randn(N, R, W, cin, generator=g).to(dtype)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    s = (torch.rand(N, cin, generator=g) + 0.5)
    noise = torch.randn(R * W, generator=g)
    bias = 0.1 * torch.randn(cout, generator=g)
    wf = layouts.fwd_matrix(w.double(), dtype).to(cuda)
    wsq = (w.double() ** 2).sum((2, 3)).float().to(cuda)
    s_d = s.to(cuda)
    demod = torch.empty(N, cout, device=cuda)
    ops.style_demod(s_d, wsq, demod)
    xd = x.to(cuda)
    kw = dict(cout=cout, in_scale=s_d, out_scale=demod, noise=noise.to(cuda), noise_w=0.3,
              bias=bias.to(cuda), act_out=ops.ACT_LRELU_S2)
    wm = torch.empty((N,) + tuple(wf.shape), dtype=dtype, device=cuda)
    y = torch.empty(N, R, W, cout, dtype=dtype, device=cuda)
    ops.conv3x3_modw(xd, wf, y, wm, **kw)
    tune("MIA_CONV_WRES128", 0)
    y_halo = torch.empty_like(y)
    wm2 = torch.empty_like(wm)
    if R % 16 == 0:
        ops.conv3x3_modw(xd, wf, y_halo, wm2, **kw)
    torch.cuda.synchronize()
    # fp32 reference on the device's own per-image weights (grouped conv: one group per image)
    K = 9 * cin
    wr = wm[:, :, :K].float().view(N, cout, 3, 3, cin).permute(0, 1, 4, 2, 3)
    ref = F.conv2d(xd.float().permute(0, 3, 1, 2).reshape(1, N * cin, R, W),
                   wr.reshape(N * cout, cin, 3, 3), padding=1, groups=N).view(N, cout, R, W)
    ref = F.leaky_relu(ref + 0.3 * noise.to(cuda).view(1, 1, R, W) + bias.to(cuda).view(1, -1, 1, 1),
                       0.2) * math.sqrt(2)
    e_ref = rel_err(nchw(y), ref)
    ulp = 2.0 ** (-10 if dtype == torch.float16 else -7)
    print(f"wres128 {dtype} {N}x{R}x{W}: rel err vs fp32 {e_ref:.2e}")
    assert e_ref < 2 * ulp
    if R % 16 == 0:
        assert torch.equal(wm, wm2)
        d = (y.float() - y_halo.float()).abs()
        lim = y_halo.float().abs() * (2 * ulp) + 2 * ulp * float(y_halo.float().abs().max()) * 1e-3
        print(f"wres128 vs halo: max |diff| {float(d.max()):.3e}, "
              f"{int((y != y_halo).sum())} of {y.numel()} differ")
        assert (d <= lim + 1e-6).all()


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,R,W,with_noise", [(20, 64, 64, True), (2, 256, 256, True),
                                               (3, 40, 48, False), (1, 8, 16, True),
                                               (2, 16, 16, False)])
def test_wres128_dgrad_sdot_bab(cuda, tune, dtype, N, R, W, with_noise):
    """The weights-resident kernel's StyledConv input gradient (OSC | SDOT | BAB: the 256² block's
    dgrad with the style-gradient dot and the fused backward front of the layer below) against
    the halo tile on the same operands (MIA_CONV_WRES128=0; R = 40 is not a halo shape, so there
    against the fp32 torch formula only) and against fp32 torch: the stored output to the output
    rounding, the ordered sdot / q sums to fp32 summation-order noise."""
    C = 128
    g = torch.Generator().manual_seed(N * 7 + R)
    gy = (torch.randn(N, R, W, C, generator=g) * 0.5).to(dtype)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    ax = (torch.randn(N, R, W, C, generator=g)).to(dtype)
    s = torch.rand(N, C, generator=g) + 0.5
    dm = torch.rand(N, C, generator=g) + 0.5
    nz = torch.randn(R * W, generator=g)
    bb = 0.1 * torch.randn(C, generator=g)
    wd = layouts.dgrad_matrix(w.double(), dtype).to(cuda)

    def run():
        y = torch.empty(N, R, W, C, dtype=dtype, device=cuda)
        sd = torch.zeros(N, C, device=cuda)
        q = torch.zeros(N, C, device=cuda)
        bab = dict(demod=dm.to(cuda), q=q, bias=bb.to(cuda))
        if with_noise:
            bab.update(noise=nz.to(cuda), noise_w=0.3)
        ops.conv3x3(gy.to(cuda), wd, y, cout=C, out_scale=s.to(cuda), aux_x=ax.to(cuda),
                    sdot=sd, bab=bab)
        torch.cuda.synchronize()
        return y, sd, q

    y, sd, q = run()
    # fp32 reference: gx = dgrad(gy); sdot = Σ gx·x; v = gx·s; front of the layer below
    wq = w.to(dtype).float().to(cuda)
    gyf = gy.float().to(cuda).permute(0, 3, 1, 2)
    xx = torch.zeros(N, C, R, W, device=cuda, requires_grad=True)
    (gx,) = torch.autograd.grad((F.conv2d(xx, wq, padding=1) * gyf).sum(), xx)
    xv = ax.float().to(cuda).permute(0, 3, 1, 2)
    sd_ref = (gx * xv).sum((2, 3))
    v = gx * s.to(cuda).view(N, C, 1, 1)
    gr = torch.where(xv > 0, math.sqrt(2), 0.2 * math.sqrt(2))
    gp = v * gr
    inv = torch.where(xv > 0, 1 / math.sqrt(2), 1 / (0.2 * math.sqrt(2)))
    z = (0.3 * nz.to(cuda).view(1, 1, R, W)) if with_noise else 0.0
    q_ref = (gp * (xv * inv - z - bb.to(cuda).view(1, C, 1, 1))).sum((2, 3))
    y_ref = gp * dm.to(cuda).view(N, C, 1, 1)
    e_y, e_s, e_q = rel_err(nchw(y), y_ref), rel_err(sd, sd_ref), rel_err(q, q_ref)
    print(f"wres128 dgrad {dtype} {N}x{R}x{W}: rel err y {e_y:.2e} sdot {e_s:.2e} q {e_q:.2e}")
    ulp = 2.0 ** (-10 if dtype == torch.float16 else -7)
    assert e_y < 2 * ulp and e_s < 1e-4 and e_q < 1e-4
    if R % 16 == 0:
        tune("MIA_CONV_WRES128", 0)
        y2, sd2, q2 = run()
        d = (y.float() - y2.float()).abs()
        print(f"wres128 vs halo dgrad: {int((y != y2).sum())} of {y.numel()} outputs differ, "
              f"max {float(d.max()):.2e}; sdot {rel_err(sd, sd2):.2e} q {rel_err(q, q2):.2e}")
        assert (d <= y2.float().abs() * (2 * ulp) + 1e-6).all()
        assert rel_err(sd, sd2) < 1e-5 and rel_err(q, q2) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("up", [False, True])
@pytest.mark.parametrize("store_act", [False, True])
def test_modconv_bwd_input_and_style(cuda, dtype, up, store_act):
    """bias_act_bwd + dgrad(sdot) + demod_bwd reproduce autograd's ∂x and ∂s of a StyledConv.
    store_act: the layout SynthesisNet uses — the producing epilogue stores a = lrelu(pre)·√2 and
    the backward recovers pre from it (from_act)."""
    N, cin, cout, R = 2, 32, 64, 8
    p, wlat, x, noise, bias = _modconv_setup(5, N, cin, cout, R)
    Ro = 2 * R if up else R
    noise = noise[..., :Ro, :Ro].contiguous()
    g = torch.Generator().manual_seed(99)
    g_a = torch.randn(N, cout, Ro, Ro, generator=g)
    pd = {k: v.double() for k, v in p.items()}
    scale = 1.0 / math.sqrt(cin * 9)
    x_in = x.double().clone().requires_grad_(True)
    s_in = F.linear(wlat.double(), pd["m.modulation.weight"] / math.sqrt(512),
                    pd["m.modulation.bias"]).requires_grad_(True)
    xa = F.leaky_relu(x_in, 0.2) * math.sqrt(2)
    xa.retain_grad()
    # per-sample formulation with style given explicitly
    wt = scale * pd["m.weight"] * s_in.view(N, 1, cin, 1, 1)
    dm = torch.rsqrt(wt.pow(2).sum([2, 3, 4]) + 1e-8)
    wt = (wt * dm.view(N, cout, 1, 1, 1))
    if up:
        wt2 = wt.transpose(1, 2).reshape(N * cin, cout, 3, 3)
        o = F.conv_transpose2d(xa.reshape(1, N * cin, R, R), wt2, stride=2, groups=N)
        o = o.view(N, cout, o.shape[2], o.shape[3])
        o = stylegan2_ref.upfirdn2d(o, stylegan2_ref.make_kernel([1, 3, 3, 1], torch.float64) * 4,
                                    pad=(1, 1))
    else:
        o = F.conv2d(xa.reshape(1, N * cin, R, R), wt.reshape(N * cout, cin, 3, 3), padding=1,
                     groups=N).view(N, cout, R, R)
    pre = o + 0.1 * noise.double() + bias.double().view(1, -1, 1, 1)
    act = F.leaky_relu(pre, 0.2) * math.sqrt(2)
    # the dgrad epilogue returns ∂L/∂(activation of the previous layer); its lrelu' is applied by
    # that layer's bias_act_bwd
    gx_ref, gs_ref = torch.autograd.grad((act * g_a.double()).sum(), [xa, s_in])
    # device path
    ws_ = pd["m.weight"][0] * scale
    wm = layouts.upconv_phases(ws_) if up else ws_
    s = s_in.detach().float().to(cuda)
    wsq = (ws_ ** 2).sum((2, 3)).float().to(cuda)
    demod = torch.empty(N, cout, device=cuda)
    ops.style_demod(s, wsq, demod)
    xd = nhwc(x, dtype).to(cuda)
    pre_d = torch.empty(N, Ro, Ro, cout, dtype=dtype, device=cuda)
    nz = noise.reshape(-1).to(cuda)
    bz = bias.to(cuda)
    ops.conv3x3(xd, layouts.fwd_matrix(wm, dtype).to(cuda), pre_d, cout=4 * cout if up else cout,
                act_in=ops.ACT_LRELU_S2, in_scale=s, out_scale=demod, noise=nz, noise_w=0.1,
                bias=bz, shuffle_out=up, act_out=ops.ACT_LRELU_S2 if store_act else ops.ACT_NONE)
    q = torch.zeros(N, cout, device=cuda)
    gy = torch.empty((N, R, R, 4 * cout) if up else (N, R, R, cout), dtype=dtype, device=cuda)
    ops.bias_act_bwd(nhwc(g_a, dtype).to(cuda), pre_d, nz, 0.1, bz, demod, gy, q, unshuffle=up,
                     from_act=store_act)
    gs = torch.zeros(N, cin, device=cuda)
    gx = torch.empty(N, R, R, cin, dtype=dtype, device=cuda)
    ops.conv3x3(gy, layouts.dgrad_matrix(wm, dtype).to(cuda), gx, cout=cin, out_scale=s, aux_x=xd,
                act_aux=ops.ACT_LRELU_S2, sdot=gs)
    ops.demod_bwd(q, demod, wsq, s, gs)
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 5e-2
    assert rel_err(nchw(pre_d), (act if store_act else pre).detach()) < tol
    assert rel_err(nchw(gx), gx_ref) < tol
    assert rel_err(gs, gs_ref) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,ceil,tap", [(8, False, True), (9, True, True), (9, False, True),
                                        (36, False, True), (7, True, False), (10, False, False)])
def test_maxpool_fwd_bwd(cuda, dtype, H, ceil, tap):
    """First-max rule with ties, ceil and floor modes on odd sizes, with and without the fused
    tap-MSE term + ReLU mask."""
    g = torch.Generator().manual_seed(H)
    N, C = 2, 16
    x = torch.randn(N, C, H, H, generator=g).relu()
    x[:, :, 0:2, 0:2] = 0.5  # ties → first max wins
    xq = x.to(dtype).double().requires_grad_(True)
    y = F.max_pool2d(xq, 2, 2, ceil_mode=ceil)
    go = torch.randn(y.shape, generator=g, dtype=torch.float64).to(dtype).double()
    t = torch.randn(N, C, H, H, generator=g)
    (gx,) = torch.autograd.grad((y * go).sum(), xq)
    if tap:
        ref_b = (gx + 0.5 * (xq.detach() - t.to(dtype).double())) * (xq.detach() > 0)
    else:
        ref_b = gx
    xd = nhwc(x, dtype).to(cuda)
    yd = torch.empty(N, y.shape[2], y.shape[3], C, dtype=dtype, device=cuda)
    ops.maxpool2_fwd(xd, yd, ceil_mode=ceil)
    gi = torch.full_like(xd, float("nan"))  # every element must be written
    ops.maxpool2_bwd(xd, nhwc(go, dtype).to(cuda), gi, ceil_mode=ceil,
                     tap_t=nhwc(t, dtype).to(cuda) if tap else None, tap_coef=0.5 if tap else 0.0,
                     mask=tap)
    torch.cuda.synchronize()
    assert torch.equal(nchw(yd).cpu(), y.detach())
    assert rel_err(nchw(gi), ref_b) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("S,pf,cpad", [(16, 1, 8), (64, 4, 8), (32, 2, 3), (48, 1, 16)])
def test_image_to_nhwc(cuda, dtype, S, pf, cpad):
    """mia_image_to_nhwc (NCHW image → avg_pool(pf) → NHWC, channels ≥ 3 zero): both forms (the
    16-byte-vector one for cpad a multiple of the vector, the element one otherwise) against the
    same sums in the same order on the host — bit-exact."""
    g = torch.Generator().manual_seed(S + pf + cpad)
    N = 3
    x = torch.rand(N, 3, S, S, generator=g) * 2 - 1
    R = S // pf
    acc = torch.zeros(N, 3, R, R)
    for dy in range(pf):
        for dx in range(pf):
            acc = acc + x[:, :, dy::pf, dx::pf]
    ref = torch.zeros(N, R, R, cpad)
    ref[..., :3] = (acc * (1.0 / (pf * pf))).permute(0, 2, 3, 1)
    y = torch.full((N, R, R, cpad), 7.0, dtype=dtype, device=cuda)
    ops.image_to_nhwc(x.to(cuda), y, pf, cpad)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), ref.to(dtype))


@pytest.mark.parametrize("up,down,pad", [(2, 1, (2, 1)), (1, 1, (1, 1)), (1, 2, (1, 1)),
                                         (2, 2, (1, 2))])
def test_upfirdn2d(cuda, up, down, pad):
    g = torch.Generator().manual_seed(3)
    k1 = [1.0, 3.0, 3.0, 1.0]
    kn = [v / 4.0 for v in k1]
    x = torch.randn(2, 3, 9, 9, generator=g, dtype=torch.float64).requires_grad_(True)
    k2 = torch.tensor(kn, dtype=torch.float64)
    k2 = k2[:, None] * k2[None, :]
    ref = stylegan2_ref.upfirdn2d(x, k2, up=up, down=down, pad=pad)
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (gx,) = torch.autograd.grad((ref * gy).sum(), x)
    y = torch.empty(ref.shape, device=cuda)
    ops.upfirdn2d_fwd(x.detach().float().to(cuda), y, kn, up=up, down=down, pad=pad)
    gxd = torch.empty(x.shape, device=cuda)
    ops.upfirdn2d_bwd(gy.float().to(cuda), gxd, kn, up=up, down=down, pad=pad)
    torch.cuda.synchronize()
    assert rel_err(y, ref.detach()) < 1e-5
    assert rel_err(gxd, gx) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cin", [8, 16, 32, 128, 512])  # 1 … 64 lanes per pixel (every level count)
@pytest.mark.parametrize("stored", ["pre", "act"])
def test_torgb_fwd_bwd(cuda, dtype, cin, stored):
    g = torch.Generator().manual_seed(cin)
    N, R = 2, 8
    pre = torch.randn(N, cin, R, R, generator=g)
    s = torch.randn(N, cin, generator=g, dtype=torch.float64).requires_grad_(True)
    wr = torch.randn(3, cin, generator=g, dtype=torch.float64) / math.sqrt(cin)
    b = torch.randn(3, generator=g, dtype=torch.float64)
    skip = torch.randn(N, 3, R // 2, R // 2, generator=g, dtype=torch.float64)
    preq = pre.to(dtype).double().requires_grad_(True)
    a = F.leaky_relu(preq, 0.2) * math.sqrt(2)
    wm = wr.view(1, 3, cin) * s.view(N, 1, cin)
    out = torch.einsum("nchw,noc->nohw", a, wm) + b.view(1, 3, 1, 1)
    up = torch.tensor([1.0, 3.0, 3.0, 1.0], dtype=torch.float64)
    up = (up[:, None] * up[None, :]) / 16.0
    out = out + stylegan2_ref.upfirdn2d(skip, up, up=2, pad=(2, 1))
    grgb = torch.randn(out.shape, generator=g, dtype=torch.float64)
    gpre, gsr = torch.autograd.grad((out * grgb).sum(), [a, s])  # ∂L/∂activation, ∂L/∂s
    act_in = ops.ACT_NONE if stored == "act" else ops.ACT_LRELU_S2
    pd = nhwc(a.detach() if stored == "act" else pre, dtype).to(cuda)
    rgb = torch.empty(N, 3, R, R, device=cuda)
    sd = s.detach().float().to(cuda)
    wrd = wr.float().to(cuda)
    ops.torgb_fwd(pd, sd, wrd, b.float().to(cuda), skip.float().to(cuda), rgb, act_in=act_in)
    ga = torch.full((N, R, R, cin), 0.25, dtype=dtype, device=cuda)
    gs = torch.zeros(N, cin, device=cuda)
    ops.torgb_bwd(grgb.float().to(cuda), pd, sd, wrd, ga, gs, accumulate=True, act_in=act_in)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel_err(rgb, out.detach()) < tol
    assert rel_err(nchw(ga) - 0.25, gpre) < tol
    assert rel_err(gs, gsr) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cin,R", [(32, 16), (64, 9), (128, 8)])
def test_torgb_bwd_front(cuda, dtype, cin, R):
    """mia_torgb_bwd_front == mia_torgb_bwd then mia_bias_act_bwd(from_act) (the topmost conv)."""
    g = torch.Generator().manual_seed(cin + R)
    N = 3
    a = F.leaky_relu(torch.randn(N, R, R, cin, generator=g), 0.2) * math.sqrt(2)
    ad = a.to(dtype).to(cuda)
    sd = torch.randn(N, cin, generator=g).to(cuda)
    wr = (torch.randn(3, cin, generator=g) / math.sqrt(cin)).to(cuda)
    grgb = torch.randn(N, 3, R, R, generator=g).to(cuda)
    demod = (torch.rand(N, cin, generator=g) + 0.5).to(cuda)
    nz = torch.randn(R * R, generator=g).to(cuda)
    bz = torch.randn(cin, generator=g).to(cuda)
    ga = torch.empty(N, R, R, cin, dtype=dtype, device=cuda)
    gs1 = torch.zeros(N, cin, device=cuda)
    ops.torgb_bwd(grgb, ad, sd, wr, ga, gs1, accumulate=False, act_in=ops.ACT_NONE)
    gy1 = torch.empty_like(ga)
    q1 = torch.zeros(N, cin, device=cuda)
    ops.bias_act_bwd(ga, ad, nz, 0.3, bz, demod, gy1, q1, from_act=True)
    gy2 = torch.empty_like(ga)
    gs2 = torch.zeros(N, cin, device=cuda)
    q2 = torch.zeros(N, cin, device=cuda)
    ops.torgb_bwd_front(grgb, ad, sd, wr, gy2, gs2, demod, nz, 0.3, bz, q2)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2  # reference path rounds g_a to dtype
    assert rel_err(gs2, gs1) < 1e-5
    assert rel_err(gy2, gy1) < tol
    assert rel_err(q2, q1) < tol


def test_sign_project_bit_exact(cuda):
    """K11 vs the oracle's torch fp32 formula, including g == 0 and the clamp edges."""
    g = torch.Generator().manual_seed(0)
    n = 1 << 16
    x0 = (torch.rand(n, generator=g) * 2 - 1)
    x0[:64] = 1.0
    x0[64:128] = -1.0
    x = (x0 + (torch.rand(n, generator=g) * 2 - 1) * 0.05).clamp(-1, 1)
    gr = torch.randn(n, generator=g)
    gr[::7] = 0.0
    e, a = 2 * 8 / 255, 2 * 2 / 255
    ref = attack_ref.project_step(x, x0, gr, e, a)
    xd = x.to(cuda)
    ops.sign_project(xd, x0.to(cuda), gr.to(cuda), float(np.float32(a)), float(np.float32(e)))
    u = torch.rand(n, generator=g) * 2 - 1
    ref_rs = torch.clamp(x0 + float(np.float32(e)) * u, -1.0, 1.0)
    rs = torch.empty(n, device=cuda)
    ops.random_start(rs, x0.to(cuda), u.to(cuda), float(np.float32(e)))
    torch.cuda.synchronize()
    assert torch.equal(xd.cpu(), ref)
    assert torch.equal(rs.cpu(), ref_rs)


def test_gemm_and_demod(cuda):
    g = torch.Generator().manual_seed(1)
    A = torch.randn(37, 70, generator=g)
    B = torch.randn(70, 45, generator=g)
    bias = torch.randn(45, generator=g)
    C = torch.randn(37, 45, generator=g)
    Cd = C.clone().to(cuda)
    ops.gemm(37, 45, 70, 0.5, A.to(cuda), 70, 1, B.to(cuda), 45, 1, 2.0, Cd, 45, 1, bias.to(cuda))
    Bt = B.t().contiguous().to(cuda)  # strided access: B[k][n] = Bt[n][k]
    C2 = torch.empty(37, 45, device=cuda)
    ops.gemm(37, 45, 70, 1.0, A.to(cuda), 70, 1, Bt, 1, 70, 0.0, C2, 45, 1)
    s = torch.randn(4, 64, generator=g)
    wsq = torch.rand(96, 64, generator=g)
    d = torch.empty(4, 96, device=cuda)
    ops.style_demod(s.to(cuda), wsq.to(cuda), d, scale2=0.3)
    torch.cuda.synchronize()
    assert rel_err(Cd, 0.5 * A @ B + 2.0 * C + bias) < 1e-5
    assert rel_err(C2, A @ B) < 1e-5
    assert rel_err(d, torch.rsqrt(0.3 * (s ** 2) @ wsq.t() + 1e-8)) < 1e-5


@pytest.mark.parametrize("M,n_groups", [(7, 3), (128, 14), (300, 20)])
def test_gemm_grouped_two_segments(cuda, M, n_groups):
    """Grouped GEMM: per group C = α(A1·B1 + A2·B2) + βC + bias with strided views; > 12 groups
    exercises the launch split, M = 300 the 64-tile path, M = 7 the 32-tile path."""
    g = torch.Generator().manual_seed(M)
    plan = ops.GemmPlan()
    want, outs = [], []
    lat = torch.randn(M, n_groups, 40, generator=g)
    latd = lat.to(cuda)
    for i in range(n_groups):
        N, K1, K2 = 33 + 7 * i, 19 + i, 40
        A1 = torch.randn(M, K1, generator=g)
        B1 = torch.randn(N, K1, generator=g)  # used transposed (k-fast)
        B2 = torch.randn(K2, N, generator=g)
        C = torch.randn(M, N, generator=g)
        bias = torch.randn(N, generator=g)
        two = i % 2 == 0
        ref = 0.5 * (A1 @ B1.t() + (lat[:, i, :] @ B2 if two else 0)) + 2.0 * C + bias
        Cd = C.to(cuda)
        segs = [(A1.to(cuda), K1, 1, B1.to(cuda), 1, K1, K1)]
        if two:
            segs.append((latd[:, i, :], n_groups * 40, 1, B2.to(cuda), N, 1, K2))
        plan.add(Cd, N, 1, M, N, segs, alpha=0.5, beta=2.0, bias=bias.to(cuda))
        want.append(ref)
        outs.append(Cd)
    plan.run()
    torch.cuda.synchronize()
    for r, o in zip(want, outs):
        assert rel_err(o, r) < 1e-5


def test_adam_step(cuda):
    g = torch.Generator().manual_seed(2)
    p = torch.randn(1000, generator=g)
    grads = [torch.randn(1000, generator=g) for _ in range(3)]
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=0.005)
    pd, m, v = p.to(cuda), torch.zeros(1000, device=cuda), torch.zeros(1000, device=cuda)
    for t, gr in enumerate(grads, 1):
        opt.zero_grad()
        pr.grad = gr.clone()
        opt.step()
        ops.adam_step(pd, gr.to(cuda), m, v, 0.005, 0.9, 0.999, 1e-8, t)
    torch.cuda.synchronize()
    assert rel_err(pd, pr.detach()) < 1e-6


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,cin,cout,R", [(3, 64, 128, 8), (2, 512, 512, 4), (1, 128, 64, 16)])
@pytest.mark.parametrize("store_act", [False, True])
def test_upconv_subpixel_fwd_bwd(cuda, dtype, N, cin, cout, R, store_act):
    """Sub-pixel transposed conv (4 phase GEMMs, one launch) + fused blur/demod/noise/bias, and the
    backward (bias_act_bwd → blur adjoint → stride-2 dgrad with style sdot → demod_bwd) against
    autograd through the oracle's per-sample conv_transpose2d + upfirdn2d formulation."""
    p, wlat, x, noise, bias = _modconv_setup(21 + cin, N, cin, cout, R)
    g = torch.Generator().manual_seed(5)
    g_a = torch.randn(N, cout, 2 * R, 2 * R, generator=g)
    pd = {k: v.double() for k, v in p.items()}
    scale = 1.0 / math.sqrt(cin * 9)
    s_in = F.linear(wlat.double(), pd["m.modulation.weight"] / math.sqrt(512),
                    pd["m.modulation.bias"]).requires_grad_(True)
    xa = (F.leaky_relu(x.double(), 0.2) * math.sqrt(2)).requires_grad_(True)
    wt = scale * pd["m.weight"] * s_in.view(N, 1, cin, 1, 1)
    dm = torch.rsqrt(wt.pow(2).sum([2, 3, 4]) + 1e-8)
    wt = wt * dm.view(N, cout, 1, 1, 1)
    wt2 = wt.transpose(1, 2).reshape(N * cin, cout, 3, 3)
    o = F.conv_transpose2d(xa.reshape(1, N * cin, R, R), wt2, stride=2, groups=N)
    o = o.view(N, cout, o.shape[2], o.shape[3])
    o = stylegan2_ref.upfirdn2d(o, stylegan2_ref.make_kernel([1, 3, 3, 1], torch.float64) * 4,
                                pad=(1, 1))
    pre_ref = o + 0.1 * noise.double() + bias.double().view(1, -1, 1, 1)
    act = F.leaky_relu(pre_ref, 0.2) * math.sqrt(2)
    gx_ref, gs_ref = torch.autograd.grad((act * g_a.double()).sum(), [xa, s_in])
    # device path
    ws_ = pd["m.weight"][0] * scale
    s = s_in.detach().float().to(cuda)
    wsq = (ws_ ** 2).sum((2, 3)).float().to(cuda)
    demod = torch.empty(N, cout, device=cuda)
    ops.style_demod(s, wsq, demod)
    xd = nhwc(x, dtype).to(cuda)
    wph = [m.to(cuda) for m in layouts.upconv_subpixel_matrices(ws_, dtype)]
    t = torch.empty(N, 2 * R + 1, 2 * R + 1, cout, dtype=dtype, device=cuda)
    # store_act: the input arrives activated (SynthesisNet layout) and the output is stored as
    # a = lrelu(pre)·√2
    act_x = ops.ACT_NONE if store_act else ops.ACT_LRELU_S2
    if store_act:
        xd = nhwc(xa.detach(), dtype).to(cuda)
    ops.upconv_fwd(xd, wph, t, cout, act_in=act_x, style=s)
    nz, bz = noise.reshape(-1).to(cuda), bias.to(cuda)
    pre = torch.empty(N, 2 * R, 2 * R, cout, dtype=dtype, device=cuda)
    ops.upconv_blur_fwd(t, pre, demod, nz, 0.1, bz,
                        act_out=ops.ACT_LRELU_S2 if store_act else ops.ACT_NONE)
    q = torch.zeros(N, cout, device=cuda)
    gy = torch.empty_like(pre)
    ops.bias_act_bwd(nhwc(g_a, dtype).to(cuda), pre, nz, 0.1, bz, demod, gy, q,
                     from_act=store_act)
    gt = torch.empty_like(t)
    ops.upconv_blur_bwd(gy, gt)
    gs = torch.zeros(N, cin, device=cuda)
    gx = torch.empty(N, R, R, cin, dtype=dtype, device=cuda)
    ops.upconv_dgrad(gt, layouts.upconv_dgrad_matrix(ws_, dtype).to(cuda), gx, cin, xd,
                     act_x, s, gs)
    ops.demod_bwd(q, demod, wsq, s, gs)
    torch.cuda.synchronize()
    tol = {torch.float32: 1e-4, torch.float16: 6e-2, torch.bfloat16: 1.2e-1}[dtype]
    assert rel_err(nchw(pre), (act if store_act else pre_ref).detach()) < tol
    assert rel_err(nchw(gx), gx_ref) < tol
    assert rel_err(gs, gs_ref) < 2 * tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("kind", ["plain", "modconv", "dgrad_sdot"])
def test_conv_large_m_tiles(cuda, dtype, kind):
    """Large-M launches on the 128×128 tile, checked against torch's conv."""
    g = torch.Generator().manual_seed(17)
    N, H, Cin, Cout = 8, 128, 64, 128
    x = torch.randn(N, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    xd = nhwc(x, dtype).to(cuda)
    xq = x.to(dtype).float().to(cuda)
    wq = w.to(dtype).float().to(cuda)
    y = torch.empty(N, H, H, Cout, dtype=dtype, device=cuda)
    if kind == "plain":
        b = torch.randn(Cout, generator=g).to(cuda)
        ref = torch.relu(F.conv2d(xq, wq, b, padding=1))
        ops.conv3x3(xd, layouts.fwd_matrix(w, dtype).to(cuda), y, cout=Cout, bias=b,
                    act_out=ops.ACT_RELU)
    elif kind == "modconv":
        s = (torch.rand(N, Cin, generator=g) + 0.5).to(cuda)
        d = (torch.rand(N, Cout, generator=g) + 0.5).to(cuda)
        xa = F.leaky_relu(xq, 0.2) * math.sqrt(2) * s.view(N, Cin, 1, 1)
        ref = F.conv2d(xa, wq, padding=1) * d.view(N, Cout, 1, 1)
        ops.conv3x3(xd, layouts.fwd_matrix(w, dtype).to(cuda), y, cout=Cout,
                    act_in=ops.ACT_LRELU_S2, in_scale=s, out_scale=d)
    else:
        # input-gradient conv (Cin_g = 64 → Cout_g = 128 roles) with style sdot vs aux tensor
        aux = torch.randn(N, Cout, H, H, generator=g)
        ref = F.conv2d(xq, wq, padding=1)
        sdot_ref = (ref * (F.leaky_relu(aux.to(dtype).float(), 0.2) * math.sqrt(2)).to(cuda)).sum((2, 3))
        sd = torch.zeros(N, Cout, device=cuda)
        ops.conv3x3(xd, layouts.fwd_matrix(w, dtype).to(cuda), y, cout=Cout,
                    aux_x=nhwc(aux, dtype).to(cuda), act_aux=ops.ACT_LRELU_S2, sdot=sd)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert rel_err(nchw(y), ref) < tol
    if kind == "dgrad_sdot":
        assert rel_err(sd, sdot_ref) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("N,H,Cin,Cout,up", [(2, 16, 128, 128, False), (2, 8, 64, 128, False),
                                             (3, 12, 64, 64, False), (2, 8, 128, 64, True)])
def test_fused_backward_front_epilogue(cuda, dtype, N, H, Cin, Cout, up):
    """dgrad (3×3 stride 1, or the stride-2 up-conv adjoint) with the fused StyledConv backward
    front of the layer below (bab_*) equals dgrad → (+ ToRGB part) → mia_bias_act_bwd."""
    g = torch.Generator().manual_seed(N + H + Cin + Cout + int(up))
    # layer below: stored activation a (N,H,H,Cout_b = Cin of the dgrad output... naming: the
    # dgrad maps Cin channels (layer above's outputs) to Cout channels (layer below's outputs)
    R = H
    if up:
        gt = torch.randn(N, Cin, 2 * R + 1, 2 * R + 1, generator=g)
        w = torch.randn(Cin, Cout, 3, 3, generator=g) / math.sqrt(9 * Cin)  # W[co_up][ci_up]
        wd = layouts.upconv_dgrad_matrix(w, dtype).to(cuda)
        xin = nhwc(gt, dtype).to(cuda)
    else:
        gy = torch.randn(N, Cin, R, R, generator=g)
        w = torch.randn(Cin, Cout, 3, 3, generator=g) / math.sqrt(9 * Cout)
        wd = layouts.dgrad_matrix(w, dtype).to(cuda)
        xin = nhwc(gy, dtype).to(cuda)
    a = (torch.randn(N, Cout, R, R, generator=g) * 1.5)
    a = torch.where(a > 0, a, 0.2 * a) * math.sqrt(2)        # a valid stored activation
    ad = nhwc(a, dtype).to(cuda)
    s = (torch.rand(N, Cout, generator=g) + 0.5).to(cuda)
    demod = (torch.rand(N, Cout, generator=g) + 0.5).to(cuda)
    nz = torch.randn(R * R, generator=g).to(cuda)
    bz = (0.1 * torch.randn(Cout, generator=g)).to(cuda)
    trgb = nhwc(torch.randn(N, Cout, R, R, generator=g), dtype).to(cuda)  # ToRGB gradient part
    # reference path: dgrad → + ToRGB part → bias_act_bwd
    g_a = torch.empty(N, R, R, Cout, dtype=dtype, device=cuda)
    sd1 = torch.zeros(N, Cout, device=cuda)
    if up:
        ops.upconv_dgrad(xin, wd, g_a, Cout, ad, ops.ACT_NONE, s, sd1)
    else:
        ops.conv3x3(xin, wd, g_a, cout=Cout, out_scale=s, aux_x=ad, sdot=sd1)
    g_a = (g_a.float() + trgb.float()).to(dtype)
    gy1 = torch.empty_like(g_a)
    q1 = torch.zeros(N, Cout, device=cuda)
    ops.bias_act_bwd(g_a, ad, nz, 0.3, bz, demod, gy1, q1, from_act=True)
    # fused
    gy2 = trgb.clone()
    sd2 = torch.zeros(N, Cout, device=cuda)
    q2 = torch.zeros(N, Cout, device=cuda)
    bab = dict(demod=demod, noise=nz, noise_w=0.3, bias=bz, q=q2)
    if up:
        ops.upconv_dgrad_fused(xin, wd, gy2, Cout, ad, s, sd2, bab, accumulate=True)
    else:
        ops.conv3x3(xin, wd, gy2, cout=Cout, out_scale=s, aux_x=ad, sdot=sd2, accumulate=True,
                    bab=bab)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert rel_err(gy2, gy1) < tol
    assert rel_err(q2, q1) < (1e-4 if dtype == torch.float32 else 3e-2)
    assert rel_err(sd2, sd1) < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,W", [(2, 32, 48), (1, 17, 16), (3, 16, 64), (4, 80, 32),
                                   (9, 256, 256)])
@pytest.mark.parametrize("thin", ["1", "0"])
@pytest.mark.parametrize("e4e", [False, True])
def test_conv_thin_vgg_input_layer(cuda, tune, dtype, N, H, W, thin, e4e):
    """VGG conv1_1 forward (8-channel padded image → 64, bias, ReLU) and its input gradient
    (64 → 8 channels, 3 real) on the thin-channel kernels (conv_thin.hip; MIA_CONV_THIN=0 = the
    implicit-GEMM tiles), against torch fp64 on the same rounded operands. e4e: the encoder's
    input layer — bias + PReLU forward, gradient accumulated into an existing one (mia_conv2d).
    fp32 runs on the VALU kernels (the padded channels skipped by their zero weights); 9 × 256²
    pixels exceed one pass of their persistent grid (and, at 2-byte types, give every wave of
    the grid-strided MFMA kernels several pixel groups)."""
    tune("MIA_CONV_THIN", thin)
    if e4e:
        return _thin_e4e_input_layer(cuda, dtype, N, H, W)
    g = torch.Generator().manual_seed(N * 100 + H + W)
    x = torch.zeros(N, 8, H, W)
    x[:, :3] = torch.rand(N, 3, H, W, generator=g) * 2 - 1
    w = torch.randn(64, 3, 3, 3, generator=g) / math.sqrt(27)
    b = torch.randn(64, generator=g) * 0.1
    wp = torch.zeros(64, 8, 3, 3)
    wp[:, :3] = w
    xq, wq = x.to(dtype).double(), wp.to(dtype).double()
    ref = F.relu(F.conv2d(xq, wq, b.double(), padding=1))
    y = torch.empty(N, H, W, 64, dtype=dtype, device=cuda)
    ops.conv3x3(nhwc(x, dtype).to(cuda), layouts.fwd_matrix(w, dtype, cin_pad=8).to(cuda), y,
                cout=64, bias=b.to(cuda), act_out=ops.ACT_RELU)
    # input gradient of conv1_1: g (64 ch) → 8 channels
    gout = torch.randn(N, 64, H, W, generator=g)
    gq = gout.to(dtype).double()
    xx = torch.zeros(N, 8, H, W, dtype=torch.float64, requires_grad=True)
    (gx_ref,) = torch.autograd.grad((F.conv2d(xx, wq, padding=1) * gq).sum(), xx)
    gx = torch.empty(N, H, W, 8, dtype=dtype, device=cuda)
    ops.conv3x3(nhwc(gout, dtype).to(cuda), layouts.dgrad_matrix(w, dtype, cin_pad=8).to(cuda), gx,
                cout=8)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < 2 * TOL[dtype]
    assert rel_err(nchw(gx), gx_ref) < 2 * TOL[dtype]


@pytest.mark.parametrize("N,H,W", [(2, 32, 48), (1, 17, 16), (9, 256, 256)])
@pytest.mark.parametrize("creal", [3, 8])
def test_conv_thin_f32_vs_fp64(cuda, N, H, W, creal):
    """The fp32 VALU thin kernels (forward 8 → 64 + bias + ReLU; the 64 → 8 input gradient on
    row strips, plain and accumulating) against fp64 torch: fp32 FMAs, so ≤ 1e-5 norm-relative;
    the accumulating form equals base + the plain gradient bit for bit (one fp32 add). creal = 8:
    every padded channel real (the gradient's general path, one pixel per thread). Round 6
    replaces the bitwise comparison of the removed launch modes (MIA_THIN_F32 0–2)."""
    g = torch.Generator().manual_seed(7 * N + H + W)
    x = torch.zeros(N, 8, H, W)
    x[:, :creal] = torch.rand(N, creal, H, W, generator=g) * 2 - 1
    w = torch.randn(64, creal, 3, 3, generator=g) / math.sqrt(9 * creal)
    b = torch.randn(64, generator=g) * 0.1
    gout = torch.randn(N, 64, H, W, generator=g)
    base = torch.randn(N, H, W, 8, generator=g).to(cuda)
    xin, gin = nhwc(x, torch.float32).to(cuda), nhwc(gout, torch.float32).to(cuda)
    wf = layouts.fwd_matrix(w, torch.float32, cin_pad=8).to(cuda)
    wd = layouts.dgrad_matrix(w, torch.float32, cin_pad=8).to(cuda)
    y = torch.empty(N, H, W, 64, device=cuda)
    ops.conv3x3(xin, wf, y, cout=64, bias=b.to(cuda), act_out=ops.ACT_RELU)
    gx = torch.empty(N, H, W, 8, device=cuda)
    ops.conv3x3(gin, wd, gx, cout=8)
    ga = base.clone()
    ops.conv3x3(gin, wd, ga, cout=8, accumulate=True)
    torch.cuda.synchronize()
    wp = torch.zeros(64, 8, 3, 3, dtype=torch.float64)
    wp[:, :creal] = w.double()
    y_ref = torch.relu(F.conv2d(x.double(), wp, b.double(), padding=1))
    gx_ref = F.conv_transpose2d(gout.double(), wp, padding=1)
    assert rel_err(nchw(y), y_ref) < 1e-5
    assert rel_err(nchw(gx), gx_ref) < 1e-5
    assert torch.equal(ga, base + gx)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,cin,cout,R", [(2, 64, 64, 16), (1, 128, 192, 32), (2, 256, 128, 16),
                                          (1, 64, 64, 8), (2, 64, 32, 32), (1, 128, 96, 16)])
@pytest.mark.parametrize("lrelu_in", [False, True])
@pytest.mark.parametrize("x6", ["1", "0"])
def test_upconv_halo_fwd(cuda, tune, dtype, N, cin, cout, R, lrelu_in, x6):
    """mia_upconv_fwd_halo(_split) (halo-tiled interior + generic last row / column) against the
    transposed conv in fp64 on the same rounded operands, and against the phase-GEMM path
    (R = 8: the library falls back to it). fp32: the split-once kernel (MIA_UPCONV_X6=1, the
    default) and the on-the-fly split kernel (0)."""
    if x6 == "0" and dtype != torch.float32:
        pytest.skip("the split-once kernel exists for fp32 only")
    tune("MIA_UPCONV_X6", x6)
    g = torch.Generator().manual_seed(N + cin + cout + R)
    x = torch.randn(N, cin, R, R, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    s = torch.rand(N, cin, generator=g) + 0.5
    xq = x.to(dtype).double()
    xin = F.leaky_relu(xq, 0.2) * math.sqrt(2) if lrelu_in else xq
    sq = (s * (math.sqrt(2) if lrelu_in else 1.0)).to(dtype).double() / (
        math.sqrt(2) if lrelu_in else 1.0)
    xm = (xin * sq.view(N, cin, 1, 1))
    wq = w.to(dtype).double()
    ref = F.conv_transpose2d(xm, wq.transpose(0, 1), stride=2)  # (N, cout, 2R+1, 2R+1)
    xd = nhwc(x, dtype).to(cuda)
    wph = [m.to(cuda) for m in layouts.upconv_subpixel_matrices(w, dtype)]
    wup = layouts.upconv_halo_matrix(w, dtype).to(cuda)
    act = ops.ACT_LRELU_S2 if lrelu_in else ops.ACT_NONE
    t1 = torch.full((N, 2 * R + 1, 2 * R + 1, cout), float("nan"), dtype=dtype, device=cuda)
    t2 = torch.empty_like(t1)
    ops.upconv_fwd(xd, wph, t1, cout, act_in=act, style=s.to(cuda), w_up=wup)
    ops.upconv_fwd(xd, wph, t2, cout, act_in=act, style=s.to(cuda))
    torch.cuda.synchronize()
    assert not torch.isnan(t1).any(), "halo path left T positions unwritten"
    assert rel_err(nchw(t1), ref) < 3 * TOL[dtype]
    assert rel_err(t1.float(), t2.float()) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("C", [64, 128])
@pytest.mark.parametrize("mode", ["bias", "acc", "bias_acc"])
def test_generic_tile_register_epilogues_stride2(cuda, tune, dtype, C, mode):
    """The generic tile's specialised register epilogues for the e4e stride-2 body convs / 1×1
    shortcuts (folded BN: bias) and the FPN laterals (accumulate, bias + accumulate): 64-column
    tile at C = 64, 128-column (fp32: X6B split-once B) at C = 128, against fp64 torch, and against
    the LDS-staged generic epilogue (MIA_CONV_REGEPI=0) of the same tile."""
    g = torch.Generator().manual_seed(C + len(mode) + (7 if dtype == torch.float16 else 0))
    N, H = 2, 32
    ho = H // 2
    x = torch.randn(N, C, H, H, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    b = torch.randn(C, generator=g) * 0.1
    y0 = torch.randn(N, C, ho, ho, generator=g)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    kp = ops.conv2d_kpad(9, C, dtype)
    wm = torch.zeros(C, kp)
    wm[:, :9 * C] = w.permute(0, 2, 3, 1).reshape(C, 9 * C)
    grp = [dict(w=wm.to(dtype).to(cuda), kh=3, kw=3, pad=(1, 1), ho=ho, wo=ho)]
    ref = F.conv2d(xq, wq, stride=2, padding=1)
    kw = {}
    if "bias" in mode:
        ref = ref + b.double().view(1, C, 1, 1)
        kw["bias"] = b.to(cuda)
    if "acc" in mode:
        ref = ref + y0.to(dtype).double()
        kw["accumulate"] = True

    def run():
        y = nhwc(y0, dtype).to(cuda)
        ops.conv2d(nhwc(x, dtype).to(cuda), grp, y, (ho, ho), cout=C, stride=2, **kw)
        torch.cuda.synchronize()
        return nchw(y)
    y_reg = run()
    tune("MIA_CONV_REGEPI", 0)
    y_lds = run()
    tol = 2e-5 if dtype == torch.float32 else 2 * TOL[dtype]
    assert rel_err(y_reg, ref) < tol
    assert rel_err(y_lds, ref) < tol
    assert rel_err(y_reg, y_lds.double()) < tol


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,W,C", [(2, 192, 192, 64), (1, 16, 16, 64), (3, 16, 48, 64),
                                     (2, 32, 16, 128)])
@pytest.mark.parametrize("mode", ["plain", "bias_relu", "tap_mask", "prelu", "bias_csum",
                                  "mask_slope", "acc", "bias"])
@pytest.mark.parametrize("spec", ["1", "0"])
def test_conv2d_register_epilogue_paths(cuda, tune, dtype, N, H, W, C, mode, spec):
    """Stride-1 C→C 3×3 convs with every epilogue feature set of the attack step (vgg.py, e4e
    IR-SE50 body). spec=1: the specialised register epilogues — at C = 64 the weights-resident
    persistent kernel (conv_wres.hip, 8 waves × 32 channels; 192² = 288 patches > one per CU
    exercises the persistent run and the halo prefetch), at C = 128 the halo kernel; spec=0:
    generic tile at 64 (MIA_CONV_WRES=0) and the runtime-feature halo epilogue at 128
    (MIA_HALO_EPI=2)."""
    tune("MIA_CONV_WRES", spec)
    tune("MIA_HALO_EPI", "2" if spec == "0" else "1")
    g = torch.Generator().manual_seed(N * 11 + H + W + C + len(mode))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    kp = ops.conv2d_kpad(9, C, dtype)
    wm = torch.zeros(C, kp)
    wm[:, :9 * C] = w.permute(0, 2, 3, 1).reshape(C, 9 * C)
    grp = [dict(w=wm.to(dtype).to(cuda), kh=3, kw=3, pad=(1, 1), ho=H, wo=W)]
    conv = F.conv2d(xq, wq, padding=1)
    y0 = torch.randn(N, C, H, W, generator=g)
    y = nhwc(y0, dtype).to(cuda)
    slope = torch.rand(C, generator=g) * 0.5 + 0.05
    sl = slope.double().view(1, C, 1, 1)
    kw, cs = {}, None
    if mode == "plain":
        ref = conv
    elif mode == "bias_relu":
        b = torch.randn(C, generator=g) * 0.1
        ref = F.relu(conv + b.double().view(1, C, 1, 1))
        kw = dict(bias=b.to(cuda), act_out=ops.ACT_RELU)
    elif mode == "tap_mask":
        a = torch.randn(N, C, H, W, generator=g).relu()
        t = torch.randn(N, C, H, W, generator=g)
        aq, tq = a.to(dtype).double(), t.to(dtype).double()
        ref = (conv + 0.37 * (aq - tq)) * (aq > 0)
        y3 = torch.empty_like(y)
        ops.conv3x3(nhwc(x, dtype).to(cuda), layouts.fwd_matrix(w, dtype).to(cuda), y3, cout=C,
                    tap_a=nhwc(a, dtype).to(cuda), tap_t=nhwc(t, dtype).to(cuda), tap_coef=0.37,
                    mask_a=nhwc(a, dtype).to(cuda))
    elif mode == "prelu":
        ref = torch.where(conv > 0, conv, sl * conv)
        kw = dict(act_out=ops.ACT_PRELU, act_slope=slope.to(cuda))
    elif mode == "bias_csum":
        b = torch.randn(C, generator=g) * 0.1
        ref = conv + b.double().view(1, C, 1, 1)
        cs = torch.zeros(N, C, device=cuda)
        kw = dict(bias=b.to(cuda), csum=cs)
    elif mode == "bias":  # e4e conv2 (the SE body; its pool sums in a separate pass)
        b = torch.randn(C, generator=g) * 0.1
        ref = conv + b.double().view(1, C, 1, 1)
        kw = dict(bias=b.to(cuda))
    elif mode == "mask_slope":
        m = torch.randn(N, C, H, W, generator=g)
        ref = torch.where(m.to(dtype).double() > 0, conv, sl * conv)
        kw = dict(mask_a=nhwc(m, dtype).to(cuda), mask_slope=slope.to(cuda))
    else:
        ref = conv + y0.to(dtype).double()
        kw = dict(accumulate=True)
    if mode == "tap_mask":
        y = y3
    else:
        ops.conv2d(nhwc(x, dtype).to(cuda), grp, y, (H, W), cout=C, **kw)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < 2 * TOL[dtype]
    if cs is not None:
        assert rel_err(cs, ref.sum((2, 3))) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,C,k,stride", [(4, 2, 512, 3, 2), (3, 8, 512, 3, 2), (2, 16, 256, 3, 2),
                                            (5, 4, 512, 1, 1), (2, 8, 128, 3, 1),
                                            (3, 4, 128, 1, 1)])
@pytest.mark.parametrize("mode", ["bias_prelu", "mask_slope_acc"])
def test_conv2d_style_head_shapes(cuda, dtype, N, H, C, k, stride, mode):
    """Generic-tile launches of the e4e style heads (stride-2 3×3, 8²…1² outputs, K up to 9·512,
    a few tiles per launch) and short-K 1×1 layers, with the head epilogues (bias + PReLU) and
    the backward ones (slope mask + accumulate), against torch fp64."""
    g = torch.Generator().manual_seed(N * 13 + H + C + k + stride)
    pad = k // 2
    ho = (H + 2 * pad - k) // stride + 1
    x = torch.randn(N, C, H, H, generator=g)
    w = torch.randn(C, C, k, k, generator=g) / math.sqrt(k * k * C)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    kp = ops.conv2d_kpad(k * k, C, dtype)
    wm = torch.zeros(C, kp)
    wm[:, :k * k * C] = w.permute(0, 2, 3, 1).reshape(C, k * k * C)
    grp = [dict(w=wm.to(dtype).to(cuda), kh=k, kw=k, pad=(pad, pad), ho=ho, wo=ho)]
    conv = F.conv2d(xq, wq, stride=stride, padding=pad)
    slope = torch.rand(C, generator=g) * 0.5 + 0.05
    sl = slope.double().view(1, C, 1, 1)
    y0 = torch.randn(N, C, ho, ho, generator=g)
    if mode == "bias_prelu":
        b = torch.randn(C, generator=g) * 0.1
        pre = conv + b.double().view(1, C, 1, 1)
        ref = torch.where(pre > 0, pre, sl * pre)
        kw = dict(bias=b.to(cuda), act_out=ops.ACT_PRELU, act_slope=slope.to(cuda))
    else:
        m = torch.randn(N, C, ho, ho, generator=g)
        ref = torch.where(m.to(dtype).double() > 0, conv, sl * conv) + y0.to(dtype).double()
        kw = dict(mask_a=nhwc(m, dtype).to(cuda), mask_slope=slope.to(cuda), accumulate=True)
    y = nhwc(y0, dtype).to(cuda)
    ops.conv2d(nhwc(x, dtype).to(cuda), grp, y, (ho, ho), cout=C, stride=stride, **kw)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < 2 * TOL[dtype]


def _thin_e4e_input_layer(cuda, dtype, N, H, W):
    g = torch.Generator().manual_seed(N * 101 + H + W)
    x = torch.zeros(N, 8, H, W)
    x[:, :3] = torch.rand(N, 3, H, W, generator=g) * 2 - 1
    wp = torch.zeros(64, 8, 3, 3)
    wp[:, :3] = torch.randn(64, 3, 3, 3, generator=g) / math.sqrt(27)
    b = torch.randn(64, generator=g) * 0.1
    slope = torch.rand(64, generator=g) * 0.5 + 0.05
    xq, wq = x.to(dtype).double(), wp.to(dtype).double()
    pre = F.conv2d(xq, wq, b.double(), padding=1)
    ref = torch.where(pre > 0, pre, slope.double().view(1, 64, 1, 1) * pre)
    kp = ops.conv2d_kpad(9, 8, dtype)
    wm = torch.zeros(64, kp)
    wm[:, :72] = wp.permute(0, 2, 3, 1).reshape(64, 72)
    y = torch.empty(N, H, W, 64, dtype=dtype, device=cuda)
    ops.conv2d(nhwc(x, dtype).to(cuda), [dict(w=wm.to(dtype).to(cuda), kh=3, kw=3, pad=(1, 1),
                                              ho=H, wo=W)], y, (H, W), cout=64, bias=b.to(cuda),
               act_out=ops.ACT_PRELU, act_slope=slope.to(cuda))
    # input gradient: g (64 ch) → 8 channels, accumulated onto gx0
    gout = torch.randn(N, 64, H, W, generator=g)
    gx0 = torch.randn(N, 8, H, W, generator=g)
    gq = gout.to(dtype).double()
    xx = torch.zeros(N, 8, H, W, dtype=torch.float64, requires_grad=True)
    (gx_ref,) = torch.autograd.grad((F.conv2d(xx, wq, padding=1) * gq).sum(), xx)
    gx_ref = gx_ref + gx0.to(dtype).double()
    wd = wp.flip(2, 3).transpose(0, 1)  # (8, 64, 3, 3): the flipped, transposed kernel
    kd = ops.conv2d_kpad(9, 64, dtype)
    wdm = torch.zeros(8, kd)
    wdm[:, :576] = wd.permute(0, 2, 3, 1).reshape(8, 576)
    gx = nhwc(gx0, dtype).to(cuda)
    ops.conv2d(nhwc(gout, dtype).to(cuda), [dict(w=wdm.to(dtype).to(cuda), kh=3, kw=3, pad=(1, 1),
                                                 ho=H, wo=W)], gx, (H, W), cout=8,
               accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < 2 * TOL[dtype]
    assert rel_err(nchw(gx), gx_ref) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,W", [(2, 32, 48), (3, 16, 16), (4, 256, 256)])
@pytest.mark.parametrize("mode", ["modconv", "dgrad_sdot", "plain", "acc"])
@pytest.mark.parametrize("path", ["wres32", "thin32", "generic"])
def test_conv_thin32_layers(cuda, tune, dtype, N, H, W, mode, path):
    """32 → 32-channel layers (StyleGAN2 1024² StyledConvs) on the LDS-halo weights-resident
    kernel (conv_wres.hip conv_wres32_kernel, the default), the global-gather kernel
    (conv_thin.hip conv_thin32_kernel: MIA_CONV_WRES32=0) and the implicit-GEMM tile (both 0):
    modulated forward with demod / noise / bias / lrelu·√2, the input gradient with the
    style-gradient sdot (4 × 256² exercises long persistent runs across images), plain and
    accumulating, against torch fp64."""
    tune("MIA_CONV_WRES32", path == "wres32")
    tune("MIA_CONV_THIN32", path != "generic")
    C = 32
    g = torch.Generator().manual_seed(N * 31 + H + W + len(mode))
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    xd = nhwc(x, dtype).to(cuda)
    wf = layouts.fwd_matrix(w, dtype).to(cuda)
    y0 = torch.randn(N, C, H, W, generator=g)
    y = nhwc(y0, dtype).to(cuda)
    sd = sd_ref = None
    if mode == "modconv":
        s = torch.rand(N, C, generator=g) + 0.5
        d = torch.rand(N, C, generator=g) + 0.5
        nz = torch.randn(H * W, generator=g)
        b = torch.randn(C, generator=g) * 0.1
        pre = F.conv2d(xq * s.to(dtype).double().view(N, C, 1, 1), wq, padding=1) * d.double().view(
            N, C, 1, 1) + 0.3 * nz.double().view(1, 1, H, W) + b.double().view(1, -1, 1, 1)
        ref = F.leaky_relu(pre, 0.2) * math.sqrt(2)
        ops.conv3x3(xd, wf, y, cout=C, in_scale=s.to(cuda), out_scale=d.to(cuda),
                    noise=nz.to(cuda), noise_w=0.3, bias=b.to(cuda), act_out=ops.ACT_LRELU_S2)
    elif mode == "dgrad_sdot":
        s = torch.rand(N, C, generator=g) + 0.5
        aux = torch.randn(N, C, H, W, generator=g)
        conv = F.conv2d(xq, wq, padding=1)
        ref = conv * s.double().view(N, C, 1, 1)
        sd_ref = (conv * aux.to(dtype).double()).sum((2, 3))
        sd = torch.zeros(N, C, device=cuda)
        ops.conv3x3(xd, wf, y, cout=C, out_scale=s.to(cuda), aux_x=nhwc(aux, dtype).to(cuda),
                    sdot=sd)
    elif mode == "plain":
        ref = F.conv2d(xq, wq, padding=1)
        ops.conv3x3(xd, wf, y, cout=C)
    else:
        ref = F.conv2d(xq, wq, padding=1) + y0.to(dtype).double()
        ops.conv3x3(xd, wf, y, cout=C, accumulate=True)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < 2 * TOL[dtype]
    if sd is not None:
        assert rel_err(sd, sd_ref) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("H,W", [(40, 48), (256, 256)])
def test_conv_thin32_sums_batch_independent(cuda, tune, dtype, H, W):
    """conv_thin32_kernel (MIA_CONV_WRES32=0): the sdot sums of an image come from work items of
    a fixed number of 16-pixel groups of that image (slot = chunk index), so they are
    bit-identical whether the image is attacked alone or in a batch of 5, and run to run
    (the per-wave partition used to depend on N and the grid)."""
    tune("MIA_CONV_WRES32", 0)
    C, N = 32, 5
    g = torch.Generator().manual_seed(H + W)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    s = torch.rand(N, C, generator=g) + 0.5
    aux = torch.randn(N, C, H, W, generator=g)
    wf = layouts.fwd_matrix(w, dtype).to(cuda)

    def run(lo, hi):
        n = hi - lo
        y = torch.empty(n, H, W, C, dtype=dtype, device=cuda)
        sd = torch.zeros(n, C, device=cuda)
        ops.conv3x3(nhwc(x[lo:hi], dtype).to(cuda), wf, y, cout=C, out_scale=s[lo:hi].to(cuda),
                    aux_x=nhwc(aux[lo:hi], dtype).to(cuda), sdot=sd)
        torch.cuda.synchronize()
        return y, sd

    y_all, sd_all = run(0, N)
    y2, sd2 = run(0, N)
    assert torch.equal(sd_all, sd2) and torch.equal(y_all, y2)
    for i in (0, 3, N - 1):
        y1, sd1 = run(i, i + 1)
        assert torch.equal(sd1, sd_all[i:i + 1]), i
        assert torch.equal(y1, y_all[i:i + 1]), i


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,W", [(2, 32, 48), (3, 16, 16), (5, 64, 32)])
@pytest.mark.parametrize("mode", ["mod", "mod_lrelu_in", "sdot", "sdot_acc", "sdot_bab",
                                  "sdot_acc_bab", "plain", "acc"])
def test_conv_wres32_matches_thin32(cuda, tune, dtype, N, H, W, mode):
    """The LDS-halo 32-channel kernel (conv_wres32_kernel) against the global-gather one
    (conv_thin32_kernel): same weights in VGPRs, same modulate<T> rounding of act(x)·s (once per
    halo in LDS vs per fragment read), the same 9 MFMAs per fragment in tap order and the same
    epilogue source, so the outputs agree to the epilogue's last rounding; the sdot / q sums are
    the same terms in a different order (per-patch LDS pre-reduction + ordered slots vs per-wave
    runs): ≤ 1e-5 relative. 5 × 64×32 puts patch runs across image boundaries; plus the 'mod'
    forward against fp64 on the same rounded operands."""
    g = torch.Generator().manual_seed(N * 7 + H + W + len(mode) + (dtype == torch.bfloat16))
    C = 32
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    y0 = torch.randn(N, C, H, W, generator=g)
    b = torch.randn(C, generator=g) * 0.1
    a = torch.randn(N, C, H, W, generator=g)
    s = torch.rand(N, C, generator=g) + 0.5
    d = torch.rand(N, C, generator=g) + 0.5
    noise = torch.randn(H * W, generator=g)
    red = mode.startswith("sdot")

    def run():
        y = nhwc(y0, dtype).to(cuda)
        sd = torch.zeros(N * C, device=cuda) if red else None
        q = torch.zeros(N * C, device=cuda) if "bab" in mode else None
        kw = {}
        if mode.startswith("mod"):
            kw = dict(in_scale=s.to(cuda), out_scale=d.to(cuda), noise=noise.to(cuda),
                      noise_w=0.3, bias=b.to(cuda), act_out=ops.ACT_LRELU_S2)
            if mode == "mod_lrelu_in":
                kw["act_in"] = ops.ACT_LRELU_S2
        elif red:
            kw = dict(out_scale=s.to(cuda), aux_x=nhwc(a, dtype).to(cuda), sdot=sd,
                      accumulate="acc" in mode)
            if q is not None:
                kw["bab"] = dict(demod=d.to(cuda), noise=noise.to(cuda), noise_w=0.3,
                                 bias=b.to(cuda), q=q)
        elif mode == "acc":
            kw = dict(accumulate=True)
        ops.conv3x3(nhwc(x, dtype).to(cuda), layouts.fwd_matrix(w, dtype).to(cuda), y, cout=C,
                    **kw)
        torch.cuda.synchronize()
        return y.clone(), sd, q

    tune("MIA_CONV_WRES32", 1)
    y_w, sd_w, q_w = run()
    tune("MIA_CONV_WRES32", 0)
    y_t, sd_t, q_t = run()
    # the compiler may contract the last fp32 multiply / add of an epilogue chain differently in
    # the two kernels' schedules (fp16: fused into the conversion, v_fma_mix*; one rounding
    # instead of two) for a few elements: ≤ 1 ulp of T there (measured ≤ 10 of 10⁵ elements;
    # most modes bit-identical)
    ulp = torch.finfo(dtype).eps * y_t.float().abs().clamp_min(2.0 ** -14)
    dd = (y_w.float() - y_t.float()).abs()
    assert (dd <= ulp).all(), (mode, dd.max().item())
    assert (dd > 0).float().mean().item() < 1e-3, mode
    for u, v in ((sd_w, sd_t), (q_w, q_t)):
        if u is not None:
            assert ((u - v).abs().max() / v.abs().max()).item() < 1e-5
    if mode == "mod":
        xm = (x.to(dtype).double() * s.to(dtype).double().view(N, C, 1, 1)).to(dtype).double()
        pre = F.conv2d(xm, w.to(dtype).double(), padding=1) * d.double().view(N, C, 1, 1) \
            + 0.3 * noise.double().view(1, 1, H, W) + b.double().view(1, C, 1, 1)
        ref = torch.where(pre > 0, pre, 0.2 * pre) * math.sqrt(2)
        got = y_w.permute(0, 3, 1, 2).double().cpu()
        tol = 2e-2 if dtype == torch.float16 else 1e-1
        assert ((got - ref).abs().max() / ref.abs().max()).item() < tol


@pytest.mark.parametrize("off,nbytes", [(0, 4096), (0, 4100), (4, 64), (1, 33), (16, 1 << 20),
                                        (3, 7), (0, 16)])
@pytest.mark.parametrize("value", [0, 0xA5])
def test_memset_fill_kernel(cuda, off, nbytes, value):
    """mia_memset (the library's own fill kernel, 16-/4-/1-byte paths by alignment) writes exactly
    [off, off + nbytes) and nothing around it."""
    buf = torch.full((nbytes + 64,), 0x3C, dtype=torch.uint8, device=cuda)
    _lib.call("mia_memset", buf.data_ptr() + off, value, nbytes, ops.stream())
    got = buf.cpu()
    want = torch.full((nbytes + 64,), 0x3C, dtype=torch.uint8)
    want[off:off + nbytes] = value
    assert torch.equal(got, want)


@pytest.mark.parametrize("path", ["halo", "halo_otf", "generic", "upconv"])
def test_fp32_arithmetic_is_fp32_accurate(cuda, tune, path):
    """The fp32 convs run as exact three-way bf16 splits with six products (conv_common.h,
    mfma_chunk<float>; the dropped mid·lo, lo·mid, lo·lo terms are < 2^-23·|ab|). At the largest
    K of the attack (9·512 = 4608) the error against fp64 is set by the fp32 accumulation, as for
    the native v_mfma_f32_16x16x4_f32 build (MIA_F32_ARITH=native, measured on these seeded
    operands: max-abs 1.12e-5 / 1.22e-5 / 5.2e-6, norm-relative 1.18e-6 / 1.19e-6 / 6.6e-7 for
    halo / generic / upconv; the split build: 1.18e-5 / 9.1e-6 / 5.6e-6 and 1.05e-6 / 1.05e-6 /
    5.8e-7). Bound: 2× the native figures. "halo" = the split-once kernel (conv_halo_x6.hip,
    pre-split weights), "halo_otf" = the on-the-fly split halo kernel (MIA_CONV_X6=0)."""
    tune("MIA_CONV_HALO", "0" if path == "generic" else "1")
    tune("MIA_CONV_X6", "0" if path == "halo_otf" else "1")
    g = torch.Generator().manual_seed(77)
    N, H, Cin, Cout = 2, 16, 512, 256
    x = torch.randn(N, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)
    if path == "upconv":  # the sub-pixel up-sampling conv (transposed, stride 2) on the halo kernel
        ref = F.conv_transpose2d(x.double(), w.double().transpose(0, 1), stride=2)
        t = torch.empty(N, 2 * H + 1, 2 * H + 1, Cout, device=cuda)
        ops.upconv_fwd(nhwc(x, torch.float32).to(cuda),
                       [m.to(cuda) for m in layouts.upconv_subpixel_matrices(w, torch.float32)],
                       t, cout=Cout, w_up=layouts.upconv_halo_matrix(w, torch.float32).to(cuda))
        got = t.permute(0, 3, 1, 2).double().cpu()
    else:
        ref = F.conv2d(x.double(), w.double(), padding=1)
        y = torch.empty(N, H, H, Cout, device=cuda)
        ops.conv3x3(nhwc(x, torch.float32).to(cuda), layouts.fwd_matrix(w, torch.float32).to(cuda),
                    y, cout=Cout)
        got = nchw(y).cpu()
    torch.cuda.synchronize()
    err = (got - ref).abs()
    native = {"halo": (1.12e-5, 1.18e-6), "generic": (1.22e-5, 1.19e-6), "upconv": (5.2e-6, 6.6e-7)}
    native["halo_otf"] = native["halo"]
    mx, nrm = err.max().item(), (err.norm() / ref.norm()).item()
    print(f"{path}: max-abs err {mx:.3e}, norm-relative {nrm:.3e} (native fp32 MFMA "
          f"{native[path][0]:.2e}, {native[path][1]:.2e})")
    assert mx <= 2 * native[path][0] and nrm <= 2 * native[path][1]


@pytest.mark.parametrize("C,H,W", [(64, 32, 48), (64, 16, 32), (128, 32, 16), (256, 16, 16)])
@pytest.mark.parametrize("mode", ["plain", "bias_relu", "prelu", "mask_slope", "acc", "mask",
                                  "tap_mask", "bias"])
def test_x6_halo_variants_bitwise(cuda, tune, C, H, W, mode):
    """fp32 split-once halo kernel (conv_halo_x6.hip): the default launch (specialised register
    epilogue, taps unrolled over lane-constant fragment offsets, weight rows past Cout clamped)
    computes the same products in the same order as the rolled loop with the runtime-feature
    epilogue (MIA_X6_UNR=0, MIA_HALO_EPI=2): outputs bit-identical, for every epilogue feature
    set of the attack's fp32 launches, on the 64- and 128-channel tiles; and both against fp64.
    The 64-channel layers' default two-blocks-per-CU tile (MIA_X6_64S=1), the 8-wave tile's
    two-taps-per-K-step loop (MIA_X6_UNR=2) and its one-tap form (MIA_X6_UNR=1) agree bit for
    bit."""
    g = torch.Generator().manual_seed(C + H * 3 + W + len(mode))
    N = 2
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    kp = ops.conv2d_kpad(9, C, torch.float32)
    wm = torch.zeros(C, kp)
    wm[:, :9 * C] = w.permute(0, 2, 3, 1).reshape(C, 9 * C)
    grp = [dict(w=wm.to(cuda), kh=3, kw=3, pad=(1, 1), ho=H, wo=W)]
    conv = F.conv2d(x.double(), w.double(), padding=1)
    y0 = torch.randn(N, C, H, W, generator=g)
    slope = torch.rand(C, generator=g) * 0.5 + 0.05
    sl = slope.double().view(1, C, 1, 1)
    b = torch.randn(C, generator=g) * 0.1
    m = torch.randn(N, C, H, W, generator=g)
    a = torch.randn(N, C, H, W, generator=g).relu()
    t = torch.randn(N, C, H, W, generator=g)
    kw, ref = {}, conv
    if mode == "bias_relu":
        ref = F.relu(conv + b.double().view(1, C, 1, 1))
        kw = dict(bias=b.to(cuda), act_out=ops.ACT_RELU)
    elif mode == "bias":
        ref = conv + b.double().view(1, C, 1, 1)
        kw = dict(bias=b.to(cuda))
    elif mode == "prelu":
        ref = torch.where(conv > 0, conv, sl * conv)
        kw = dict(act_out=ops.ACT_PRELU, act_slope=slope.to(cuda))
    elif mode == "mask_slope":
        ref = torch.where(m.double() > 0, conv, sl * conv)
        kw = dict(mask_a=nhwc(m, torch.float32).to(cuda), mask_slope=slope.to(cuda))
    elif mode == "mask":
        ref = conv * (m.double() > 0)
        kw = dict(mask_a=nhwc(m, torch.float32).to(cuda))
    elif mode == "acc":
        ref = conv + y0.double()
        kw = dict(accumulate=True)

    def run():
        y = nhwc(y0, torch.float32).to(cuda)
        xc = nhwc(x, torch.float32).to(cuda)
        if mode == "tap_mask":
            ops.conv3x3(xc, layouts.fwd_matrix(w, torch.float32).to(cuda), y, cout=C,
                        tap_a=nhwc(a, torch.float32).to(cuda),
                        tap_t=nhwc(t, torch.float32).to(cuda), tap_coef=0.37,
                        mask_a=nhwc(a, torch.float32).to(cuda))
        else:
            ops.conv2d(xc, grp, y, (H, W), cout=C, **kw)
        torch.cuda.synchronize()
        return y

    if mode == "tap_mask":
        ref = (conv + 0.37 * (a.double() - t.double())) * (a.double() > 0)
    y_def = run()  # Cout 64: the two-blocks-per-CU tile (MIA_X6_64S=1)
    tune("MIA_X6_64S", "0")  # the 8-wave 64-column tile, two taps per K-step (MIA_X6_UNR=2)
    assert torch.equal(run(), y_def)
    tune("MIA_X6_UNR", "1")  # one tap per K-step: the same MFMAs in the same order
    assert torch.equal(run(), y_def)
    tune("MIA_X6_UNR", "0")
    tune("MIA_HALO_EPI", "2")
    y_gen = run()
    assert torch.equal(y_def, y_gen)
    assert rel_err(nchw(y_def), ref) < 2 * TOL[torch.float32]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("C,H,W", [(128, 32, 16), (256, 16, 32), (64, 32, 32)])
@pytest.mark.parametrize("mode", ["plain", "bias_relu", "mask", "tap", "mod", "sdot_bab"])
def test_halo_lowp_unrolled_bitwise(cuda, tune, dtype, C, H, W, mode):
    """fp16 / bf16 halo kernel (conv_halo.hip): the specialised-epilogue launches run the taps
    unrolled over lane-constant fragment offsets; the runtime-feature epilogue (MIA_HALO_EPI=2)
    runs the rolled loop. Same reads, same MFMAs in the same order: outputs (and sdot / q sums)
    bit-identical; both within the dtype's tolerance of fp64. 'mod' = the StyledConv forward
    (modulated input, halo modulated once in LDS; demod, noise, bias, LeakyReLU·√2)."""
    g = torch.Generator().manual_seed(C + H + W + len(mode) + (dtype == torch.bfloat16))
    if C == 64:  # the 64-channel halo tile for every 64-channel launch (default: bf16 forward)
        tune("MIA_HALO_C64", 1)
    N = 2
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    wq = w.to(dtype).double()
    y0 = torch.randn(N, C, H, W, generator=g)
    b = torch.randn(C, generator=g) * 0.1
    m = torch.randn(N, C, H, W, generator=g)
    a = torch.randn(N, C, H, W, generator=g).relu()
    t = torch.randn(N, C, H, W, generator=g)
    s = torch.rand(N, C, generator=g) + 0.5
    d = torch.rand(N, C, generator=g) + 0.5
    noise = torch.randn(H * W, generator=g)
    xq = x.to(dtype).double()
    f32 = torch.float32

    def run():
        y = nhwc(y0, dtype).to(cuda)
        xc = nhwc(x, dtype).to(cuda)
        sd = torch.zeros(N * C, device=cuda) if mode == "sdot_bab" else None
        q = torch.zeros(N * C, device=cuda) if mode == "sdot_bab" else None
        kw = {}
        if mode == "bias_relu":
            kw = dict(bias=b.to(cuda), act_out=ops.ACT_RELU)
        elif mode == "mask":
            kw = dict(mask_a=nhwc(m, dtype).to(cuda))
        elif mode == "tap":
            kw = dict(tap_a=nhwc(a, dtype).to(cuda), tap_t=nhwc(t, dtype).to(cuda), tap_coef=0.37)
        elif mode == "mod":
            kw = dict(in_scale=s.to(cuda), act_in=ops.ACT_LRELU_S2, out_scale=d.to(cuda),
                      noise=noise.to(cuda), noise_w=0.3, bias=b.to(cuda),
                      act_out=ops.ACT_LRELU_S2)
        elif mode == "sdot_bab":
            kw = dict(out_scale=s.to(cuda), aux_x=nhwc(a, dtype).to(cuda), sdot=sd,
                      bab=dict(demod=d.to(cuda), noise=noise.to(cuda), noise_w=0.3,
                               bias=b.to(cuda), q=q))
        ops.conv3x3(xc, layouts.fwd_matrix(w, dtype).to(cuda), y, cout=C, **kw)
        torch.cuda.synchronize()
        return y.clone(), sd, q

    y_def, sd_def, q_def = run()
    tune("MIA_HALO_EPI", "2")
    y_rol, sd_rol, q_rol = run()
    if mode != "sdot_bab":
        assert torch.equal(y_def, y_rol), (mode, (y_def.float() - y_rol.float()).abs().max().item())
    else:
        # the main loop is the same code for every EPI ≥ 0 (bit-identity shown by the other
        # modes); the runtime-feature epilogue's backward front rounds its fp32 chain differently
        # from the specialised one in rare elements: ≤ 1 ulp of T on the outputs
        ulp = torch.finfo(dtype).eps * y_rol.float().abs().clamp_min(1e-3)
        assert ((y_def.float() - y_rol.float()).abs() <= ulp).all()
        for u, v in ((sd_def, sd_rol), (q_def, q_rol)):
            assert ((u - v).abs().max() / v.abs().max()).item() < 1e-5
    # against fp64 on the same rounded operands
    if mode == "mod":
        xa = torch.where(xq > 0, xq, 0.2 * xq) * math.sqrt(2)
        xm = (xa * s.double().view(N, C, 1, 1)).to(dtype).double()
        pre = F.conv2d(xm, wq, padding=1) * d.double().view(N, C, 1, 1) \
            + 0.3 * noise.double().view(1, 1, H, W) + b.double().view(1, C, 1, 1)
        ref = torch.where(pre > 0, pre, 0.2 * pre) * math.sqrt(2)
    else:
        conv = F.conv2d(xq, wq, padding=1)
        ref = {"plain": conv, "bias_relu": F.relu(conv + b.double().view(1, C, 1, 1)),
               "mask": conv * (m.to(dtype).double() > 0),
               "tap": conv + 0.37 * (a.to(dtype).double() - t.to(dtype).double()),
               "sdot_bab": None}[mode]
    if ref is not None:
        got = y_def.permute(0, 3, 1, 2).double().cpu()
        tol = 2e-2 if dtype == torch.float16 else 1e-1
        assert ((got - ref).abs().max() / ref.abs().max()).item() < tol, mode


@pytest.mark.parametrize("R,cin,cout", [(16, 64, 128), (32, 128, 64)])
def test_upconv_x6_two_block_form_bitwise(cuda, tune, R, cin, cout):
    """fp32 split-once up-conv kernels: the 8 × 16-patch two-blocks-per-CU form (MIA_UPCONV_X6S=1,
    default for the stride-2 input gradients with Cin ≤ 512) computes the same MFMAs in the same
    order as the 8-wave 16 × 16 form (0): the stride-2 input gradient with mask + accumulate
    (2-source multi form) is bit-identical; the up-sampling conv forward (modulated, lrelu input)
    too, and against fp64."""
    N = 2
    g = torch.Generator().manual_seed(R + cin + cout)
    x = torch.randn(N, cin, R, R, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    s = torch.rand(N, cin, generator=g) + 0.5
    xd = nhwc(x, torch.float32).to(cuda)
    wph = [m.to(cuda) for m in layouts.upconv_subpixel_matrices(w, torch.float32)]
    wup = layouts.upconv_halo_matrix(w, torch.float32).to(cuda)
    # s2 dgrad: two sources of Cg = cout channels each (the multi-source K loop), into cin channels
    wd = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    gs = [nhwc(torch.randn(N, cout, R, R, generator=g), torch.float32).to(cuda) for _ in range(2)]
    wh = torch.cat([layouts.s2_dgrad_halo_matrix(wd, torch.float32)] * 2).to(cuda)
    a_below = nhwc(torch.randn(N, cin, 2 * R, 2 * R, generator=g), torch.float32).to(cuda)
    base = nhwc(torch.randn(N, cin, 2 * R, 2 * R, generator=g), torch.float32).to(cuda)
    sl = torch.full((cin,), 0.25, device=cuda)

    def run():
        t = torch.full((N, 2 * R + 1, 2 * R + 1, cout), float("nan"), device=cuda)
        ops.upconv_fwd(xd, wph, t, cout, act_in=ops.ACT_LRELU_S2, style=s.to(cuda), w_up=wup)
        gx = base.clone()
        ops.s2_dgrad_halo(gs, wh, gx, mask_a=a_below, mask_slope=sl, accumulate=True)
        torch.cuda.synchronize()
        return t, gx

    t1, g1 = run()  # the dgrad (Cin = 2·cout ≤ 512) on the two-block form, the forward 8-wave
    tune("MIA_UPCONV_X6S", "0")
    t0, g0 = run()
    assert torch.equal(t1, t0) and torch.equal(g1, g0)
    xin = F.leaky_relu(x.double(), 0.2) * math.sqrt(2) * s.double().view(N, cin, 1, 1)
    ref = F.conv_transpose2d(xin, w.double().transpose(0, 1), stride=2)
    assert rel_err(nchw(t1), ref) < 3 * TOL[torch.float32]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,R,W", [(6, 128, 128), (3, 40, 48), (1, 8, 16)])
@pytest.mark.parametrize("mode", ["bias_relu", "mask", "prelu", "bias", "mask_slope", "acc"])
def test_wres128_shared_weight_epilogues(cuda, tune, dtype, N, R, W, mode):
    """The weights-resident 128-channel kernel on the shared-weight launches: VGG conv2_2
    forward (bias + ReLU) and input gradient (ReLU mask); the e4e IR-SE body at 128 channels,
    conv1 (PReLU), conv2 (bias), the conv2 input gradient (PReLU' mask with slope) and the conv1
    input gradient accumulated onto the identity shortcut's; against torch fp64 and against the
    halo tile (MIA_CONV_WRES128=0; both accumulate in fp32, in different orders)."""
    C = 128
    g = torch.Generator().manual_seed(N * 7 + R + W + len(mode))
    x = torch.randn(N, C, R, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    wf = layouts.fwd_matrix(w, dtype).to(cuda)
    grp = [dict(w=wf, kh=3, kw=3, pad=(1, 1), ho=R, wo=W)]
    conv = F.conv2d(xq, wq, padding=1)
    slope = torch.rand(C, generator=g) * 0.5 + 0.05
    sl = slope.double().view(1, C, 1, 1)
    y0 = torch.randn(N, C, R, W, generator=g)
    b = torch.randn(C, generator=g) * 0.1
    m = torch.randn(N, C, R, W, generator=g)
    if mode == "bias_relu":
        ref = F.relu(conv + b.double().view(1, C, 1, 1))
        kw = dict(bias=b.to(cuda), act_out=ops.ACT_RELU)
    elif mode == "mask":
        ref = conv * (m.to(dtype).double() > 0)
        kw = dict(mask_a=nhwc(m, dtype).to(cuda))
    elif mode == "prelu":
        ref = torch.where(conv > 0, conv, sl * conv)
        kw = dict(act_out=ops.ACT_PRELU, act_slope=slope.to(cuda))
    elif mode == "bias":
        ref = conv + b.double().view(1, C, 1, 1)
        kw = dict(bias=b.to(cuda))
    elif mode == "mask_slope":
        ref = torch.where(m.to(dtype).double() > 0, conv, sl * conv)
        kw = dict(mask_a=nhwc(m, dtype).to(cuda), mask_slope=slope.to(cuda))
    else:
        ref = conv + y0.to(dtype).double()
        kw = dict(accumulate=True)
    xd = nhwc(x, dtype).to(cuda)
    y = nhwc(y0, dtype).to(cuda)
    ops.conv2d(xd, grp, y, (R, W), cout=C, **kw)
    tune("MIA_CONV_WRES128", 0)
    y_halo = nhwc(y0, dtype).to(cuda)
    if R % 16 == 0:
        ops.conv2d(xd, grp, y_halo, (R, W), cout=C, **kw)
    torch.cuda.synchronize()
    e = rel_err(nchw(y), ref)
    print(f"wres128 shared-weight {mode} {dtype} {N}x{R}x{W}: rel err vs fp64 {e:.2e}")
    assert e < 2 * TOL[dtype]
    if R % 16 == 0:
        assert rel_err(nchw(y), nchw(y_halo).double()) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,R,W", [(4, 128, 128), (2, 24, 32), (1, 8, 16)])
@pytest.mark.parametrize("mode", ["bias_relu", "prelu"])
def test_wres128_cin64_forward(cuda, tune, dtype, N, R, W, mode):
    """The weights-resident kernel with Cin = 64 (two 32-channel sub-planes, two 4-pixel groups
    per DMA piece) on the 64 → 128 forward launches (VGG conv2_1 bias + ReLU, the e4e stage-2
    conv1 PReLU): against torch fp64 and the halo tile (MIA_CONV_WRES128=0)."""
    cin, C = 64, 128
    g = torch.Generator().manual_seed(N * 13 + R + W + len(mode))
    x = torch.randn(N, cin, R, W, generator=g)
    w = torch.randn(C, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    wf = layouts.fwd_matrix(w, dtype).to(cuda)
    grp = [dict(w=wf, kh=3, kw=3, pad=(1, 1), ho=R, wo=W)]
    conv = F.conv2d(xq, wq, padding=1)
    if mode == "bias_relu":
        b = torch.randn(C, generator=g) * 0.1
        ref = F.relu(conv + b.double().view(1, C, 1, 1))
        kw = dict(bias=b.to(cuda), act_out=ops.ACT_RELU)
    else:
        slope = torch.rand(C, generator=g) * 0.5 + 0.05
        ref = torch.where(conv > 0, conv, slope.double().view(1, C, 1, 1) * conv)
        kw = dict(act_out=ops.ACT_PRELU, act_slope=slope.to(cuda))
    xd = nhwc(x, dtype).to(cuda)
    y = torch.full((N, R, W, C), float("nan"), dtype=dtype, device=cuda)
    ops.conv2d(xd, grp, y, (R, W), cout=C, **kw)
    tune("MIA_CONV_WRES128", 0)
    y_halo = torch.full_like(y, float("nan"))
    if R % 16 == 0:
        ops.conv2d(xd, grp, y_halo, (R, W), cout=C, **kw)
    torch.cuda.synchronize()
    e = rel_err(nchw(y), ref)
    print(f"wres128 Cin 64 {mode} {dtype} {N}x{R}x{W}: rel err vs fp64 {e:.2e}")
    assert e < 2 * TOL[dtype]
    if R % 16 == 0:
        assert rel_err(nchw(y), nchw(y_halo).double()) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,R,W", [(4, 128, 128), (2, 24, 32), (1, 8, 16)])
@pytest.mark.parametrize("mode", ["plain", "acc", "mask_slope"])
def test_wres128_cout64(cuda, tune, dtype, N, R, W, mode):
    """The weights-resident kernel with Cout = 64 (8 waves = 2 row groups × 4 channel groups of
    16) on the 128 → 64 input gradients (VGG conv2_1, the e4e stage-2 conv1: plain, accumulated,
    PReLU'-masked): against torch fp64 and the halo tile (MIA_CONV_WRES128=0)."""
    cin, C = 128, 64
    g = torch.Generator().manual_seed(N * 17 + R + W + len(mode))
    x = torch.randn(N, cin, R, W, generator=g)
    w = torch.randn(C, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    wf = layouts.fwd_matrix(w, dtype).to(cuda)
    grp = [dict(w=wf, kh=3, kw=3, pad=(1, 1), ho=R, wo=W)]
    conv = F.conv2d(xq, wq, padding=1)
    y0 = torch.randn(N, C, R, W, generator=g)
    if mode == "plain":
        ref, kw = conv, {}
    elif mode == "acc":
        ref, kw = conv + y0.to(dtype).double(), dict(accumulate=True)
    else:
        m = torch.randn(N, C, R, W, generator=g)
        slope = torch.rand(C, generator=g) * 0.5 + 0.05
        ref = torch.where(m.to(dtype).double() > 0, conv, slope.double().view(1, C, 1, 1) * conv)
        kw = dict(mask_a=nhwc(m, dtype).to(cuda), mask_slope=slope.to(cuda))
    xd = nhwc(x, dtype).to(cuda)
    y = nhwc(y0, dtype).to(cuda)
    ops.conv2d(xd, grp, y, (R, W), cout=C, **kw)
    tune("MIA_CONV_WRES128", 0)
    y_halo = nhwc(y0, dtype).to(cuda)
    if R % 16 == 0:
        ops.conv2d(xd, grp, y_halo, (R, W), cout=C, **kw)
    torch.cuda.synchronize()
    e = rel_err(nchw(y), ref)
    print(f"wres128 Cout 64 {mode} {dtype} {N}x{R}x{W}: rel err vs fp64 {e:.2e}")
    assert e < 2 * TOL[dtype]
    if R % 16 == 0:
        assert rel_err(nchw(y), nchw(y_halo).double()) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("cin,N,R,W", [(128, 3, 64, 64), (64, 2, 32, 48), (128, 1, 8, 16)])
@pytest.mark.parametrize("mode", ["bias_relu", "prelu"])
def test_wres128_cout256_column_tiles(cuda, tune, dtype, cin, N, R, W, mode):
    """The weights-resident kernel over two 128-channel column tiles (Cout = 256: VGG conv3_1
    forward, the e4e stage-3 conv1): against torch fp64 and the halo tile (MIA_CONV_WRES128=0)."""
    C = 256
    g = torch.Generator().manual_seed(N * 19 + R + W + cin + len(mode))
    x = torch.randn(N, cin, R, W, generator=g)
    w = torch.randn(C, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    xq, wq = x.to(dtype).double(), w.to(dtype).double()
    wf = layouts.fwd_matrix(w, dtype).to(cuda)
    grp = [dict(w=wf, kh=3, kw=3, pad=(1, 1), ho=R, wo=W)]
    conv = F.conv2d(xq, wq, padding=1)
    if mode == "bias_relu":
        b = torch.randn(C, generator=g) * 0.1
        ref = F.relu(conv + b.double().view(1, C, 1, 1))
        kw = dict(bias=b.to(cuda), act_out=ops.ACT_RELU)
    else:
        slope = torch.rand(C, generator=g) * 0.5 + 0.05
        ref = torch.where(conv > 0, conv, slope.double().view(1, C, 1, 1) * conv)
        kw = dict(act_out=ops.ACT_PRELU, act_slope=slope.to(cuda))
    xd = nhwc(x, dtype).to(cuda)
    y = torch.full((N, R, W, C), float("nan"), dtype=dtype, device=cuda)
    ops.conv2d(xd, grp, y, (R, W), cout=C, **kw)
    tune("MIA_CONV_WRES128", 0)
    y_halo = torch.full_like(y, float("nan"))
    if R % 16 == 0:
        ops.conv2d(xd, grp, y_halo, (R, W), cout=C, **kw)
    torch.cuda.synchronize()
    e = rel_err(nchw(y), ref)
    print(f"wres128 Cout 256 (Cin {cin}) {mode} {dtype} {N}x{R}x{W}: rel err vs fp64 {e:.2e}")
    assert e < 2 * TOL[dtype]
    if R % 16 == 0:
        assert rel_err(nchw(y), nchw(y_halo).double()) < 2 * TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_survey_named_aliases(cuda, dtype):
    """The SURVEY.md §8(b) names (round 6): mia_vgg_conv_relu_dgrad equals mia_vgg_conv_dgrad bit
    for bit and both match fp64 torch (conv_transpose + tap-MSE term + ReLU mask of the layer
    below); mia_mse_fwd_bwd equals mia_mse_sum + mia_mse_grad_f32 / mia_tap_grad bit for bit."""
    g = torch.Generator().manual_seed(61)
    N, H, W, cin, cout = 2, 16, 32, 64, 128
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    gy = torch.randn(N, cout, H, W, generator=g)
    tap_a = torch.relu(torch.randn(N, cin, H, W, generator=g))  # the layer below's post-ReLU
    tap_t = torch.randn(N, cin, H, W, generator=g)
    coef = 0.37
    wd = layouts.dgrad_matrix(w, dtype).to(cuda)
    kpad = wd.shape[1]
    gin, ta, tt = (nhwc(t, dtype).to(cuda) for t in (gy, tap_a, tap_t))
    outs = []
    for name in ("mia_vgg_conv_dgrad", "mia_vgg_conv_relu_dgrad"):
        gx = torch.empty(N, H, W, cin, dtype=dtype, device=cuda)
        ops.call(name, ops.ptr(gin), ops.ptr(wd), ops.ptr(gx), N, H, W, cout, cin, kpad,
                 ops.ptr(ta), ops.ptr(tt), coef, ops.ptr(ta), ops.dt(dtype), ops.stream())
        outs.append(gx)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    rd = lambda t: t.to(dtype).double()  # noqa: E731  (the operands as the device holds them)
    ref = F.conv_transpose2d(rd(gy), rd(w), padding=1) + coef * (rd(tap_a) - rd(tap_t))
    ref = ref * (rd(tap_a) > 0)
    assert rel_err(nchw(outs[1]), ref) < (2e-5 if dtype == torch.float32 else 2e-2)

    n, L = 3, 5000
    a = torch.randn(n, L, generator=g).to(dtype).to(cuda)
    b = torch.randn(n, L, generator=g).to(dtype).to(cuda)
    base = torch.randn(n, L, generator=g).to(dtype).to(cuda)
    l1 = torch.full((n,), 0.5, device=cuda)
    l2 = l1.clone()
    g1, g2 = base.clone(), base.clone()
    acc = int(dtype == torch.float32)
    ops.call("mia_mse_fwd_bwd", ops.ptr(a), ops.ptr(b), ops.ptr(l1), ops.ptr(g1), n, L,
             1.0 / L, 2.0 / L, acc, ops.dt(dtype), ops.stream())
    ops.call("mia_mse_sum", ops.ptr(a), ops.ptr(b), ops.ptr(l2), n, L, 1.0 / L, ops.dt(dtype),
             ops.stream())
    if dtype == torch.float32:
        ops.call("mia_mse_grad_f32", ops.ptr(a), ops.ptr(b), ops.ptr(g2), n * L, 2.0 / L, 1,
                 ops.stream())
    else:
        ops.call("mia_tap_grad", ops.ptr(a), ops.ptr(b), ops.ptr(g2), n * L, 2.0 / L, 0,
                 ops.dt(dtype), ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(g1, g2)
    ref_l = 0.5 + ((a.double() - b.double()) ** 2).mean(dim=1)
    assert torch.allclose(l1.double(), ref_l, rtol=1e-5)
    if dtype != torch.float32:  # a 2-byte gradient cannot accumulate (fp32 only)
        with pytest.raises(_lib.MiaError, match="fp32 only"):
            ops.call("mia_mse_fwd_bwd", ops.ptr(a), ops.ptr(b), ops.ptr(l1), ops.ptr(g1), n, L,
                     1.0 / L, 2.0 / L, 1, ops.dt(dtype), ops.stream())


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,R,C", [(2, 16, 128), (1, 24, 64), (2, 32, 512), (1, 40, 256),
                                   (2, 8, 128), (1, 16, 32)])
def test_upconv_blur_fwd_bwd_vs_fp64(cuda, dtype, N, R, C):
    """mia_upconv_blur_fwd / _bwd (the up-sampling StyledConv's Blur, rosinality upfirdn2d with
    [1,3,3,1]⊗[1,3,3,1]/64·4, pad (1,1), + demod + noise + bias + lrelu·√2; and its adjoint)
    against fp64 on the device's own (rounded) inputs, at strip-ragged sizes (2R not a multiple
    of the 8-row strips at R = 24 / 40; the 2R + 1 adjoint rows / columns) and C = 32 … 512."""
    g = torch.Generator().manual_seed(R * 7 + C)
    S = 2 * R + 1
    t = torch.randn(N, S, S, C, generator=g).to(dtype)
    demod = (0.5 + torch.rand(N, C, generator=g))
    noise = torch.randn(2 * R, 2 * R, generator=g)
    bias = 0.1 * torch.randn(C, generator=g)
    gy = torch.randn(N, 2 * R, 2 * R, C, generator=g).to(dtype)
    k = stylegan2_ref.make_kernel([1, 3, 3, 1], torch.float64) * 4
    blur = stylegan2_ref.upfirdn2d(t.permute(0, 3, 1, 2).double(), k, pad=(1, 1))
    pre = blur * demod.double().view(N, C, 1, 1) + 0.1 * noise.double() + bias.double().view(1, -1, 1, 1)
    ref = F.leaky_relu(pre, 0.2) * math.sqrt(2)
    # the adjoint: autograd of the same linear map
    tt = t.permute(0, 3, 1, 2).double().requires_grad_(True)
    (gt_ref,) = torch.autograd.grad(stylegan2_ref.upfirdn2d(tt, k, pad=(1, 1)),
                                    tt, gy.permute(0, 3, 1, 2).double())
    out = torch.empty(N, 2 * R, 2 * R, C, dtype=dtype, device=cuda)
    ops.upconv_blur_fwd(t.to(cuda), out, demod.to(cuda), noise.reshape(-1).to(cuda), 0.1,
                        bias.to(cuda), act_out=ops.ACT_LRELU_S2)
    gt = torch.empty(N, S, S, C, dtype=dtype, device=cuda)
    ops.upconv_blur_bwd(gy.to(cuda), gt)
    torch.cuda.synchronize()
    tol = {torch.float32: 2e-6, torch.float16: 2e-3, torch.bfloat16: 1.5e-2}[dtype]
    assert rel_err(nchw(out), ref) < tol
    assert rel_err(nchw(gt), gt_ref) < tol
