"""fp32 split arithmetic, per conv kernel class of the headline path (shared by
``__graft_entry__.smoke()`` and ``tests/test_gpu_kernels.py``; not a test module).

The fp32 convs run as exact three-way bf16 splits with six products on the bf16 matrix pipe
(DESIGN.md §3). Each check below runs ONE kernel class on seeded unit-scale operands at a shape the
bench launches it with, and compares with fp64 torch. Bound, per class: the norm-relative error
≤ 2.4e-6 — 2× the native fp32 MFMA build's at the attack's largest K (9·512:
test_fp32_arithmetic_is_fp32_accurate measured 1.18e-6) — and max|Δ| ≤ 1e-5·max|ref| (the native
build: 1.12e-5 max-abs on outputs of max ≈ 4.5, i.e. 2.5e-6 relative; 4× that). torch's CPU
fp32 error on the same operands is printed beside it as a native-fp32 point of comparison.
"""
import math

import torch
import torch.nn.functional as F

NRM_BOUND, MAX_BOUND = 2.4e-6, 1e-5


def _rnd(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g, dtype=torch.float64) * scale


def _nhwc(t, dev):
    return t.permute(0, 2, 3, 1).contiguous().float().to(dev)


def _nchw(t):
    return t.permute(0, 3, 1, 2).double().cpu()


def _err(got, ref):
    d = (got.double() - ref).abs()
    return (d.norm() / ref.norm()).item(), (d.max() / ref.abs().max()).item()


def _halo(dev, N, H, cin, cout, seed):
    from gfa_amd import layouts, ops
    x = _rnd((N, cin, H, H), seed)
    w = _rnd((cout, cin, 3, 3), seed + 1, 1 / math.sqrt(9 * cin))
    y = torch.empty(N, H, H, cout, device=dev)
    ops.conv3x3(_nhwc(x, dev), layouts.fwd_matrix(w, torch.float32).to(dev), y, cout=cout)
    ref = F.conv2d(x, w, padding=1)
    return _nchw(y), ref, F.conv2d(x.float(), w.float(), padding=1)


def _stride2(dev, N, H, cin, cout, seed):
    from gfa_amd import layouts, ops
    x = _rnd((N, cin, H, H), seed)
    w = _rnd((cout, cin, 3, 3), seed + 1, 1 / math.sqrt(9 * cin))
    ho = (H - 1) // 2 + 1
    y = torch.empty(N, ho, ho, cout, device=dev)
    ops.conv2d(_nhwc(x, dev), [dict(w=layouts.fwd_matrix(w, torch.float32).to(dev), kh=3, kw=3,
                                    pad=(1, 1), ho=ho, wo=ho)], y, (ho, ho), cout=cout, stride=2)
    return (_nchw(y), F.conv2d(x, w, stride=2, padding=1),
            F.conv2d(x.float(), w.float(), stride=2, padding=1))


def _upconv(dev, N, R, cin, cout, seed):
    from gfa_amd import layouts, ops
    x = _rnd((N, cin, R, R), seed)
    w = _rnd((cout, cin, 3, 3), seed + 1, 1 / math.sqrt(9 * cin))
    t = torch.empty(N, 2 * R + 1, 2 * R + 1, cout, device=dev)
    ops.upconv_fwd(_nhwc(x, dev),
                   [m.to(dev) for m in layouts.upconv_subpixel_matrices(w, torch.float32)], t,
                   cout=cout, w_up=layouts.upconv_halo_matrix(w, torch.float32).to(dev))
    wt = w.transpose(0, 1)
    return (_nchw(t), F.conv_transpose2d(x, wt, stride=2),
            F.conv_transpose2d(x.float(), wt.float(), stride=2))


def _s2_dgrad_multi(dev, N, R, ng, cg, cx, seed):
    from gfa_amd import layouts, ops
    ws = [_rnd((cg, cx, 3, 3), seed + i, 1 / math.sqrt(9 * cx)) for i in range(ng)]
    gs = [_rnd((N, cg, R, R), seed + 50 + i) for i in range(ng)]
    gx = torch.empty(N, 2 * R, 2 * R, cx, device=dev)
    ops.s2_dgrad_halo([_nhwc(g, dev) for g in gs],
                      torch.cat([layouts.s2_dgrad_halo_matrix(w, torch.float32)
                                 for w in ws]).to(dev), gx)

    def adj(dtype):
        xx = torch.zeros(N, cx, 2 * R, 2 * R, dtype=dtype, requires_grad=True)
        loss = sum((F.conv2d(xx, w.to(dtype), stride=2, padding=1) * g.to(dtype)).sum()
                   for w, g in zip(ws, gs))
        return torch.autograd.grad(loss, xx)[0].detach()
    return _nchw(gx), adj(torch.float64), adj(torch.float32)


def _batched(dev, N, H, S, C, seed):
    from gfa_amd import ops
    ho = (H - 1) // 2 + 1
    ws = [_rnd((C, C, 3, 3), seed + i, 1 / math.sqrt(9 * C)) for i in range(S)]
    xs = _rnd((S * N, C, H, H), seed + 100)
    groups = []
    for k in range(S):
        kp = ops.conv2d_kpad(9, C, torch.float32)
        wm = torch.zeros(C, kp, dtype=torch.float64)
        wm[:, :9 * C] = ws[k].permute(0, 2, 3, 1).reshape(C, 9 * C)
        groups.append(dict(w=wm.float().to(dev), kh=3, kw=3, pad=(1, 1), ho=ho, wo=ho,
                           n_in=k * N, n_out=k * N, c_off=k * C))
    y = torch.empty(S * N, ho, ho, C, device=dev)
    ops.conv2d_batched(_nhwc(xs, dev), groups, y, (ho, ho), n=N, cout=C, stride=2)
    ref = torch.cat([F.conv2d(xs[k * N:(k + 1) * N], ws[k], stride=2, padding=1)
                     for k in range(S)])
    cpu = torch.cat([F.conv2d(xs[k * N:(k + 1) * N].float(), ws[k].float(), stride=2, padding=1)
                     for k in range(S)])
    return _nchw(y), ref, cpu


# (name, builder, args): the classes of the fp32 headline path at bench shapes (K up to 9·512)
CASES = [
    ("x6 halo 128-ch tile (StyledConv 32² 512→512)", _halo, (1, 32, 512, 512, 11)),
    ("x6 halo 128-ch tile (VGG conv2_2 128→128)", _halo, (2, 64, 128, 128, 13)),
    ("x6 halo 64-ch tile (VGG conv1_2 64→64)", _halo, (2, 64, 64, 64, 15)),
    ("X6B generic tile (e4e stride-2 512→512)", _stride2, (2, 16, 512, 512, 17)),
    ("upconv_x6 forward (StyleGAN2 up-conv 512→256)", _upconv, (1, 32, 512, 256, 19)),
    ("upconv_x6 DG multi-source (3 heads, 512→512)", _s2_dgrad_multi, (1, 16, 3, 512, 512, 21)),
    ("batched heads (4 stride-2 convs 512→512)", _batched, (2, 8, 4, 512, 23)),
]


def run(dev, verbose=True):
    """Run every class; returns [(name, nrm, maxrel, cpu_nrm, cpu_maxrel)] and raises
    AssertionError naming the first class over the bound."""
    out = []
    for name, fn, args in CASES:
        got, ref, cpu = fn(dev, *args)
        torch.cuda.synchronize()
        nrm, mx = _err(got, ref)
        cn, cm = _err(cpu, ref)
        out.append((name, nrm, mx, cn, cm))
        if verbose:
            print(f"  fp32 split {name}: norm-rel {nrm:.2e} max-rel {mx:.2e} "
                  f"(torch CPU fp32 {cn:.2e} / {cm:.2e})", flush=True)
    for name, nrm, mx, _, _ in out:
        assert nrm <= NRM_BOUND and mx <= MAX_BOUND, (name, nrm, mx)
    return out
