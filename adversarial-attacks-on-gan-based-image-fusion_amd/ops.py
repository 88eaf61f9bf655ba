"""Typed host wrappers over the C ABI: torch tensors in, device pointers + the current HIP stream
out. Every wrapper validates shapes/dtypes/contiguity on the host before a kernel is launched, so a
malformed call raises here instead of faulting on the GPU."""
import ctypes

import torch

from . import _lib, layouts
from ._lib import ACT_LRELU_S2, ACT_NONE, ACT_PRELU, ACT_RELU, ConvArgs, call  # noqa: F401

DTYPES = {torch.float32: _lib.MIA_F32, torch.float16: _lib.MIA_F16, torch.bfloat16: _lib.MIA_BF16}
VEC = {torch.float32: 4, torch.float16: 8, torch.bfloat16: 8}


def dt(t_or_dtype):
    d = t_or_dtype if isinstance(t_or_dtype, torch.dtype) else t_or_dtype.dtype
    if d not in DTYPES:
        raise TypeError(f"unsupported dtype {d}")
    return DTYPES[d]


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("device tensor required (the attack path runs on the GPU only)")
    if not t.is_contiguous():
        raise ValueError("contiguous tensor required")
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _need(t, shape, dtype=None, name="tensor"):
    if t is None:
        raise ValueError(f"{name} is required")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(shape)}")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype} != {dtype}")


def _numel_ok(t, n, dtype=None, name="tensor"):
    if t is None:
        return
    if t.numel() != n:
        raise ValueError(f"{name}: numel {t.numel()} != {n}")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype} != {dtype}")


def conv_kpad(cin, dtype):
    bk = 32 if dtype == torch.float32 else 64
    return (9 * cin + bk - 1) // bk * bk


# Live per-launch timing of the conv kernel (bench.py roofline): when PROFILE is a list, every
# conv3x3 call is bracketed by HIP events on the launch stream and (start, end, algorithmic
# FLOPs) is appended. None (default) = no events.
PROFILE = None
# Tuning aid (tools/layer_table.py): when a list, one label per PROFILE entry (API + shape).
PROFILE_TAGS = None


def _tag(label):
    if PROFILE_TAGS is not None:
        PROFILE_TAGS.append(label)


def conv3x3(x, w, y, *, cout, act_in=ACT_NONE, in_scale=None, out_scale=None, bias=None,
            noise=None, noise_w=0.0, act_out=ACT_NONE, shuffle_out=False, aux_x=None,
            act_aux=ACT_NONE, sdot=None, tap_a=None, tap_t=None, tap_coef=0.0, mask_a=None,
            accumulate=False, y_cstride=0, bab=None, flops=None):
    """Generic MFMA implicit-GEMM conv (mia_conv3x3). x: (N,H,W,Cin); w: (Cout,Kpad).
    ``bab``: dict(demod, noise, noise_w, bias, q) — fused StyledConv backward front of the layer
    whose stored activation is aux_x (mia_conv_args.bab_*).
    ``flops``: algorithmic FLOPs of this launch for profiling (default 2·N·H·W·9·Cin·Cout)."""
    N, H, W, Cin = x.shape
    T = x.dtype
    kpad = conv_kpad(Cin, T)
    _need(w, (cout, kpad), T, "w")
    if Cin % VEC[T]:
        raise ValueError("Cin must be a multiple of the 16-byte vector")
    cm = cout // 4 if shuffle_out else cout
    ys = y_cstride or cm
    if y is not None:
        if shuffle_out:
            _need(y, (N, 2 * H, 2 * W, ys), T, "y")
        else:
            _need(y, (N, H, W, ys), T, "y")
    f32 = torch.float32
    _numel_ok(in_scale, N * Cin, f32, "in_scale")
    _numel_ok(out_scale, N * cm, f32, "out_scale")
    _numel_ok(bias, cm, f32, "bias")
    Ho, Wo = (2 * H, 2 * W) if shuffle_out else (H, W)
    _numel_ok(noise, Ho * Wo, f32, "noise")
    for name, a in (("aux_x", aux_x), ("tap_a", tap_a), ("tap_t", tap_t), ("mask_a", mask_a)):
        if a is not None:
            _need(a, (N, H, W, cout), T, name)
    _numel_ok(sdot, N * cout, f32, "sdot")
    if bab is not None:
        _numel_ok(bab["demod"], N * cout, f32, "bab.demod")
        _numel_ok(bab["q"], N * cout, f32, "bab.q")
        _numel_ok(bab.get("noise"), H * W, f32, "bab.noise")
        _numel_ok(bab.get("bias"), cout, f32, "bab.bias")
        if aux_x is None:
            raise ValueError("bab needs aux_x (the stored activation)")
    a = ConvArgs()
    a.x, a.w, a.y = ptr(x), ptr(w), ptr(y)
    a.N, a.H, a.W, a.Cin, a.Cout, a.Kpad = N, H, W, Cin, cout, kpad
    a.y_cstride = ys
    a.act_in = act_in
    a.in_scale, a.out_scale, a.bias, a.noise = ptr(in_scale), ptr(out_scale), ptr(bias), ptr(noise)
    a.noise_w = float(noise_w)
    a.act_out = act_out
    a.shuffle_out = int(bool(shuffle_out))
    a.aux_x, a.act_aux, a.sdot = ptr(aux_x), act_aux, ptr(sdot)
    a.tap_a, a.tap_t, a.tap_coef, a.mask_a = ptr(tap_a), ptr(tap_t), float(tap_coef), ptr(mask_a)
    a.accumulate = int(bool(accumulate))
    ws = layouts.split_for(w) if T == torch.float32 and not shuffle_out else None
    a.w_split = ptr(ws)
    if bab is not None:
        a.bab_demod, a.bab_q = ptr(bab["demod"]), ptr(bab["q"])
        a.bab_noise, a.bab_noise_w = ptr(bab.get("noise")), float(bab.get("noise_w", 0.0))
        a.bab_bias = ptr(bab.get("bias"))
    prof = PROFILE
    if prof is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    call("mia_conv3x3", ctypes.byref(a), dt(T), stream())
    if prof is not None:
        e1.record()
        prof.append((e0, e1, flops if flops is not None else 2 * N * H * W * 9 * Cin * cout))
        _tag(f"conv3x3 {H}x{W} {Cin}->{cout}" + (" mod" if in_scale is not None else "")
             + (" bab" if bab is not None else "") + (" sdot" if sdot is not None else "")
             + (" tap" if tap_a is not None else "") + (" shuf" if shuffle_out else ""))
    return y


def conv3x3_modw(x, w, y, w_mod, *, cout, in_scale, out_scale=None, bias=None, noise=None,
                 noise_w=0.0, act_out=ACT_NONE, flops=None):
    """The StyledConv forward on per-image weights (fp16 / bf16): mia_modulate_weights writes
    w_mod[n] = w·in_scale[n]·out_scale[n] (the modulation and demodulation folded into the
    weights), then mia_conv3x3_wmod convolves the unmodulated x. Same result as
    conv3x3(x, w, y, in_scale=…, out_scale=…) up to where the one rounding to T happens.
    Profiled as ONE conv call (the weight pass included)."""
    N, H, W, Cin = x.shape
    T = x.dtype
    if T not in (torch.float16, torch.bfloat16):
        raise ValueError("per-image weights: fp16 / bf16 only")
    kpad = conv_kpad(Cin, T)
    _need(w, (cout, kpad), T, "w")
    _need(w_mod, (N, cout, kpad), T, "w_mod")
    _need(y, (N, H, W, cout), T, "y")
    f32 = torch.float32
    _numel_ok(in_scale, N * Cin, f32, "in_scale")
    _numel_ok(out_scale, N * cout, f32, "out_scale")
    _numel_ok(bias, cout, f32, "bias")
    _numel_ok(noise, H * W, f32, "noise")
    if in_scale is None:
        raise ValueError("in_scale (the style) is required")
    a = ConvArgs()
    a.x, a.w, a.y = ptr(x), ptr(w_mod), ptr(y)
    a.N, a.H, a.W, a.Cin, a.Cout, a.Kpad = N, H, W, Cin, cout, kpad
    a.y_cstride = cout
    a.act_in = ACT_NONE
    a.bias, a.noise = ptr(bias), ptr(noise)
    a.noise_w = float(noise_w)
    a.act_out = act_out
    prof = PROFILE
    if prof is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    call("mia_modulate_weights", ptr(w), ptr(in_scale), ptr(out_scale), ptr(w_mod), N, cout, Cin,
         kpad, dt(T), stream())
    call("mia_conv3x3_wmod", ctypes.byref(a), cout * kpad, dt(T), stream())
    if prof is not None:
        e1.record()
        prof.append((e0, e1, flops if flops is not None else 2 * N * H * W * 9 * Cin * cout))
        _tag(f"conv3x3 {H}x{W} {Cin}->{cout} mod wmod")
    return y


def _prof_call(name, flops, *args):
    prof = PROFILE
    if prof is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    call(name, *args)
    if prof is not None:
        e1.record()
        prof.append((e0, e1, flops))
        _tag(f"{name} " + (f"R{args[6]} x{args[1]}" if name == "mia_conv_s2_dgrad_halo_multi"
                             else f"{args[5:8]}" if name.endswith("_split")
                             else f"{args[4:7]}"))


def upconv_kpad(cin, phase, dtype):
    kh, kw = 2 - (phase >> 1), 2 - (phase & 1)
    bk = 32 if dtype == torch.float32 else 64
    return (kh * kw * cin + bk - 1) // bk * bk


def upconv_fwd(x, w_phases, t_out, cout, act_in=ACT_NONE, style=None, flops=None, w_up=None):
    """conv_transpose2d(stride 2) as 4 sub-pixel phase GEMMs (one launch). x: (N,R,R,Cin) →
    T: (N, 2R+1, 2R+1, Cout). ``w_up`` (layouts.upconv_halo_matrix): the halo-tiled kernel
    (mia_upconv_fwd_halo; the library falls back to the phase GEMMs where it does not apply)."""
    N, R, R2, Cin = x.shape
    T = x.dtype
    if R != R2:
        raise ValueError("square inputs only")
    if len(w_phases) != 4:
        raise ValueError("4 phase weight matrices required")
    for ph, w in enumerate(w_phases):
        _need(w, (cout, upconv_kpad(Cin, ph, T)), T, f"w_phase[{ph}]")
    _need(t_out, (N, 2 * R + 1, 2 * R + 1, cout), T, "t_out")
    _numel_ok(style, N * Cin, torch.float32, "style")
    wp = (ctypes.c_void_p * 4)(*[w.data_ptr() for w in w_phases])
    for w in w_phases:
        ptr(w)
    fl = flops if flops is not None else 2 * N * R * R * 9 * Cin * cout
    if w_up is not None:
        bk = layouts.halo_bk(T)
        _need(w_up, (Cin // bk, 5, 2, cout, bk), T, "w_up")
        ws = layouts.split_for(w_up) if T == torch.float32 else None
        _prof_call("mia_upconv_fwd_halo_split", fl, ptr(x), wp, ptr(w_up), ptr(ws), ptr(t_out), N,
                   R, Cin, cout, act_in, ptr(style), dt(T), stream())
        return t_out
    _prof_call("mia_upconv_fwd", fl, ptr(x), wp, ptr(t_out), N, R, Cin, cout, act_in, ptr(style),
               dt(T), stream())
    return t_out


def upconv_blur_fwd(t, pre, demod, noise, noise_w, bias, act_out=ACT_NONE):
    N, TS, _, C = t.shape
    R = (TS - 1) // 2
    _need(pre, (N, 2 * R, 2 * R, C), t.dtype, "pre")
    _numel_ok(demod, N * C, torch.float32, "demod")
    _numel_ok(noise, 4 * R * R, torch.float32, "noise")
    _numel_ok(bias, C, torch.float32, "bias")
    call("mia_upconv_blur_fwd", ptr(t), ptr(pre), ptr(demod), ptr(noise), float(noise_w),
         ptr(bias), N, R, C, int(act_out), dt(t), stream())
    return pre


def upconv_blur_bwd(gy, gt):
    N, S, _, C = gy.shape
    R = S // 2
    _need(gt, (N, 2 * R + 1, 2 * R + 1, C), gy.dtype, "gt")
    call("mia_upconv_blur_bwd", ptr(gy), ptr(gt), N, R, C, dt(gy), stream())
    return gt


def upconv_dgrad(g_t, w_t, gx, cin, x_fwd, act_x, style, sdot, flops=None):
    N, TS, _, Cout = g_t.shape
    R = (TS - 1) // 2
    T = g_t.dtype
    _need(w_t, (cin, conv_kpad(Cout, T)), T, "w_t")
    if gx is not None:
        _need(gx, (N, R, R, cin), T, "gx")
    _need(x_fwd, (N, R, R, cin), T, "x_fwd")
    _numel_ok(style, N * cin, torch.float32, "style")
    _numel_ok(sdot, N * cin, torch.float32, "sdot")
    _prof_call("mia_upconv_dgrad", flops if flops is not None else 2 * N * R * R * 9 * Cout * cin,
               ptr(g_t), ptr(w_t), ptr(gx), N, R, Cout, cin, ptr(x_fwd), act_x, ptr(style),
               ptr(sdot), dt(T), stream())
    return gx


def upconv_dgrad_fused(g_t, w_t, gx, cin, x_fwd, style, sdot, bab, accumulate, flops=None):
    """upconv_dgrad with the fused backward front of the layer below (mia_upconv_dgrad_fused):
    gx ← demod-scaled pre-activation gradient of that layer; bab = dict(demod, noise, noise_w,
    bias, q)."""
    N, TS, _, Cout = g_t.shape
    R = (TS - 1) // 2
    T = g_t.dtype
    _need(w_t, (cin, conv_kpad(Cout, T)), T, "w_t")
    _need(gx, (N, R, R, cin), T, "gx")
    _need(x_fwd, (N, R, R, cin), T, "x_fwd")
    _numel_ok(style, N * cin, torch.float32, "style")
    _numel_ok(sdot, N * cin, torch.float32, "sdot")
    _numel_ok(bab["demod"], N * cin, torch.float32, "bab.demod")
    _numel_ok(bab["q"], N * cin, torch.float32, "bab.q")
    _numel_ok(bab.get("noise"), R * R, torch.float32, "bab.noise")
    _numel_ok(bab.get("bias"), cin, torch.float32, "bab.bias")
    ws = layouts.split_for(w_t) if T == torch.float32 else None
    _prof_call("mia_upconv_dgrad_fused_split",
               flops if flops is not None else 2 * N * R * R * 9 * Cout * cin,
               ptr(g_t), ptr(w_t), ptr(ws), ptr(gx), N, R, Cout, cin, ptr(x_fwd), ptr(style),
               ptr(sdot),
               int(bool(accumulate)), ptr(bab["demod"]), ptr(bab.get("noise")),
               float(bab.get("noise_w", 0.0)), ptr(bab.get("bias")), ptr(bab["q"]), dt(T),
               stream())
    return gx


def bias_act_fwd(x, noise, noise_w, bias, y):
    N, H, W, C = x.shape
    _need(y, x.shape, x.dtype, "y")
    _numel_ok(noise, H * W, torch.float32, "noise")
    _numel_ok(bias, C, torch.float32, "bias")
    call("mia_bias_act_fwd", ptr(x), ptr(noise), float(noise_w), ptr(bias), ptr(y), N, H, W, C,
         dt(x), stream())
    return y


def bias_act_bwd(g_a, pre, noise, noise_w, bias, demod, gy, q, unshuffle=False, from_act=False):
    N, H, W, C = pre.shape
    _need(g_a, pre.shape, pre.dtype, "g_a")
    _numel_ok(noise, H * W, torch.float32, "noise")
    _numel_ok(bias, C, torch.float32, "bias")
    _numel_ok(demod, N * C, torch.float32, "demod")
    _numel_ok(q, N * C, torch.float32, "q")
    if unshuffle:
        _need(gy, (N, H // 2, W // 2, 4 * C), pre.dtype, "gy")
    else:
        _need(gy, pre.shape, pre.dtype, "gy")
    call("mia_bias_act_bwd", ptr(g_a), ptr(pre), ptr(noise), float(noise_w), ptr(bias), ptr(demod),
         ptr(gy), ptr(q), N, H, W, C, int(bool(unshuffle)), int(bool(from_act)), dt(pre), stream())
    return gy


def _updn_out(H, up, down, p0, p1, kt):
    return (H * up + p0 + p1 - kt) // down + 1


def upfirdn2d_fwd(x, y, k1d, up=1, down=1, pad=(0, 0)):
    """x: (..., H, W) fp32; k1d: host list of taps."""
    H, W = x.shape[-2:]
    planes = x.numel() // (H * W)
    kt = len(k1d)
    Ho, Wo = _updn_out(H, up, down, pad[0], pad[1], kt), _updn_out(W, up, down, pad[0], pad[1], kt)
    _need(y, tuple(x.shape[:-2]) + (Ho, Wo), torch.float32, "y")
    k = (ctypes.c_float * kt)(*k1d)
    call("mia_upfirdn2d_fwd", ptr(x), ptr(y), planes, H, W, k, kt, up, down, pad[0], pad[1],
         stream())
    return y


def upfirdn2d_bwd(gy, gx, k1d, up=1, down=1, pad=(0, 0)):
    H, W = gx.shape[-2:]
    planes = gx.numel() // (H * W)
    kt = len(k1d)
    Ho, Wo = _updn_out(H, up, down, pad[0], pad[1], kt), _updn_out(W, up, down, pad[0], pad[1], kt)
    _need(gy, tuple(gx.shape[:-2]) + (Ho, Wo), torch.float32, "gy")
    k = (ctypes.c_float * kt)(*k1d)
    call("mia_upfirdn2d_bwd", ptr(gy), ptr(gx), planes, H, W, k, kt, up, down, pad[0], pad[1],
         stream())
    return gx


def torgb_fwd(pre, style, wr, bias, skip, rgb, act_in=ACT_LRELU_S2):
    N, H, W, Cin = pre.shape
    _numel_ok(style, N * Cin, torch.float32, "style")
    _need(wr, (3, Cin), torch.float32, "wr")
    _numel_ok(bias, 3, torch.float32, "bias")
    if skip is not None:
        _need(skip, (N, 3, H // 2, W // 2), torch.float32, "skip")
    _need(rgb, (N, 3, H, W), torch.float32, "rgb")
    call("mia_torgb_fwd", ptr(pre), ptr(style), ptr(wr), ptr(bias), ptr(skip), ptr(rgb), N, H, W,
         Cin, int(act_in), dt(pre), stream())
    return rgb


def torgb_bwd(g_rgb, pre, style, wr, g_a, gs, accumulate, act_in=ACT_LRELU_S2):
    N, H, W, Cin = pre.shape
    _need(g_rgb, (N, 3, H, W), torch.float32, "g_rgb")
    _numel_ok(style, N * Cin, torch.float32, "style")
    _need(wr, (3, Cin), torch.float32, "wr")
    _need(g_a, pre.shape, pre.dtype, "g_a")
    _numel_ok(gs, N * Cin, torch.float32, "gs")
    call("mia_torgb_bwd", ptr(g_rgb), ptr(pre), ptr(style), ptr(wr), ptr(g_a), ptr(gs), N, H, W,
         Cin, int(bool(accumulate)), int(act_in), dt(pre), stream())


def torgb_bwd_front(g_rgb, act, style, wr, gy, gs, demod, noise, noise_w, bias, q):
    """ToRGB backward + the topmost StyledConv's backward front (mia_torgb_bwd_front)."""
    N, H, W, Cin = act.shape
    _need(g_rgb, (N, 3, H, W), torch.float32, "g_rgb")
    _need(gy, act.shape, act.dtype, "gy")
    _numel_ok(style, N * Cin, torch.float32, "style")
    _numel_ok(wr, 3 * Cin, torch.float32, "wr")
    _numel_ok(gs, N * Cin, torch.float32, "gs")
    _numel_ok(demod, N * Cin, torch.float32, "demod")
    _numel_ok(q, N * Cin, torch.float32, "q")
    _numel_ok(noise, H * W, torch.float32, "noise")
    _numel_ok(bias, Cin, torch.float32, "bias")
    call("mia_torgb_bwd_front", ptr(g_rgb), ptr(act), ptr(style), ptr(wr), ptr(gy), ptr(gs), N,
         H, W, Cin, ptr(demod), ptr(noise), float(noise_w), ptr(bias), ptr(q), dt(act), stream())
    return gy


def pool_out(H, ceil_mode):
    return (H + 1) // 2 if ceil_mode else H // 2


def maxpool2_fwd(x, y, ceil_mode=False):
    N, H, W, C = x.shape
    _need(y, (N, pool_out(H, ceil_mode), pool_out(W, ceil_mode), C), x.dtype, "y")
    call("mia_maxpool2_fwd", ptr(x), ptr(y), N, H, W, C, int(bool(ceil_mode)), dt(x), stream())
    return y


def maxpool2_bwd(x, g_out, g_in, ceil_mode=False, tap_t=None, tap_coef=0.0, mask=False):
    N, H, W, C = x.shape
    _need(g_out, (N, pool_out(H, ceil_mode), pool_out(W, ceil_mode), C), x.dtype, "g_out")
    _need(g_in, x.shape, x.dtype, "g_in")
    if tap_t is not None:
        _need(tap_t, x.shape, x.dtype, "tap_t")
    call("mia_maxpool2_bwd", ptr(x), ptr(g_out), ptr(g_in), N, H, W, C, int(bool(ceil_mode)),
         ptr(tap_t), float(tap_coef), int(bool(mask)), dt(x), stream())
    return g_in


def avgpool_fwd(x, y, k):
    H, W = x.shape[-2:]
    planes = x.numel() // (H * W)
    _need(y, tuple(x.shape[:-2]) + (H // k, W // k), torch.float32, "y")
    call("mia_avgpool_fwd", ptr(x), ptr(y), planes, H, W, k, stream())
    return y


def avgpool_bwd(gy, gx, k, accumulate=False):
    H, W = gx.shape[-2:]
    planes = gx.numel() // (H * W)
    _need(gy, tuple(gx.shape[:-2]) + (H // k, W // k), torch.float32, "gy")
    call("mia_avgpool_bwd", ptr(gy), ptr(gx), planes, H, W, k, int(bool(accumulate)), stream())
    return gx


def image_to_nhwc(x, y, pf, cpad):
    N, C, S, _ = x.shape
    if C != 3 or x.dtype != torch.float32:
        raise ValueError("x must be (N,3,S,S) fp32")
    _need(y, (N, S // pf, S // pf, cpad), None, "y")
    call("mia_image_to_nhwc", ptr(x), ptr(y), N, S, pf, cpad, dt(y), stream())
    return y


def mse_sum(a, b, loss, coef=1.0):
    """loss[n] += coef·Σ (a[n] − b[n])²."""
    n = a.shape[0]
    _need(b, a.shape, a.dtype, "b")
    _numel_ok(loss, n, torch.float32, "loss")
    call("mia_mse_sum", ptr(a), ptr(b), ptr(loss), n, a.numel() // n, float(coef), dt(a), stream())
    return loss


def ssim_workspace_numel(N, H, W):
    """fp64 elements of mia_ssim2's scratch (one partial per image and output tile)."""
    return int(_lib.load().mia_ssim_workspace_size(N, H, W)) // 8


def ssim(ref, imgs, data_range, work, out):
    """mia_ssim2: ref (3,H,W), imgs (N,3,H,W) fp32 → out[n] = SSIM(gray(ref), gray(imgs[n]))."""
    N, _, H, W = imgs.shape
    _need(ref, (3, H, W), torch.float32, "ref")
    _need(imgs, (N, 3, H, W), torch.float32, "imgs")
    _numel_ok(work, ssim_workspace_numel(N, H, W), torch.float64, "work")
    _numel_ok(out, N, torch.float32, "out")
    call("mia_ssim2", ptr(ref), ptr(imgs), N, H, W, float(data_range), ptr(work),
         work.numel() * work.element_size(), ptr(out), stream())
    return out


def mse_grad_f32(a, b, g, coef, accumulate=False):
    _need(b, a.shape, torch.float32, "b")
    _need(g, a.shape, torch.float32, "g")
    call("mia_mse_grad_f32", ptr(a), ptr(b), ptr(g), a.numel(), float(coef),
         int(bool(accumulate)), stream())
    return g


def tap_grad(a, t, g, coef, mask=True):
    _need(t, a.shape, a.dtype, "t")
    _need(g, a.shape, a.dtype, "g")
    call("mia_tap_grad", ptr(a), ptr(t), ptr(g), a.numel(), float(coef), int(bool(mask)), dt(a),
         stream())
    return g


def image_grad(rec, t, g_vgg, g_img, pf, coef):
    N, _, S, _ = rec.shape
    _need(t, rec.shape, torch.float32, "t")
    _need(g_img, rec.shape, torch.float32, "g_img")
    cpad = 8
    if g_vgg is not None:
        _need(g_vgg, (N, S // pf, S // pf, g_vgg.shape[-1]), None, "g_vgg")
        cpad = g_vgg.shape[-1]
    gdt = dt(g_vgg) if g_vgg is not None else _lib.MIA_F32
    call("mia_image_grad", ptr(rec), ptr(t), ptr(g_vgg), ptr(g_img), N, S, pf, cpad, float(coef),
         gdt, stream())
    return g_img


def pgd_update(x, x0, g_vgg, g_enc, pf, enc_res, coef_img, a, e, lo=-1.0, hi=1.0,
               nonfinite=None):
    N, _, S, _ = x.shape
    _numel_ok(nonfinite, N, torch.int32, "nonfinite")
    _need(x0, x.shape, torch.float32, "x0")
    cpad = 8
    if g_vgg is not None:
        _need(g_vgg, (N, S // pf, S // pf, g_vgg.shape[-1]), None, "g_vgg")
        cpad = g_vgg.shape[-1]
    if g_enc is not None:
        _numel_ok(g_enc, N * 3 * enc_res * enc_res, torch.float32, "g_enc")
    gdt = dt(g_vgg) if g_vgg is not None else _lib.MIA_F32
    call("mia_pgd_update", ptr(x), ptr(x0), ptr(g_vgg), ptr(g_enc), N, S, pf, cpad, enc_res,
         float(coef_img), float(a), float(e), float(lo), float(hi), ptr(nonfinite), gdt, stream())
    return x


def grad_assemble(x, x0, g_vgg, g_enc, g, pf, enc_res, coef_img, scale=1.0, nonfinite=None):
    """∇_x L (fp32 NCHW) from the VGG input-path and encoder gradients (mia_grad_assemble)."""
    N, C, S, S2 = x.shape
    _numel_ok(nonfinite, N, torch.int32, "nonfinite")
    if C != 3 or S != S2:
        raise ValueError("x must be (N,3,S,S)")
    _need(x0, x.shape, torch.float32, "x0")
    _need(g, x.shape, torch.float32, "g")
    R = S // pf
    cpad = g_vgg.shape[-1] if g_vgg is not None else 8
    if g_vgg is not None:
        _need(g_vgg, (N, R, R, cpad), None, "g_vgg")
    if g_enc is not None:
        _need(g_enc, (N, 3, enc_res, enc_res), torch.float32, "g_enc")
    T = g_vgg.dtype if g_vgg is not None else torch.float32
    call("mia_grad_assemble", ptr(x), ptr(x0), ptr(g_vgg), ptr(g_enc), ptr(g), N, S, pf, cpad,
         enc_res, float(coef_img), float(scale), ptr(nonfinite), dt(T), stream())
    return g


def cw_init(x, w):
    _need(w, x.shape, torch.float32, "w")
    call("mia_cw_init", ptr(x), ptr(w), x.numel(), stream())
    return w


def cw_tanh(w, adv):
    _need(adv, w.shape, torch.float32, "adv")
    call("mia_cw_tanh", ptr(w), ptr(adv), w.numel(), stream())
    return adv


def cw_grad(adv, x, g_f, g_w, c, scale=1.0):
    for name, t in (("x", x), ("g_f", g_f), ("g_w", g_w)):
        _need(t, adv.shape, torch.float32, name)
    call("mia_cw_grad", ptr(adv), ptr(x), ptr(g_f), ptr(g_w), adv.numel(), float(c), float(scale),
         stream())
    return g_w


def cw_select(adv, best_adv, sq, best_l2, f, f0, l2_scale):
    N = adv.shape[0]
    _need(best_adv, adv.shape, torch.float32, "best_adv")
    for name, t in (("sq", sq), ("best_l2", best_l2), ("f", f), ("f0", f0)):
        _numel_ok(t, N, torch.float32, name)
    call("mia_cw_select", ptr(adv), ptr(best_adv), ptr(sq), ptr(best_l2), ptr(f), ptr(f0), N,
         adv.numel() // N, float(l2_scale), stream())
    return best_adv


def random_start(x, x0, u, e, lo=-1.0, hi=1.0):
    _need(x0, x.shape, torch.float32, "x0")
    _need(u, x.shape, torch.float32, "u")
    call("mia_random_start", ptr(x), ptr(x0), ptr(u), x.numel(), float(e), float(lo), float(hi),
         stream())
    return x


def sign_project(x, x0, g, a, e, lo=-1.0, hi=1.0):
    _need(x0, x.shape, torch.float32, "x0")
    _need(g, x.shape, torch.float32, "g")
    call("mia_sign_project", ptr(x), ptr(x0), ptr(g), x.numel(), float(a), float(e), float(lo),
         float(hi), stream())
    return x


def adam_step(p, g, m, v, lr, beta1, beta2, eps, t):
    for name, z in (("g", g), ("m", m), ("v", v)):
        _need(z, p.shape, torch.float32, name)
    call("mia_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr), float(beta1),
         float(beta2), float(eps), int(t), stream())
    return p


def patch_update(patch, g, img, mask, adv, lo, hi):
    """adversarial_patch.py:131-134: patch −= g (g None: composite only); adv ← clamp((1−m)·img +
    m·patch, lo, hi). patch / mask: img's shape, or one image's shape (composite only)."""
    _need(adv, img.shape, torch.float32, "adv")
    _need(img, img.shape, torch.float32, "img")
    full = patch.numel() == img.numel()
    if not full and (g is not None or img.numel() % patch.numel()):
        raise ValueError("patch / mask: img's shape, or one image's shape for the composite")
    _need(mask, patch.shape, torch.float32, "mask")
    if g is not None:
        _need(g, img.shape, torch.float32, "g")
    call("mia_patch_update", ptr(patch), ptr(g) if g is not None else None, ptr(img), ptr(mask),
         ptr(adv), img.numel(), 0 if full else patch.numel(), float(lo), float(hi), stream())
    return adv


def gemm(M, N, K, alpha, A, sam, sak, B, sbk, sbn, beta, C, scm, scn, bias=None):
    """C[m,n] = alpha Σ_k A[m*sam+k*sak] B[k*sbk+n*sbn] + beta C[m*scm+n*scn] + bias[n] (fp32).
    Offsets into A/B/C are given by passing views (data_ptr of a strided view is honoured)."""
    for name, t, span in (("A", A, (M - 1) * sam + (K - 1) * sak),
                          ("B", B, (K - 1) * sbk + (N - 1) * sbn),
                          ("C", C, (M - 1) * scm + (N - 1) * scn)):
        if t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError(f"gemm {name}: cuda fp32 required")
        avail = t.untyped_storage().nbytes() // 4 - t.storage_offset()
        if span >= avail:
            raise ValueError(f"gemm {name}: strided span {span} exceeds storage {avail}")
    _numel_ok(bias, N, torch.float32, "bias")
    c = ctypes.c_void_p
    call("mia_gemm_f32", M, N, K, float(alpha), c(A.data_ptr()), sam, sak, c(B.data_ptr()), sbk,
         sbn, float(beta), c(C.data_ptr()), scm, scn, ptr(bias), stream())
    return C


def _span_ok(name, t, span):
    if t.dtype != torch.float32 or not t.is_cuda:
        raise ValueError(f"gemm {name}: cuda fp32 required")
    avail = t.untyped_storage().nbytes() // 4 - t.storage_offset()
    if span >= avail:
        raise ValueError(f"gemm {name}: strided span {span} exceeds storage {avail}")


class GemmPlan:
    """A validated, reusable list of grouped-GEMM descriptors (mia_gemm_f32_grouped).

    ``add(C, scm, scn, M, N, segs, alpha, beta, bias)`` with ``segs`` = [(A, sam, sak, B, sbk,
    sbn, K), ...] (≤ 2). Tensors are kept alive by the plan; the descriptor array is built once
    and launched by ``run()`` (the buffers are workspace-resident, so the pointers are stable)."""

    def __init__(self):
        self.groups = []
        self._keep = []
        self._arr = None

    def add(self, C, scm, scn, M, N, segs, alpha=1.0, beta=0.0, bias=None):
        if not 1 <= len(segs) <= 2:
            raise ValueError("1 or 2 segments per group")
        _span_ok("C", C, (M - 1) * scm + (N - 1) * scn)
        _numel_ok(bias, N, torch.float32, "bias")
        g = _lib.GemmGroup()
        g.C, g.bias = C.data_ptr(), (bias.data_ptr() if bias is not None else None)
        g.scm, g.scn, g.M, g.N = scm, scn, M, N
        g.alpha, g.beta, g.nseg = float(alpha), float(beta), len(segs)
        for i, (A, sam, sak, B, sbk, sbn, K) in enumerate(segs):
            _span_ok("A", A, (M - 1) * sam + (K - 1) * sak)
            _span_ok("B", B, (K - 1) * sbk + (N - 1) * sbn)
            g.seg[i] = _lib.GemmSeg(A.data_ptr(), B.data_ptr(), sam, sak, sbk, sbn, K)
            self._keep += [A, B]
        self._keep += [C] + ([bias] if bias is not None else [])
        self.groups.append(g)
        self._arr = None

    def run(self):
        if not self.groups:
            return
        if self._arr is None:
            self._arr = (_lib.GemmGroup * len(self.groups))(*self.groups)
        call("mia_gemm_f32_grouped", self._arr, len(self.groups), stream())


def style_demod(s, wsq, demod, scale2=1.0):
    N, Cin = s.shape
    Cout = wsq.shape[0]
    _need(wsq, (Cout, Cin), torch.float32, "wsq")
    _need(demod, (N, Cout), torch.float32, "demod")
    call("mia_style_demod", ptr(s), ptr(wsq), ptr(demod), N, Cin, Cout, float(scale2), stream())
    return demod


def demod_bwd(q, demod, wsq, s, gs, scale2=1.0):
    N, Cin = s.shape
    Cout = wsq.shape[0]
    _need(q, (N, Cout), torch.float32, "q")
    _need(demod, (N, Cout), torch.float32, "demod")
    _need(gs, (N, Cin), torch.float32, "gs")
    call("mia_demod_bwd", ptr(q), ptr(demod), ptr(wsq), ptr(s), ptr(gs), N, Cin, Cout,
         float(scale2), stream())
    return gs


def repeat(src, dst, count):
    if dst.numel() != src.numel() * count or dst.dtype != src.dtype:
        raise ValueError("repeat: size mismatch")
    call("mia_repeat", ptr(src), ptr(dst), src.numel() * src.element_size(), count, stream())
    return dst


def pixel_norm(x, y, eps=1e-8):
    rows, cols = x.shape
    _need(y, x.shape, torch.float32, "y")
    call("mia_pixel_norm", ptr(x), ptr(y), rows, cols, float(eps), stream())
    return y


def truncate(w, mean, psi, out):
    cols = w.shape[-1]
    rows = w.numel() // cols
    _need(out, w.shape, torch.float32, "out")
    _numel_ok(mean, cols, torch.float32, "mean")
    call("mia_truncate", ptr(w), ptr(mean), float(psi), ptr(out), rows, cols, stream())
    return out


def zero_(t):
    call("mia_memset", ptr(t), 0, t.numel() * t.element_size(), stream())
    return t


# ---- general-geometry conv and the e4e encoder kernels (csrc/encoder.hip) ----------------------
def conv2d_kpad(taps, cin, dtype):
    bk = 32 if dtype == torch.float32 else 64
    return (taps * cin + bk - 1) // bk * bk


def conv2d(x, groups, y, out_hw, *, cout, stride=1, bias=None, act_out=ACT_NONE, act_slope=None,
           mask_a=None, mask_slope=None, csum=None, accumulate=False, out_scale=None, flops=None):
    """mia_conv2d: 1..4 problems over x (N,H,W,Cin) sharing one epilogue. ``groups``: list of
    dict(w, kh, kw, pad=(py,px), ho, wo, a=(ay,ax), b=(by,bx)); w is [Cout][conv2d_kpad(kh·kw,
    Cin)]. y: (N, out_h, out_w, Cout). mask_a lives on y's pixel grid."""
    N, H, W, Cin = x.shape
    T = x.dtype
    oh, ow = out_hw
    if Cin % VEC[T]:
        raise ValueError("Cin must be a multiple of the 16-byte vector")
    if not 1 <= len(groups) <= 4:
        raise ValueError("1..4 groups")
    _need(y, (N, oh, ow, cout), T, "y")
    f32 = torch.float32
    _numel_ok(bias, cout, f32, "bias")
    _numel_ok(act_slope, cout, f32, "act_slope")
    _numel_ok(mask_slope, cout, f32, "mask_slope")
    _numel_ok(csum, N * cout, f32, "csum")
    _numel_ok(out_scale, N * cout, f32, "out_scale")
    if mask_a is not None:
        _need(mask_a, (N, oh, ow, cout), T, "mask_a")
    if act_out == ACT_PRELU and act_slope is None:
        raise ValueError("ACT_PRELU needs act_slope")
    garr = (_lib.ConvGroup * len(groups))()
    keep = []
    mac = 0
    for i, g in enumerate(groups):
        kh, kw = g["kh"], g["kw"]
        _need(g["w"], (cout, conv2d_kpad(kh * kw, Cin, T)), T, f"w[{i}]")
        py, px = g.get("pad", (0, 0))
        ay, ax = g.get("a", (1, 1))
        by, bx = g.get("b", (0, 0))
        ho, wo = g["ho"], g["wo"]
        if ho <= 0 or wo <= 0 or ay * (ho - 1) + by >= oh or ax * (wo - 1) + bx >= ow:
            raise ValueError(f"group {i}: placement outside the output grid")
        wsp = layouts.split_for(g["w"]) if T == torch.float32 else None
        garr[i] = _lib.ConvGroup(ptr(g["w"]).value, kh, kw, py, px, ho, wo, ay, by, ax, bx,
                                 ptr(wsp).value if wsp is not None else None)
        keep.append(g["w"])
        keep.append(wsp)
        mac += N * ho * wo * kh * kw * Cin * cout
    a = ConvArgs()
    a.x, a.y = ptr(x), ptr(y)
    a.N, a.H, a.W, a.Cin, a.Cout = N, H, W, Cin, cout
    a.bias, a.out_scale = ptr(bias), ptr(out_scale)
    a.act_out, a.act_slope = act_out, ptr(act_slope)
    a.mask_a, a.mask_slope, a.csum = ptr(mask_a), ptr(mask_slope), ptr(csum)
    a.accumulate = int(bool(accumulate))
    prof = PROFILE
    if prof is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    call("mia_conv2d", ctypes.byref(a), int(stride), garr, len(groups), oh, ow, dt(T), stream())
    if prof is not None:
        e1.record()
        prof.append((e0, e1, flops if flops is not None else 2 * mac))
        _tag(f"conv2d {H}x{W} {Cin}->{cout} s{stride} g{len(groups)} k{groups[0]['kh']}"
             + (" mask" if mask_a is not None else "") + (" acc" if accumulate else ""))
    return y


def conv2d_batched(x, groups, y, out_hw, *, n, cout, stride=1, bias=None, act_out=ACT_NONE,
                   act_slope=None, mask_a=None, mask_slope=None, accumulate=False, flops=None):
    """mia_conv2d_batched: up to 16 independent convs of one launch. x (Sx·n, H, W, Cin) and y
    (Sy·n, out_h, out_w, Cout) hold the groups' images stacked along N; each group dict is as in
    conv2d plus n_in / n_out (first input / output image) and c_off (channel offset into the
    concatenated per-channel operands bias, act_slope, mask_slope). mask_a lives on y's grid."""
    _, H, W, Cin = x.shape
    T = x.dtype
    oh, ow = out_hw
    if Cin % VEC[T]:
        raise ValueError("Cin must be a multiple of the 16-byte vector")
    if not 1 <= len(groups) <= 16:
        raise ValueError("1..16 groups")
    if y.dim() != 4 or tuple(y.shape[1:]) != (oh, ow, cout) or y.dtype != T:
        raise ValueError(f"y: (S·n, {oh}, {ow}, {cout}) {T} required")
    if mask_a is not None and (mask_a.shape != y.shape or mask_a.dtype != T):
        raise ValueError("mask_a must match y")
    if act_out == ACT_PRELU and act_slope is None:
        raise ValueError("ACT_PRELU needs act_slope")
    garr = (_lib.ConvGroup * len(groups))()
    barr = (_lib.ConvBatch * len(groups))()
    keep = []
    mac = 0
    for i, g in enumerate(groups):
        kh, kw = g["kh"], g["kw"]
        _need(g["w"], (cout, conv2d_kpad(kh * kw, Cin, T)), T, f"w[{i}]")
        py, px = g.get("pad", (0, 0))
        ay, ax = g.get("a", (1, 1))
        by, bx = g.get("b", (0, 0))
        ho, wo = g["ho"], g["wo"]
        if ho <= 0 or wo <= 0 or ay * (ho - 1) + by >= oh or ax * (wo - 1) + bx >= ow:
            raise ValueError(f"group {i}: placement outside the output grid")
        n_in, n_out, c_off = g.get("n_in", 0), g.get("n_out", 0), g.get("c_off", 0)
        if n_in < 0 or n_in + n > x.shape[0] or n_out < 0 or n_out + n > y.shape[0]:
            raise ValueError(f"group {i}: image range outside x / y")
        if c_off % 8:
            raise ValueError(f"group {i}: c_off must be a multiple of 8")
        for name, t in (("bias", bias), ("act_slope", act_slope), ("mask_slope", mask_slope)):
            if t is not None and (t.dtype != torch.float32 or t.numel() < c_off + cout):
                raise ValueError(f"group {i}: {name} shorter than c_off + cout")
        wsp = layouts.split_for(g["w"]) if T == torch.float32 else None
        garr[i] = _lib.ConvGroup(ptr(g["w"]).value, kh, kw, py, px, ho, wo, ay, by, ax, bx,
                                 ptr(wsp).value if wsp is not None else None)
        barr[i] = _lib.ConvBatch(n_in, n_out, c_off)
        keep += [g["w"], wsp]
        mac += n * ho * wo * kh * kw * Cin * cout
    a = ConvArgs()
    a.x, a.y = ptr(x), ptr(y)
    a.N, a.H, a.W, a.Cin, a.Cout = n, H, W, Cin, cout
    a.bias = ptr(bias)
    a.act_out, a.act_slope = act_out, ptr(act_slope)
    a.mask_a, a.mask_slope = ptr(mask_a), ptr(mask_slope)
    a.accumulate = int(bool(accumulate))
    prof = PROFILE
    if prof is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    call("mia_conv2d_batched", ctypes.byref(a), int(stride), garr, barr, len(groups), oh, ow, dt(T),
         stream())
    if prof is not None:
        e1.record()
        prof.append((e0, e1, flops if flops is not None else 2 * mac))
        _tag(f"conv2d_batched {H}x{W} {Cin}->{cout} s{stride} x{len(groups)} k{groups[0]['kh']}"
             + (" mask" if mask_a is not None else "") + (" acc" if accumulate else ""))
    return y


def conv2d_planes(x, w, b, y, out_hw, *, planes, act_out=ACT_NONE, act_slope=None, flops=None):
    """mia_conv2d_planes: one stride-2 pad-1 3×3 conv over x (N,H,W,Cin) with Cout = planes·C
    (w: [planes·C][Kpad], the heads' matrices concatenated along Cout; b: planes·C), output
    plane p (channels p·C … p·C+C−1) written to y[p·N:(p+1)·N] of y (planes·N, oh, ow, C)."""
    N, H, W, Cin = x.shape
    T = x.dtype
    oh, ow = out_hw
    P = int(planes)
    C = y.shape[-1]
    cout = P * C
    _need(y, (P * N, oh, ow, C), T, "y")
    _need(w, (cout, conv2d_kpad(9, Cin, T)), T, "w")
    _numel_ok(b, cout, torch.float32, "b")
    if act_out == ACT_PRELU and (act_slope is None or act_slope.numel() < cout):
        raise ValueError("ACT_PRELU needs act_slope of Cout entries")
    wsp = layouts.split_for(w) if T == torch.float32 else None
    g = _lib.ConvGroup(ptr(w).value, 3, 3, 1, 1, oh, ow, 1, 0, 1, 0,
                       ptr(wsp).value if wsp is not None else None)
    a = ConvArgs()
    a.x, a.y = ptr(x), ptr(y)
    a.N, a.H, a.W, a.Cin, a.Cout = N, H, W, Cin, cout
    a.y_cstride = C
    a.bias = ptr(b)
    a.act_out, a.act_slope = act_out, ptr(act_slope)
    prof = PROFILE
    if prof is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    call("mia_conv2d_planes", ctypes.byref(a), 2, ctypes.byref(g), oh, ow, C, N * oh * ow * C,
         dt(T), stream())
    if prof is not None:
        e1.record()
        prof.append((e0, e1, flops if flops is not None else 2 * N * oh * ow * 9 * Cin * cout))
        _tag(f"conv2d_planes {H}x{W} {Cin}->{C} s2 x{P}")
    return y


def se_fwd(csum, w1, w2, u, s, hw):
    N, C = csum.shape
    Cr = w1.shape[0]
    _need(w1, (Cr, C), torch.float32, "w1")
    _need(w2, (C, Cr), torch.float32, "w2")
    _need(u, (N, Cr), torch.float32, "u")
    _need(s, (N, C), torch.float32, "s")
    call("mia_se_fwd", ptr(csum), ptr(w1), ptr(w2), ptr(u), ptr(s), N, C, Cr, 1.0 / hw, stream())
    return s


def _parts_ok(part, N, hw, C):
    nch = chan_sum_parts(N, hw)
    if part.dtype != torch.float32 or part.numel() < N * nch * C:
        raise ValueError("SE partials: fp32 scratch of N · chan_sum_parts · C floats")
    return nch


def se_fwd_parts(part, hw, w1, w2, u, s):
    """se_fwd from chan_sum's partials (chan_sum(..., out=None)): the pool sum is finished inside
    the SE kernel in the same chunk order (mia_se_fwd_parts, bit-identical, one launch fewer)."""
    N, C = s.shape
    Cr = w1.shape[0]
    _need(w1, (Cr, C), torch.float32, "w1")
    _need(w2, (C, Cr), torch.float32, "w2")
    _need(u, (N, Cr), torch.float32, "u")
    nch = _parts_ok(part, N, hw, C)
    call("mia_se_fwd_parts", ptr(part), nch, ptr(w1), ptr(w2), ptr(u), ptr(s), N, C, Cr, 1.0 / hw,
         stream())
    return s


def se_bwd_parts(part, hw, s, u, w1, w2, gavg):
    """se_bwd from chan_sum's partials of gs = Σ ∂out·r (mia_se_bwd_parts)."""
    N, C = s.shape
    Cr = w1.shape[0]
    _need(u, (N, Cr), torch.float32, "u")
    _need(gavg, (N, C), torch.float32, "gavg")
    nch = _parts_ok(part, N, hw, C)
    call("mia_se_bwd_parts", ptr(part), nch, ptr(s), ptr(u), ptr(w1), ptr(w2), ptr(gavg), N, C,
         Cr, 1.0 / hw, stream())
    return gavg


def se_apply(r, s, sc, ss, out, g=None, b=None, xb=None):
    """out = r·s + sc (sc read at stride ss), xb = out·g + b (either output may be None)."""
    N, H, W, C = r.shape
    _numel_ok(s, N * C, torch.float32, "s")
    if sc is not None:
        _need(sc, (N, H * ss, W * ss, C), r.dtype, "sc")
    if out is not None:
        _need(out, r.shape, r.dtype, "out")
    if xb is not None:
        _need(xb, r.shape, r.dtype, "xb")
        _numel_ok(g, C, torch.float32, "g")
        _numel_ok(b, C, torch.float32, "b")
    call("mia_se_apply", ptr(r), ptr(s), ptr(sc), int(ss), ptr(out), ptr(g), ptr(b), ptr(xb), N,
         H, W, C, dt(r), stream())
    return out if out is not None else xb


def chan_dot(a, b, gs, accumulate=False):
    N, H, W, C = a.shape
    _need(b, a.shape, a.dtype, "b")
    _need(gs, (N, C), torch.float32, "gs")
    call("mia_chan_dot", ptr(a), ptr(b), ptr(gs), N, H * W, C, int(bool(accumulate)), dt(a),
         stream())
    return gs


def chan_sum_parts(N, HW):
    """Chunks per image of mia_chan_sum (host-side helper of the library, no device work)."""
    return _lib.load().mia_chan_sum_parts(int(N), int(HW))


def chan_sum(a, b, part, out, accumulate=False):
    """mia_chan_sum: out (N, C) fp32 (+)= Σ_pixels a·b (b given) or Σ_pixels a, deterministic;
    part: fp32 scratch of N · chan_sum_parts(N, H·W) · C floats. out None: only the ordered
    per-chunk partials (for se_fwd_parts / se_bwd_parts); returns part then."""
    N, H, W, C = a.shape
    if b is not None:
        _need(b, a.shape, a.dtype, "b")
    if out is not None:
        _need(out, (N, C), torch.float32, "out")
    elif accumulate:
        raise ValueError("chan_sum: accumulate needs out")
    if part.dtype != torch.float32 or part.numel() < N * chan_sum_parts(N, H * W) * C:
        raise ValueError("chan_sum: part scratch too small")
    call("mia_chan_sum", ptr(a), ptr(b), ptr(part), ptr(out), N, H * W, C,
         int(bool(accumulate)), dt(a), stream())
    return out if out is not None else part


def se_bwd(gs, s, u, w1, w2, gavg, hw):
    N, C = s.shape
    Cr = w1.shape[0]
    _need(gs, (N, C), torch.float32, "gs")
    _need(u, (N, Cr), torch.float32, "u")
    _need(gavg, (N, C), torch.float32, "gavg")
    call("mia_se_bwd", ptr(gs), ptr(s), ptr(u), ptr(w1), ptr(w2), ptr(gavg), N, C, Cr, 1.0 / hw,
         stream())
    return gavg


def se_grad_scale(g_out, s, gavg, g_r, gamma=None):
    N, H, W, C = g_out.shape
    _need(g_r, g_out.shape, g_out.dtype, "g_r")
    _numel_ok(gamma, C, torch.float32, "gamma")
    call("mia_se_grad_scale", ptr(g_out), ptr(s), ptr(gavg), ptr(gamma), ptr(g_r), N, H * W, C,
         dt(g_out), stream())
    return g_r


def prelu_bwd_scale(g_a, a, slope, g, gamma=None):
    C = g_a.shape[-1]
    _need(a, g_a.shape, g_a.dtype, "a")
    _need(g, g_a.shape, g_a.dtype, "g")
    _numel_ok(slope, C, torch.float32, "slope")
    _numel_ok(gamma, C, torch.float32, "gamma")
    call("mia_prelu_bwd_scale", ptr(g_a), ptr(a), ptr(slope), ptr(gamma), ptr(g),
         g_a.numel() // C, C, dt(g_a), stream())
    return g


def prelu_fwd(pre, slope, a):
    """a = pre > 0 ? pre : slope[c]·pre (NHWC, per-channel fp32 slope)."""
    C = pre.shape[-1]
    _need(a, pre.shape, pre.dtype, "a")
    _numel_ok(slope, C, torch.float32, "slope")
    call("mia_prelu_fwd", ptr(pre), ptr(slope), ptr(a), pre.numel() // C, C, dt(pre), stream())
    return a


def subsample_add(g, gx):
    N, H, W, C = g.shape
    _need(gx, (N, 2 * H, 2 * W, C), g.dtype, "gx")
    call("mia_subsample_add", ptr(g), ptr(gx), N, H, W, C, dt(g), stream())
    return gx


def bilinear_fwd(x, y, accumulate=False):
    N, Hi, Wi, C = x.shape
    _, Ho, Wo, C2 = y.shape
    if y.shape[0] != N or C2 != C or y.dtype != x.dtype:
        raise ValueError("bilinear_fwd: shape/dtype mismatch")
    call("mia_bilinear_fwd", ptr(x), ptr(y), N, Hi, Wi, Ho, Wo, C, int(bool(accumulate)), dt(x),
         stream())
    return y


def bilinear_bwd(gy, gx, accumulate=False):
    N, Ho, Wo, C = gy.shape
    _, Hi, Wi, C2 = gx.shape
    if gx.shape[0] != N or C2 != C or gx.dtype != gy.dtype:
        raise ValueError("bilinear_bwd: shape/dtype mismatch")
    call("mia_bilinear_bwd", ptr(gy), ptr(gx), N, Hi, Wi, Ho, Wo, C, int(bool(accumulate)),
         dt(gy), stream())
    return gx


def cast(x, y, scale=1.0):
    if x.numel() != y.numel():
        raise ValueError("cast: size mismatch")
    call("mia_cast", ptr(x), dt(x), ptr(y), dt(y), x.numel(), float(scale), stream())
    return y


def s2_dgrad_halo(g, w_halo, gx, mask_a=None, mask_slope=None, accumulate=False, flops=None):
    """mia_conv_s2_dgrad_halo(_multi): gx (N,2R,2R,Cx) ← input gradient of a stride-2 3×3 conv from
    g (N,R,R,Cg) (+ slope mask, + accumulate). ``g`` may be a list of up to 8 output gradients of
    convs reading the same tensor, with ``w_halo`` their packed matrices concatenated along dim 0:
    the sum of their input gradients in one K loop. fp32 passes the split_f32 copy of w_halo (the
    split-once kernel takes long K loops)."""
    gs = list(g) if isinstance(g, (list, tuple)) else [g]
    if not 1 <= len(gs) <= 8:
        raise ValueError("s2_dgrad_halo: 1..8 source gradients")
    N, R, R2, Cg = gs[0].shape
    for t in gs[1:]:
        _need(t, gs[0].shape, gs[0].dtype, "g[i]")
    Cx = gx.shape[-1]
    T = gs[0].dtype
    if R != R2:
        raise ValueError("square inputs only")
    bk = layouts.halo_bk(T)
    _need(w_halo, (len(gs) * Cg // bk, 5, 2, Cx, bk), T, "w_halo")
    _need(gx, (N, 2 * R, 2 * R, Cx), T, "gx")
    if mask_a is not None:
        _need(mask_a, gx.shape, T, "mask_a")
    _numel_ok(mask_slope, Cx, torch.float32, "mask_slope")
    gp = (ctypes.c_void_p * len(gs))(*[ptr(t).value for t in gs])
    ws = layouts.split_for(w_halo) if T == torch.float32 else None
    _prof_call("mia_conv_s2_dgrad_halo_multi",
               flops if flops is not None else 2 * N * R * R * 9 * len(gs) * Cg * Cx,
               gp, len(gs), ptr(w_halo), ptr(ws), ptr(gx), N, R, Cg, Cx, ptr(mask_a),
               ptr(mask_slope), int(bool(accumulate)), dt(T), stream())
    return gx


def s2_dgrad_halo_ok(dtype, R, Cg, Cx):
    """Host mirror of s2_dgrad_halo_eligible (csrc/conv_upconv.hip)."""
    if _lib.get_tuning("MIA_S2DG_HALO") == 0:
        return False
    return R % 16 == 0 and Cg % 64 == 0 and Cx % 64 == 0


def sum_slices(x, y):
    """y (N, D) = Σ_s x[:, s, :] for x (N, S, D) fp32."""
    N, S, D = x.shape
    _need(y, (N, D), torch.float32, "y")
    if x.dtype != torch.float32:
        raise ValueError("sum_slices: fp32 required")
    call("mia_sum_slices", ptr(x), ptr(y), N, S, D, stream())
    return y
