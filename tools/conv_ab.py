"""A/B timing of the 3×3 conv kernels on the attack step's layer shapes (GPU, tuning aid).

Usage: python tools/conv_ab.py [--batch 128] [--iters 5] VAR=a,b ...
Each VAR=v1,v2 names a kernel-variant switch of libmiattack (mia_set_tuning: MIA_CONV_HALO,
MIA_HALO_EPI, ...); every combination is timed on every shape with HIP events on the current
stream, and the algorithmic TFLOP/s (2·M·9·Cin·Cout) is printed. Not part of the product path."""
import argparse
import itertools
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import _lib, ops  # noqa: E402

# (name, H, Cin, Cout, mode)
SHAPES = [
    ("mod 256² 128→128", 256, 128, 128, "mod"),
    ("mod 128² 256→256", 128, 256, 256, "mod"),
    ("mod 64² 512→512", 64, 512, 512, "mod"),
    ("vgg 128² 64→128", 128, 64, 128, "vgg"),
    ("vgg 128² 128→128", 128, 128, 128, "vgg"),
    ("vgg 64² 256→256", 64, 256, 256, "vgg"),
    ("vgg 32² 512→512", 32, 512, 512, "vgg"),
    ("dgrad+sdot 256² 128→128", 256, 128, 128, "sdot"),
    ("dgrad+tap 64² 256→256", 64, 256, 256, "tap"),
    ("thin vgg1_1 256² 8→64", 256, 8, 64, "vgg"),
    ("thin dgrad 256² 64→8", 256, 64, 8, "plain"),
    # the attack's thin layers: an RGB image padded to 8 channels (3 real, zero weights elsewhere)
    ("thin rgb vgg1_1 256² 8→64", 256, 8, 64, "rgb"),
    ("thin rgb dgrad 256² 64→8", 256, 64, 8, "rgb"),
    ("thin rgb dgrad+acc 256² 64→8", 256, 64, 8, "rgbacc"),
    ("vgg 256² 64→64", 256, 64, 64, "vgg"),
    ("dgrad+tap 256² 64→64", 256, 64, 64, "tap"),
    ("dgrad 128² 128→64", 128, 128, 64, "plain"),
    ("mod 1024² 32→32", 1024, 32, 32, "mod"),
    ("mod 512² 64→64", 512, 64, 64, "mod"),
    ("dgrad+sdot 512² 64→64", 512, 64, 64, "sdot"),
    ("dgrad+sdot 1024² 32→32", 1024, 32, 32, "sdot"),
    ("dgrad+bab 1024² 32→32", 1024, 32, 32, "bab"),
    ("up 128²→256² 256→128", 128, 256, 128, "up"),
    ("up 64²→128² 512→256", 64, 512, 256, "up"),
    ("up 32²→64² 512→512", 32, 512, 512, "up"),
    # e4e IR-SE50 body (mia_conv2d epilogue features)
    ("e4e in prelu 256² 8→64", 256, 8, 64, "prelu"),
    ("e4e prelu 256² 64→64", 256, 64, 64, "prelu"),
    ("e4e bias+csum 128² 64→64", 128, 64, 64, "csum"),
    ("e4e mask+slope 128² 64→64", 128, 64, 64, "mslope"),
    ("e4e acc 128² 64→64", 128, 64, 64, "acc"),
    ("e4e prelu 64² 128→128", 64, 128, 128, "prelu"),
    ("e4e bias+csum 32² 256→256", 32, 256, 256, "csum"),
    ("e4e mask+slope 32² 256→256", 32, 256, 256, "mslope"),
    ("e4e acc 32² 256→256", 32, 256, 256, "acc"),
    # e4e GradualStyleBlock convs (stride 2, bias + LeakyReLU(0.01)); H = output side
    ("head s2 →32² 512→512", 32, 512, 512, "head"),
    ("head s2 →16² 512→512", 16, 512, 512, "head"),
    ("head s2 →8² 512→512", 8, 512, 512, "head"),
    ("head s2 →4² 512→512", 4, 512, 512, "head"),
    ("head s2 →2² 512→512", 2, 512, 512, "head"),
    ("head s2 →1² 512→512", 1, 512, 512, "head"),
]

E4E_MODES = ("prelu", "csum", "mslope", "acc", "head")


def run_e4e(H, Cin, Cout, mode, N, iters, dtype, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    s2 = 2 if mode == "head" else 1
    x = torch.randn(N, H * s2, H * s2, Cin, device=dev, generator=g).to(dtype)
    kp = ops.conv2d_kpad(9, Cin, dtype)
    w = (torch.randn(Cout, kp, device=dev, generator=g) / math.sqrt(9 * Cin)).to(dtype)
    y = torch.empty(N, H, H, Cout, device=dev, dtype=dtype)
    grp = [dict(w=w, kh=3, kw=3, pad=(1, 1), ho=H, wo=H)]
    slope = torch.rand(Cout, device=dev, generator=g) * 0.5 + 0.05
    kw = {}
    if mode in ("prelu", "head"):
        kw = dict(act_out=ops.ACT_PRELU, act_slope=slope)
    if mode == "head":
        kw.update(stride=2, bias=torch.randn(Cout, device=dev, generator=g))
    elif mode == "csum":
        kw = dict(bias=torch.randn(Cout, device=dev, generator=g),
                  csum=torch.zeros(N, Cout, device=dev))
    elif mode == "mslope":
        kw = dict(mask_a=torch.randn(N, H, H, Cout, device=dev, generator=g).to(dtype),
                  mask_slope=slope)
    elif mode == "acc":
        kw = dict(accumulate=True)
    call = lambda: ops.conv2d(x, grp, y, (H, H), cout=Cout, **kw)  # noqa: E731
    y.zero_()
    call()
    torch.cuda.synchronize()
    ref = y.float().clone()
    if "csum" in kw:
        ref = torch.cat([ref.flatten(), kw["csum"].flatten() / (H * H)])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, 2.0 * N * H * H * 9 * Cin * Cout / (ms * 1e-3) / 1e12, ref


def run_up(H, Cin, Cout, N, iters, dtype, dev):
    from gfa_amd import layouts
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=dev, generator=g).to(dtype)
    w = torch.randn(Cout, Cin, 3, 3, generator=torch.Generator().manual_seed(1)) / math.sqrt(9 * Cin)
    wph = [m.to(dev) for m in layouts.upconv_subpixel_matrices(w, dtype)]
    wup = layouts.upconv_halo_matrix(w, dtype).to(dev)
    s = torch.rand(N, Cin, device=dev, generator=g) + 0.5
    t = torch.empty(N, 2 * H + 1, 2 * H + 1, Cout, device=dev, dtype=dtype)
    call = lambda: ops.upconv_fwd(x, wph, t, Cout, style=s, w_up=wup)  # noqa: E731
    call()
    torch.cuda.synchronize()
    ref = t.float().clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, 2.0 * N * H * H * 9 * Cin * Cout / (ms * 1e-3) / 1e12, ref


def run(name, H, Cin, Cout, mode, N, iters, dtype, dev):
    if mode == "up":
        return run_up(H, Cin, Cout, N, iters, dtype, dev)
    if mode in E4E_MODES:
        return run_e4e(H, Cin, Cout, mode, N, iters, dtype, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=dev, generator=g).to(dtype)
    kp = ops.conv_kpad(Cin, dtype)
    w = (torch.randn(Cout, kp, device=dev, generator=g) / math.sqrt(9 * Cin)).to(dtype)
    y = torch.empty(N, H, H, Cout, device=dev, dtype=dtype)
    kw = {}
    if mode == "mod":
        kw = dict(in_scale=torch.rand(N, Cin, device=dev, generator=g) + 0.5,
                  out_scale=torch.rand(N, Cout, device=dev, generator=g) + 0.5,
                  noise=torch.randn(H * H, device=dev, generator=g), noise_w=0.1,
                  bias=torch.randn(Cout, device=dev, generator=g), act_out=ops.ACT_LRELU_S2)
    elif mode == "vgg":
        kw = dict(bias=torch.randn(Cout, device=dev, generator=g), act_out=ops.ACT_RELU)
    elif mode in ("rgb", "rgbacc"):
        if Cin == 8:  # forward: K = tap·8 + ci, channels ≥ 3 padded
            w.view(Cout, -1)[:, :72].view(Cout, 9, 8)[:, :, 3:] = 0
            x[..., 3:] = 0
            kw = dict(bias=torch.randn(Cout, device=dev, generator=g), act_out=ops.ACT_RELU)
        else:  # input gradient: output channels ≥ 3 padded
            w[3:] = 0
            kw = dict(accumulate=mode == "rgbacc")
    elif mode == "sdot":
        kw = dict(out_scale=torch.rand(N, Cout, device=dev, generator=g) + 0.5,
                  aux_x=torch.randn(N, H, H, Cout, device=dev, generator=g).to(dtype),
                  sdot=torch.zeros(N, Cout, device=dev))
    elif mode == "bab":  # StyledConv input gradient + the layer below's bias-act backward
        kw = dict(out_scale=torch.rand(N, Cout, device=dev, generator=g) + 0.5,
                  aux_x=torch.randn(N, H, H, Cout, device=dev, generator=g).to(dtype),
                  sdot=torch.zeros(N, Cout, device=dev),
                  bab=dict(demod=torch.rand(N, Cout, device=dev, generator=g) + 0.5,
                           noise=torch.randn(H * H, device=dev, generator=g), noise_w=0.1,
                           bias=torch.randn(Cout, device=dev, generator=g),
                           q=torch.zeros(N, Cout, device=dev)))
    elif mode == "tap":
        a = torch.randn(N, H, H, Cout, device=dev, generator=g).relu().to(dtype)
        kw = dict(tap_a=a, tap_t=torch.randn(N, H, H, Cout, device=dev, generator=g).to(dtype), tap_coef=0.3, mask_a=a)
    ops.conv3x3(x, w, y, cout=Cout, **kw)
    torch.cuda.synchronize()
    ref = y.float().clone()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.conv3x3(x, w, y, cout=Cout, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tf = 2.0 * N * H * H * 9 * Cin * Cout / (ms * 1e-3) / 1e12
    return ms, tf, ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "fp32"])
    ap.add_argument("--only", default="")
    ap.add_argument("vars", nargs="*")
    a = ap.parse_args()
    dtype = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype]
    dev = torch.device("cuda:0")
    keys = [v.split("=")[0] for v in a.vars]
    vals = [v.split("=")[1].split(",") for v in a.vars]
    combos = list(itertools.product(*vals)) or [()]
    for name, H, Cin, Cout, mode in SHAPES:
        if a.only and not any(o in name for o in a.only.split("|")):
            continue
        refs = []
        line = f"{name:28s}"
        for c in combos:
            for k, v in zip(keys, c):
                _lib.set_tuning(k, int(v))
            ms, tf, ref = run(name, H, Cin, Cout, mode, a.batch, a.iters, dtype, dev)
            refs.append(ref)
            d = (ref - refs[0]).abs().max().item() / max(refs[0].abs().max().item(), 1e-30)
            tag = ",".join(f"{k}={v}" for k, v in zip(keys, c))
            line += f" | {tag}: {ms:7.3f} ms {tf:6.1f} TF/s (d={d:.1e})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
