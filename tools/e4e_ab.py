"""Per-layer timing of the e4e encoder's convolutions at the bench batch (GPU, tuning aid).

Usage: python tools/e4e_ab.py [--batch 128] [--iters 5] [VAR=a,b ...]
Times each conv shape of Encoder4Editing(50, 'ir_se') at 256² input (forward and input gradient)
with HIP events and prints algorithmic TFLOP/s; VAR=v1,v2 kernel-variant switches (mia_set_tuning) are A/B-compared as in tools/conv_ab.py. Not part of the product path."""
import argparse
import itertools
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import _lib, e4e, layouts, ops  # noqa: E402

# (name, kind, H_in, Cin, Cout, stride, count per encoder pass)
SHAPES = [
    ("stage1 conv1 128² 64→64 s1", "fwd", 128, 64, 64, 1, 5),
    ("stage1 conv2 256²→128² 64 s2", "fwd", 256, 64, 64, 2, 1),
    ("stage2 conv 64² 128 s1", "fwd", 64, 128, 128, 1, 6),
    ("stage3 conv 32² 256 s1", "fwd", 32, 256, 256, 1, 26),
    ("stage4 conv 16² 512 s1", "fwd", 16, 512, 512, 1, 4),
    ("stage3 conv2 64²→32² 256 s2", "fwd", 64, 256, 256, 2, 1),
    ("head fine 64²→32² 512 s2", "fwd", 64, 512, 512, 2, 7),
    ("head 32²→16² 512 s2", "fwd", 32, 512, 512, 2, 11),
    ("head 16²→8² 512 s2", "fwd", 16, 512, 512, 2, 14),
    ("head 8²→4² 512 s2", "fwd", 8, 512, 512, 2, 14),
    ("stage3 dgrad 32² 256 s1", "dgrad", 32, 256, 256, 1, 26),
    ("head fine dgrad 32²→64² 512", "dgrad", 64, 512, 512, 2, 7),
    ("head dgrad 16²→32² 512", "dgrad", 32, 512, 512, 2, 11),
    ("head dgrad 8²→16² 512", "dgrad", 16, 512, 512, 2, 14),
    ("stage1 dgrad 128²→256² 64 s2", "dgrad", 256, 64, 64, 2, 1),
]


def run(kind, H, Cin, Cout, stride, N, iters, dtype, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    w = torch.randn(Cout, Cin, 3, 3, generator=torch.Generator().manual_seed(1)) / math.sqrt(9 * Cin)
    ho = (H - 1) // 2 + 1 if stride == 2 else H
    if kind == "fwd":
        x = torch.randn(N, H, H, Cin, device=dev, generator=g).to(dtype)
        y = torch.empty(N, ho, ho, Cout, device=dev, dtype=dtype)
        wm = layouts.fwd_matrix(w, dtype).to(dev)
        slope = torch.full((Cout,), 0.01, device=dev)
        call = lambda: ops.conv2d(x, [e4e._g3(wm, ho)], y, (ho, ho), cout=Cout,  # noqa: E731
                                  stride=stride, act_out=ops.ACT_PRELU, act_slope=slope)
    else:
        gy = torch.randn(N, ho, ho, Cout, device=dev, generator=g).to(dtype)
        y = torch.empty(N, H, H, Cin, device=dev, dtype=dtype)
        a = torch.randn(N, H, H, Cin, device=dev, generator=g).to(dtype)
        slope = torch.full((Cin,), 0.25, device=dev)
        if stride == 2:
            ph = [(m.to(dev), py, px) for m, py, px in layouts.s2_dgrad_phases(w, dtype)]
            wh = layouts.s2_dgrad_halo_matrix(w, dtype).to(dev)
            call = lambda: e4e.E4EEncoder._s2_dgrad(gy, ph, wh, y, a, slope, False)  # noqa: E731
        else:
            groups = [e4e._g3(layouts.dgrad_matrix(w, dtype).to(dev), H)]
            call = lambda: ops.conv2d(gy, groups, y, (H, H), cout=Cin, mask_a=a,  # noqa: E731
                                      mask_slope=slope)
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, 2.0 * N * ho * ho * 9 * Cin * Cout / (ms * 1e-3) / 1e12, y.float().clone()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("vars", nargs="*")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    keys = [v.split("=")[0] for v in a.vars]
    vals = [v.split("=")[1].split(",") for v in a.vars]
    combos = list(itertools.product(*vals)) or [()]
    tot = {}
    for name, kind, H, Cin, Cout, stride, cnt in SHAPES:
        if a.only and not any(o in name for o in a.only.split("|")):
            continue
        line = f"{name:32s} x{cnt:2d}"
        ref = None
        for c in combos:
            for k, v in zip(keys, c):
                _lib.set_tuning(k, int(v))
            ms, tf, y = run(kind, H, Cin, Cout, stride, a.batch, a.iters, torch.float16, dev)
            ref = y if ref is None else ref
            d = (y - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
            tag = ",".join(f"{k}={v}" for k, v in zip(keys, c))
            line += f" | {tag}: {ms:7.3f} ms {tf:6.1f} TF/s (d={d:.1e}) Σ {ms * cnt:6.2f} ms"
            tot[tag] = tot.get(tag, 0.0) + ms * cnt
        print(line, flush=True)
    print("total per pass:", {k: round(v, 2) for k, v in tot.items()})


if __name__ == "__main__":
    main()
