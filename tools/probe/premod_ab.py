"""A/B of the fp16 / bf16 halo kernel's modulated forward (conv_halo.hip, PRO launches): run the
StyledConv forward shapes of the 256² / 1024² generators with the loaded build and save outputs +
per-call times; `--compare A B` checks two saved runs bit for bit (tuning aid, not product).

    MIA_LIB_VARIANT=premod0 python tools/probe/premod_ab.py --out gpurun_out/premod0.pt
    python tools/probe/premod_ab.py --out gpurun_out/premod1.pt
    python tools/probe/premod_ab.py --compare gpurun_out/premod0.pt gpurun_out/premod1.pt
"""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import layouts, ops  # noqa: E402

SHAPES = [(128, 256, 128), (128, 128, 256), (128, 64, 512), (32, 512, 64), (32, 1024, 32)]


def run(out):
    dev = torch.device("cuda:0")
    res = {}
    for dtype in (torch.float16, torch.bfloat16):
        for N, H, C in SHAPES:
            g = torch.Generator().manual_seed(H + C)
            x = torch.randn(N, H, H, C, generator=g).to(dtype).to(dev)
            w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
            wm = layouts.fwd_matrix(w, dtype).to(dev)
            s = (torch.rand(N, C, generator=g) + 0.5).to(dev)
            d = (torch.rand(N, C, generator=g) + 0.5).to(dev)
            b = (torch.randn(C, generator=g) * 0.1).to(dev)
            nz = torch.randn(H * H, generator=g).to(dev)
            y = torch.empty(N, H, H, C, dtype=dtype, device=dev)

            def call():
                ops.conv3x3(x, wm, y, cout=C, in_scale=s, out_scale=d, noise=nz, noise_w=0.3,
                            bias=b, act_out=ops.ACT_LRELU_S2)
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            tf = 2 * N * H * H * 9 * C * C / (us * 1e-6) / 1e12
            key = f"{str(dtype)[6:]} N{N} {H}² {C}->{C}"
            print(f"{key:28s} {us:9.1f} us  {tf:7.1f} TF/s", flush=True)
            res[key] = (y.cpu(), us)
    torch.save(res, out)


def compare(a, b):
    A, B = torch.load(a, weights_only=False), torch.load(b, weights_only=False)
    ok = True
    for k in A:
        same = torch.equal(A[k][0], B[k][0])
        ok &= same
        print(f"{k:28s} bitwise {'equal' if same else 'DIFFERENT'}  {A[k][1]:9.1f} -> "
              f"{B[k][1]:9.1f} us ({100 * (A[k][1] / B[k][1] - 1):+.1f} % speed)")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    compare(*a.compare) if a.compare else run(a.out)
