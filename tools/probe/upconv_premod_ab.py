"""A/B of the 2-byte up-conv forward's style modulation (conv_upconv.hip upconv_halo_kernel, PRO
launches): run the up-sampling StyledConv shapes of the 256² / 1024² generators with the loaded
build, save outputs + per-call times; `--compare A B` checks two saved runs bit for bit (tuning
aid, not product). `--dtypes fp32,fp16` picks the dtypes (fp32: the split-once kernel + its
generic edge launch, as the product calls it).

    MIA_LIB_VARIANT=premod0 python tools/probe/upconv_premod_ab.py --out /tmp/up0.pt
    python tools/probe/upconv_premod_ab.py --out /tmp/up1.pt
    python tools/probe/upconv_premod_ab.py --compare /tmp/up0.pt /tmp/up1.pt
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

# (N, R input, Cin, Cout): the 256² generator's up-convs at 128 images, the 1024² one's at 32
SHAPES = [(128, 128, 256, 128), (128, 64, 512, 256), (128, 32, 512, 512), (128, 16, 512, 512),
          (32, 256, 128, 64), (32, 512, 64, 32)]


def run(out, dtypes):
    dev = torch.device("cuda:0")
    res = {}
    for dtype in dtypes:
        for N, R, cin, cout in SHAPES:
            g = torch.Generator().manual_seed(R + cin)
            x = torch.randn(N, R, R, cin, generator=g).to(dtype).to(dev)
            w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
            wph = [m.to(dev) for m in layouts.upconv_subpixel_matrices(w, dtype)]
            wup = layouts.upconv_halo_matrix(w, dtype).to(dev)
            s = (torch.rand(N, cin, generator=g) + 0.5).to(dev)
            t = torch.empty(N, 2 * R + 1, 2 * R + 1, cout, dtype=dtype, device=dev)
            for _ in range(2):
                ops.upconv_fwd(x, wph, t, cout, style=s, w_up=wup)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.upconv_fwd(x, wph, t, cout, style=s, w_up=wup)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 10 * 1e3
            tf = 2 * N * R * R * 9 * cin * cout / (us * 1e-6) / 1e12
            key = f"{str(dtype)[6:]} N{N} R{R} {cin}->{cout}"
            print(f"{key:32s} {us:9.1f} us/call {tf:7.1f} TFLOP/s", flush=True)
            res[key] = t.cpu()
    torch.save(res, out)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    for k in A:
        nd = int((A[k] != B[k]).sum())
        print(f"{k:32s} {'bit-identical' if nd == 0 else f'{nd} values differ'}")
        assert nd == 0, k


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--dtypes", default="fp16,bf16", help="comma list of fp32, fp16, bf16")
    a = ap.parse_args()
    if a.compare:
        compare(*a.compare)
    else:
        DT = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
        run(a.out, [DT[d] for d in a.dtypes.split(",")])
