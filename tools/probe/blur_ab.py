"""Up-conv Blur forward / adjoint timing at the bench's generator shapes (tuning aid; GPU only).

    MIA_LIB_VARIANT=<lib> python tools/probe/blur_ab.py [--dtype fp16] [--batch 128]

For each up-sampling StyledConv of the 256² generator (R = 4 … 128, its Cout) times
mia_upconv_blur_fwd (demod + noise + bias + lrelu·√2) and mia_upconv_blur_bwd with HIP events
over 20 calls each; prints µs per call and the algorithmic HBM rate (input once + output once)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "fp32"])
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    T = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype]
    dev = torch.device("cuda:0")
    N = a.batch
    tot_f = tot_b = 0.0
    for R, C in ((128, 128), (64, 256), (32, 512), (16, 512), (8, 512), (4, 512)):
        S = 2 * R + 1
        t = torch.randn(N, S, S, C, device=dev).to(T)
        out = torch.empty(N, 2 * R, 2 * R, C, dtype=T, device=dev)
        gt = torch.empty_like(t)
        dm = torch.rand(N, C, device=dev) + 0.5
        nz = torch.randn(4 * R * R, device=dev)
        bs = torch.randn(C, device=dev) * 0.1
        res = []
        for fwd in (True, False):
            def call():
                if fwd:
                    ops.upconv_blur_fwd(t, out, dm, nz, 0.1, bs, act_out=ops.ACT_LRELU_S2)
                else:
                    ops.upconv_blur_bwd(out, gt)
            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            nbytes = (t.numel() + out.numel()) * t.element_size()
            res.append((us, nbytes / us / 1e6))
        tot_f += res[0][0]
        tot_b += res[1][0]
        print(f"R={R:3d} C={C:3d}: fwd {res[0][0]:8.1f} us {res[0][1]:6.2f} TB/s | "
              f"bwd {res[1][0]:8.1f} us {res[1][1]:6.2f} TB/s", flush=True)
    print(f"per generator forward: fwd {tot_f:.1f} us, bwd {tot_b:.1f} us "
          f"(x20 per PGD-20 step: {tot_f * 20 / 1e3:.1f} + {tot_b * 20 / 1e3:.1f} ms)")


if __name__ == "__main__":
    main()
