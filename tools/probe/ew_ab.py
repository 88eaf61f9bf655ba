"""Timing of the e4e elementwise kernels (SE apply, SE gradient scale, PReLU gradient scale) at
the IR-SE50 stage shapes of the 128 × 256² bench batch (GPU, tuning aid; MIA_LIB_VARIANT selects
a variant library). Prints µs per call and the algorithmic GB/s."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
N = 128
for dtype in (torch.float32, torch.float16):
    es = torch.tensor([], dtype=dtype).element_size()
    for H, C in ((128, 64), (64, 128), (32, 256), (16, 512)):
        g = torch.Generator(device=dev).manual_seed(0)
        r = torch.randn(N, H, H, C, device=dev, generator=g).to(dtype)
        sc = torch.randn(N, H, H, C, device=dev, generator=g).to(dtype)
        a = torch.randn(N, H, H, C, device=dev, generator=g).to(dtype)
        s = torch.rand(N, C, device=dev, generator=g)
        gv, bv = torch.rand(C, device=dev, generator=g), torch.rand(C, device=dev, generator=g)
        out, xb = torch.empty_like(r), torch.empty_like(r)
        nb = r.numel() * es
        cases = (("se_apply out+xb", lambda: ops.se_apply(r, s, sc, 1, out, gv, bv, xb), 4 * nb),
                 ("se_grad_scale", lambda: ops.se_grad_scale(r, s, s, out, gamma=gv), 2 * nb),
                 ("prelu_bwd_scale", lambda: ops.prelu_bwd_scale(r, a, gv, out, gamma=bv), 3 * nb))
        for name, fn, traffic in cases:
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(f"{str(dtype)[6:]:8s} {H:4d}^2 x {C:4d} {name:16s} {ms * 1e3:8.1f} us "
                  f"{traffic / ms / 1e6:7.0f} GB/s  chk {float(out.float().sum()):.6e}", flush=True)
