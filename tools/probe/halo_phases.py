"""Block phases of the fp16 / bf16 halo kernel (conv_halo.hip) on the StyledConv forward shapes
(diagnostic build only: make -C …/csrc variant VARIANT=htime
VARIANT_FLAGS="-DMIA_HALO_TIMING -DMIA_HALO_TIMING_COARSE"; run with MIA_LIB_VARIANT=htime).
Prints, per shape, wave 0's cycles per block in prologue (first halo + weight stages landed),
main loop, epilogue and the final store drain, and the loop's share of the block. Tuning aid."""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import _lib, layouts, ops  # noqa: E402

SHAPES = [(128, 256, 128), (128, 128, 256), (128, 64, 512)]


def main():
    lib = _lib.load()
    fn = lib.mia_debug_halo_timing
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = (ctypes.c_ulonglong * 8)()
    dev = torch.device("cuda:0")
    for dtype in (torch.float16,):
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
            wmod = torch.empty((N,) + tuple(wm.shape), dtype=dtype, device=dev)
            for mode in ("mod", "wmod", "plain"):
                kw = dict(in_scale=s, out_scale=d, noise=nz, noise_w=0.3, bias=b,
                          act_out=ops.ACT_LRELU_S2) if mode != "plain" else {}

                def call():
                    if mode == "wmod":  # per-image modulated weights (round 4)
                        ops.conv3x3_modw(x, wm, y, wmod, cout=C, **kw)
                    else:
                        ops.conv3x3(x, wm, y, cout=C, **kw)
                call()
                torch.cuda.synchronize()
                fn(out, 1)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    call()
                e1.record()
                torch.cuda.synchronize()
                fn(out, 1)
                blocks = max(out[5], 1)
                pro, loop, epi, drain = out[0] / blocks, out[6] / blocks, out[4] / blocks, \
                    out[7] / blocks
                tot = pro + loop + epi + drain
                us = e0.elapsed_time(e1) / 3 * 1e3
                print(f"{str(dtype)[6:]} {mode:5s} N{N} {H}² {C}->{C}: {us:8.1f} us  "
                      f"{2 * N * H * H * 9 * C * C / us / 1e6:7.1f} TF/s | per block (cycles, "
                      f"wave 0): prologue {pro:7.0f} loop {loop:7.0f} epilogue {epi:6.0f} "
                      f"drain {drain:6.0f}  loop {loop / tot:.2f}", flush=True)


if __name__ == "__main__":
    main()
