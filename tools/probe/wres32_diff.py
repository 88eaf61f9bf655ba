"""Where conv_wres32 and conv_thin32 outputs differ (tuning aid, not product): per mode, the
number of differing elements and their pixel / channel pattern."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd import _lib, layouts, ops  # noqa: E402

dev = torch.device("cuda:0")
for dtype in (torch.float16, torch.bfloat16):
    for mode in ("plain", "mod_nos", "mod"):
        N, C, H, W = 2, 32, 32, 48
        g = torch.Generator().manual_seed(5)
        x = torch.randn(N, H, W, C, generator=g).to(dtype).to(dev)
        w = torch.randn(C, C, 3, 3, generator=g) / math.sqrt(9 * C)
        wm = layouts.fwd_matrix(w, dtype).to(dev)
        s = (torch.rand(N, C, generator=g) + 0.5).to(dev)
        d = (torch.rand(N, C, generator=g) + 0.5).to(dev)
        b = (torch.randn(C, generator=g) * 0.1).to(dev)
        nz = torch.randn(H * W, generator=g).to(dev)
        outs = []
        for v in (1, 0):
            _lib.set_tuning("MIA_CONV_WRES32", v)
            y = torch.zeros(N, H, W, C, dtype=dtype, device=dev)
            kw = {}
            if mode == "mod":
                kw = dict(in_scale=s, out_scale=d, noise=nz, noise_w=0.3, bias=b,
                          act_out=ops.ACT_LRELU_S2)
            elif mode == "mod_nos":  # modulated input, plain epilogue (generic-epilogue launch)
                kw = dict(in_scale=s, out_scale=d)
            try:
                ops.conv3x3(x, wm, y, cout=C, **kw)
            except Exception as e:  # no specialisation for this mask
                print(dtype, mode, "skip:", e)
                break
            torch.cuda.synchronize()
            outs.append(y.float().cpu())
        if len(outs) < 2:
            continue
        dif = (outs[0] != outs[1])
        idx = dif.nonzero()
        print(f"{str(dtype)[6:]} {mode}: {dif.sum().item()} / {dif.numel()} differ, max "
              f"{(outs[0] - outs[1]).abs().max().item():.3g}", flush=True)
        if len(idx):
            print("  n", idx[:, 0].unique().tolist()[:8], "y", idx[:, 1].unique().tolist()[:16],
                  "x", idx[:, 2].unique().tolist()[:16], "c", idx[:, 3].unique().tolist()[:32])
_lib.set_tuning("MIA_CONV_WRES32", 1)
