import sys, os, math
sys.path.insert(0, os.getcwd())
import torch
import gfa_import  # noqa
from gfa_amd import ops, layouts, e4e
dev = torch.device("cuda:0")
C, N, H, S, dtype = 64, 2, 8, 3, torch.float32
ho = (H - 1) // 2 + 1
g = torch.Generator().manual_seed(0)
ws = [torch.randn(C, C, 3, 3, generator=g, dtype=torch.float64) * 0.05 for _ in range(S)]
gy = torch.randn(S * N, ho, ho, C, generator=g).to(dev)
def run(perm_in, perm_out, ph=3, kind="dgrad"):
    b = torch.full((S * N, H, H, C), float("nan"), device=dev)
    grp = []
    for k in range(S):
        pg = e4e._phase_groups([layouts.s2_dgrad_phases(ws[k], dtype)[ph]], H)[0]
        pg = dict(pg, w=pg["w"].to(dev))
        grp.append(dict(pg, n_in=perm_in[k] * N, n_out=perm_out[k] * N, c_off=k * C))
    ops.conv2d_batched(gy, grp, b, (H, H), n=N, cout=C)
    torch.cuda.synchronize()
    res = []
    for k in range(S):
        o = perm_out[k] * N
        v = b[o:o + N][:, 1::2, 1::2]
        res.append((round(v.abs().max().item(), 3), bool(torch.isnan(v).any())))
    return res
print("id/id", run([0, 1, 2], [0, 1, 2]))
print("perm/id", run([2, 1, 0], [0, 1, 2]))
print("id/perm", run([0, 1, 2], [2, 1, 0]))
print("ph0 id/id", run([0, 1, 2], [0, 1, 2], ph=0))
# single group, n_in = 2N
b = torch.full((S * N, H, H, C), float("nan"), device=dev)
pg = e4e._phase_groups([layouts.s2_dgrad_phases(ws[0], dtype)[3]], H)[0]
pg = dict(pg, w=pg["w"].to(dev))
ops.conv2d_batched(gy, [dict(pg, n_in=2 * N, n_out=0, c_off=0)], b, (H, H), n=N, cout=C)
a = torch.full((N, H, H, C), float("nan"), device=dev)
ops.conv2d(gy[2 * N:3 * N].contiguous(), [pg], a, (H, H), cout=C)
torch.cuda.synchronize()
print("single n_in=2N", b[:N, 1::2, 1::2].abs().max().item(), a[:, 1::2, 1::2].abs().max().item(),
      (b[:N, 1::2, 1::2] - a[:, 1::2, 1::2]).abs().max().item())
# same with pad-1 3x3 stride 1
kp = ops.conv2d_kpad(9, C, dtype)
wm = torch.zeros(C, kp); wm[:, :9 * C] = ws[0].permute(0, 2, 3, 1).reshape(C, 9 * C)
g3 = dict(w=wm.to(dev), kh=3, kw=3, pad=(1, 1), ho=ho, wo=ho)
b2 = torch.full((S * N, ho, ho, C), float("nan"), device=dev)
a2 = torch.full((N, ho, ho, C), float("nan"), device=dev)
ops.conv2d_batched(gy, [dict(g3, n_in=2 * N, n_out=0, c_off=0)], b2, (ho, ho), n=N, cout=C)
ops.conv2d(gy[2 * N:3 * N].contiguous(), [g3], a2, (ho, ho), cout=C)
torch.cuda.synchronize()
print("3x3 s1 n_in=2N", b2[:N].abs().max().item(), a2.abs().max().item(), (b2[:N] - a2).abs().max().item())
