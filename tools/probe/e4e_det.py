"""Determinism probe of the e4e input gradient (fp32, 256², N=1): two backward passes on the same
forward, and per-switch differences."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
import gfa_import  # noqa
from gfa_amd import e4e
from gfa_amd.weights import make_e4e_weights
from gfa_amd.workspace import Workspace
dev = torch.device("cuda:0")
enc = e4e.E4EEncoder(make_e4e_weights(256, seed=1), 256, dtype=torch.float32, device=dev)
g = torch.Generator().manual_seed(0)
xin = torch.zeros(1, 256, 256, 8)
xin[..., :3] = torch.rand(1, 256, 256, 3, generator=g) * 2 - 1
xin = xin.to(dev)
ws = Workspace(dev)
enc.forward_nhwc(xin, ws)
gl = (torch.randn(1, 14, 512, generator=g)).to(dev)
outs = []
for r in range(4):
    gx = torch.zeros_like(xin)
    enc.debug = {}
    enc.backward_nhwc(gl, ws, gx)
    torch.cuda.synchronize()
    outs.append((gx.clone(), {k: v.clone() for k, v in enc.debug.items()}))
    enc.debug = None
ref = outs[0]
for r in range(1, 4):
    d = (outs[r][0] - ref[0]).abs().max().item()
    keys = [k for k in ref[1] if not torch.equal(ref[1][k], outs[r][1][k])]
    print("run", r, "max|Δgx|", d, "rel", d / ref[0].abs().max().item(), "differing debug:", keys[:8])
# forward determinism: activations and latents of two forwards on the same input
def snap():
    lat = enc.forward_nhwc(xin, ws).clone()
    torch.cuda.synchronize()
    acts = {"a0": enc._a0.clone()}
    for i, U in enumerate(enc.units):
        acts[f"a1_{i}"] = U["_a1"].clone()
        acts[f"r_{i}"] = U["_r"].clone()
        acts[f"u_{i}"] = U["_u"].clone()
    for i, hd in enumerate(enc.heads):
        for j, a in enumerate(hd["_acts"]):
            acts[f"h{i}_{j}"] = a.clone()
    return lat, acts
l0, a0 = snap()
for r in range(3):
    l1, a1 = snap()
    diff = [k for k in a0 if not torch.equal(a0[k], a1[k])]
    flips = sum(int(((a0[k] > 0) != (a1[k] > 0)).sum()) for k in a0)
    print("fwd run", r, "lat max|Δ|", (l1 - l0).abs().max().item(), "differing", len(diff), diff[:6],
          "sign flips", flips)
