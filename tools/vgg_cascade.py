"""The VGG16 cascade of the attack objective on its own (code/vgg.py:44-64 forward + the tap-MSE
input gradient of one objective call, vgg.VGGNet.backward), for per-layer rocprofv3 evidence.

    python tools/vgg_cascade.py [--dtype fp32] [--batch 128] [--reps 3]

One rep = 25 library calls on one stream, in this order (the labels tools/vgg_layers_summary.py
assigns to the rep's kernel dispatches): forward conv1_1 conv1_2 pool1 conv2_1 conv2_2 pool2
conv3_1 conv3_2 conv3_3 pool3 conv4_1 conv4_2; backward tap4_2 dconv4_2 dconv4_1 dpool3 dconv3_3
dconv3_2 dconv3_1 dpool2 dconv2_2 dconv2_1 dpool1 dconv1_2 dconv1_1."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gfa_import  # noqa: E402,F401
from gfa_amd.vgg import CPAD, VGGNet  # noqa: E402
from gfa_amd.weights import make_vgg_weights  # noqa: E402
from gfa_amd.workspace import Workspace  # noqa: E402

LABELS = ("conv1_1 conv1_2 pool1 conv2_1 conv2_2 pool2 conv3_1 conv3_2 conv3_3 pool3 conv4_1 "
          "conv4_2 tap4_2 dconv4_2 dconv4_1 dpool3 dconv3_3 dconv3_2 dconv3_1 dpool2 dconv2_2 "
          "dconv2_1 dpool1 dconv1_2 dconv1_1").split()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp16", "bf16"])
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    T = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[a.dtype]
    dev = torch.device("cuda:0")
    net = VGGNet(make_vgg_weights(1234), dtype=T, device=dev)
    ws = Workspace(dev)
    N, R = a.batch, 256
    g = torch.Generator().manual_seed(5)
    x = torch.zeros(N, R, R, CPAD, dtype=T)
    x[..., :3] = (torch.rand(N, R, R, 3, generator=g) * 2 - 1).to(T)
    t = torch.zeros_like(x)
    t[..., :3] = (torch.rand(N, R, R, 3, generator=g) * 2 - 1).to(T)
    x, t = x.to(dev), t.to(dev)
    taps_t = [v.clone() for v in VGGNet.taps(net.forward(t, ws, "t"))]
    coefs = [2.0 / v[0].numel() for v in taps_t]
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
    for r in range(a.reps):
        ev[2 * r].record()
        act = net.forward(x, ws, "x")
        net.backward(act, taps_t, coefs, ws, "x")
        ev[2 * r + 1].record()
    torch.cuda.synchronize()
    fl = 2 * net.flops_fwd_per_image * N
    for r in range(a.reps):
        ms = ev[2 * r].elapsed_time(ev[2 * r + 1])
        print(f"rep {r}: {ms:.2f} ms fwd+dgrad, {fl / (ms * 1e-3) / 1e12:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
