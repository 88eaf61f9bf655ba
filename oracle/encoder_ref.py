"""CPU oracle: synthetic linear encoder (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Stand-in for e4e behind ``net.encoder``: E(x) = W_E·vec(avgpool(x)) /
sqrt(768) + b_E → (N, n_latent, 512), where avgpool reduces a 256² image to 16². Parity unpinned
(the build's own definition; the real IR-SE50 e4e is a "next" row).
"""
import math

import torch.nn.functional as F


def encode(e, x):
    n, _, h, _ = x.shape
    v = F.avg_pool2d(x, h // 16).reshape(n, -1)
    w = e["enc.weight"].to(x.dtype)
    lat = F.linear(v, w * (1.0 / math.sqrt(w.shape[1])), e["enc.bias"].to(x.dtype))
    return lat.view(n, -1, 512)
