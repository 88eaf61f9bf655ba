"""Synthetic linear encoder behind the reference's ``net.encoder`` slot.

The reference calls e4e (``Encoder4Editing(50, 'ir_se')``, un-vendored; loader
``code/utils/model_utils.py:7-35``) as ``net.encoder(x) -> (N, n_latent, 512)``
(``code/attack/attack_main2.py:597,622``). Offline there is no checkpoint, so the build uses a
deterministic linear stand-in: E(x) = W_E·vec(avgpool16(x'))/√768 + b_E.
The real IR-SE50 encoder is SURVEY.md §8f row 1.
"""
import math

import torch

from . import ops
from .weights import ENC_POOL_RES, STYLE_DIM, n_latent_for


class SyntheticEncoder:
    def __init__(self, e, size, device="cuda"):
        self.size = int(size)
        self.n_latent = n_latent_for(self.size)
        dev = torch.device(device)
        w = e["enc.weight"].double() / math.sqrt(e["enc.weight"].shape[1])
        self.w = w.float().contiguous().to(dev)  # (n_latent*512, 768)
        self.b = e["enc.bias"].float().contiguous().to(dev)
        self.latent_avg = e["latent_avg"].float().to(dev)
        self.d_in = 3 * ENC_POOL_RES * ENC_POOL_RES

    def forward(self, x, ws, tag="e"):
        """x: (N,3,S,S) fp32 (full resolution; the reference's avg_pool2d(·, S/256) then this
        encoder's 16² pooling compose into one S/16 pooling). Returns (N, n_latent, 512) fp32."""
        N = x.shape[0]
        v = ws.get(f"{tag}.v", (N, 3, ENC_POOL_RES, ENC_POOL_RES), torch.float32)
        if x.shape[-1] % ENC_POOL_RES or x.shape[-1] != x.shape[-2]:
            raise ValueError("encoder input must be square with side a multiple of 16")
        ops.avgpool_fwd(x, v, x.shape[-1] // ENC_POOL_RES)
        lat = ws.get(f"{tag}.lat", (N, self.n_latent, STYLE_DIM), torch.float32)
        D = self.n_latent * STYLE_DIM
        ops.gemm(N, D, self.d_in, 1.0, v, self.d_in, 1, self.w, 1, self.d_in, 0.0, lat, D, 1,
                 bias=self.b)
        return lat

    def backward(self, g_lat, ws, tag="e"):
        """∂L/∂v (N,3,16,16) from ∂L/∂lat; the caller spreads it over the pooled pixels."""
        N = g_lat.shape[0]
        D = self.n_latent * STYLE_DIM
        gv = ws.get(f"{tag}.gv", (N, 3, ENC_POOL_RES, ENC_POOL_RES), torch.float32)
        ops.gemm(N, self.d_in, D, 1.0, g_lat, D, 1, self.w, self.d_in, 1, 0.0, gv, self.d_in, 1)
        return gv

    def __call__(self, x):
        """Reference-shaped call ``net.encoder(x)`` (returns a fresh tensor)."""
        from .workspace import Workspace
        ws = Workspace(x.device)
        return self.forward(x.float().contiguous(), ws).clone()
