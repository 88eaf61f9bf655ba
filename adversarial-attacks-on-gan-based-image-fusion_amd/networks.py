"""Reference-shaped module objects around the device networks.

* ``Decoder``  — ``net.decoder``: ``decoder([w+], input_is_latent=True, randomize_noise=False,
  return_latents=True) -> (img, latents)`` and ``.size`` (code/attack/attack_main2.py:590,619-621).
* ``Encoder``  — ``net.encoder(x) -> (N, n_latent, 512)`` (attack_main2.py:597,622).
* ``PSPNet``   — the pSp bundle: encoder, decoder, latent_avg, opts.start_from_latent_avg
  (attack_main2.py:137-146; utils/model_utils.py:7-18).
* ``VGGBase`` / ``vgg16(pth)`` — code/vgg.py:6-81: ``vgg(x) -> (conv1_1, conv1_2, conv3_2, conv4_2)``.
* ``get_latents(net, x)`` — attack_main2.py:137-146 (adds latent_avg when the option is set).
* ``MappingNet`` — the rosinality mapping MLP (z → w) behind the fusion entry point
  (style_fusion_simple.py:110-119, mean_latent at :58).

Forward calls here allocate their outputs and return NCHW fp32 tensors (reference layout); the
attack itself works on the NHWC device buffers directly.
"""
import argparse
import math

import torch

from .e4e import E4EEncoder
from .encoder import SyntheticEncoder
from .stylegan2 import SynthesisNet
from .vgg import CPAD, VGGNet
from .weights import (LR_MLP, N_MLP, STYLE_DIM, make_e4e_weights, make_encoder_weights,
                      make_generator_weights,
                      make_vgg_weights)
from .workspace import Workspace
from . import ops


class MappingNet:
    """rosinality Generator.style on device: PixelNorm, then N_MLP × EqualLinear(512, 512,
    lr_mul=0.01, fused_lrelu) = GEMM (mia_gemm_f32) + lrelu(·+b·lr_mul)·√2 (mia_bias_act_fwd)."""

    def __init__(self, params, device="cuda"):
        dev = torch.device(device)
        self.device = dev
        scale = LR_MLP / math.sqrt(STYLE_DIM)
        self.w = [(params[f"style.{i}.weight"].double() * scale).float().contiguous().to(dev)
                  for i in range(1, N_MLP + 1)]
        self.b = [(params[f"style.{i}.bias"].double() * LR_MLP).float().contiguous().to(dev)
                  for i in range(1, N_MLP + 1)]
        self._ws = Workspace(dev)

    def __call__(self, z):
        """z: (N, 512) → w: (N, 512) fp32 (a new tensor)."""
        z = z.to(self.device, torch.float32).contiguous()
        N = z.shape[0]
        if tuple(z.shape) != (N, STYLE_DIM):
            raise ValueError("z must be (N, 512)")
        a = self._ws.get("map.a", (N, STYLE_DIM), torch.float32)
        b = self._ws.get("map.b", (N, STYLE_DIM), torch.float32)
        ops.pixel_norm(z, a)
        for w, bias in zip(self.w, self.b):
            # y = a·Wᵀ: B[k][n] = W[n][k]
            ops.gemm(N, STYLE_DIM, STYLE_DIM, 1.0, a, STYLE_DIM, 1, w, 1, STYLE_DIM, 0.0, b,
                     STYLE_DIM, 1)
            ops.bias_act_fwd(b.view(N, 1, 1, STYLE_DIM), None, 0.0, bias,
                             a.view(N, 1, 1, STYLE_DIM))
        return a.clone()

    def mean_latent(self, n_latent=4096, seed=0):
        """Generator.mean_latent: the mean of n_latent mapped z ~ N(0, I) (host-seeded draws;
        the mean is a ones-vector GEMM)."""
        g = torch.Generator().manual_seed(int(seed))
        z = torch.randn(n_latent, STYLE_DIM, generator=g)
        w = self(z)
        ones = self._ws.get("map.ones", (1, n_latent), torch.float32)
        ones.fill_(1.0)
        mean = torch.empty(1, STYLE_DIM, device=self.device)
        ops.gemm(1, STYLE_DIM, n_latent, 1.0 / n_latent, ones, n_latent, 1, w, STYLE_DIM, 1, 0.0,
                 mean, STYLE_DIM, 1)
        return mean


class Decoder:
    def __init__(self, params, size, dtype=torch.float32, device="cuda"):
        self.impl = SynthesisNet(params, size, dtype=dtype, device=device)
        self.size = self.impl.size
        self.n_latent = self.impl.n_latent
        self.device = self.impl.device
        self._ws = Workspace(self.device)
        self.mapping = MappingNet(params, device) if "style.1.weight" in params else None

    def _truncate(self, lat, truncation, truncation_latent):
        if truncation == 1:
            return lat
        if truncation_latent is None:
            raise ValueError("truncation != 1 needs truncation_latent")
        mean = truncation_latent.to(self.device, torch.float32).reshape(-1).contiguous()
        out = torch.empty_like(lat)
        return ops.truncate(lat, mean, float(truncation), out)

    def __call__(self, styles, input_is_latent=True, randomize_noise=False, return_latents=False,
                 truncation=1, truncation_latent=None):
        """rosinality Generator.forward subset: [w] or [w+] with input_is_latent=True
        (attack_main2.py:619-621), or [z] through the mapping MLP; truncation toward
        truncation_latent; fixed noise only."""
        if randomize_noise:
            raise ValueError("randomize_noise=False only (fixed noise buffers, attack_main2.py:620)")
        lat = styles[0] if isinstance(styles, (list, tuple)) else styles
        lat = lat.to(self.device, torch.float32).contiguous()
        if not input_is_latent:
            if self.mapping is None:
                raise ValueError("z input needs the mapping MLP weights (style.{1..8}.*)")
            if lat.dim() != 2:
                raise ValueError("z must be (N, 512)")
            lat = self.mapping(lat)
        lat = self._truncate(lat, truncation, truncation_latent)
        if lat.dim() == 2:
            lat = lat.unsqueeze(1).repeat(1, self.n_latent, 1)
        lat = lat.contiguous()
        img = self.impl.forward(lat, self._ws).clone()
        return img, (lat if return_latents else None)


class Encoder:
    """``net.encoder``: e4e ``Encoder4Editing(50, 'ir_se')`` (params from make_e4e_weights or an
    e4e checkpoint's ``encoder.*`` state dict + ``latent_avg``) or the linear stand-in."""

    def __init__(self, params, size, device="cuda", dtype=torch.float32):
        if params.get("kind") == "e4e":
            self.impl = E4EEncoder(params, size, dtype=dtype, device=device)
        else:
            self.impl = SyntheticEncoder(params, size, device=device)
        self._ws = Workspace(torch.device(device))

    def __call__(self, x):
        x = x.to(self.impl.latent_avg.device, torch.float32).contiguous()
        return self.impl.forward(x, self._ws).clone()


class PSPNet:
    def __init__(self, encoder, decoder, latent_avg, start_from_latent_avg=True):
        self.encoder = encoder
        self.decoder = decoder
        self.latent_avg = latent_avg
        self.opts = argparse.Namespace(start_from_latent_avg=start_from_latent_avg)
        self.vgg = None
        self.default_target = None

    def eval(self):
        return self


class VGGBase:
    """code/vgg.py VGGBase: forward returns the four taps (NCHW fp32)."""

    def __init__(self, pth, dtype=torch.float32, device="cuda"):
        self.pth = pth
        self.impl = VGGNet(pth, dtype=dtype, device=device)
        self._ws = Workspace(torch.device(device))

    def __call__(self, image):
        x = image.to(self.impl.device, torch.float32).contiguous()
        N, _, H, W = x.shape
        if H != W:
            raise ValueError("square images only")
        xin = self._ws.get("in", (N, H, W, CPAD), self.impl.dtype)
        ops.image_to_nhwc(x, xin, 1, CPAD)
        a = self.impl.forward(xin, self._ws, "")
        return tuple(t.permute(0, 3, 1, 2).float().contiguous() for t in VGGNet.taps(a))

    def eval(self):
        return self


def vgg16(pth, dtype=torch.float32, device="cuda"):
    return VGGBase(pth, dtype=dtype, device=device)


def get_latents(net, x, is_cars=False):
    """attack_main2.py:137-146."""
    codes = net.encoder(x)
    if net.opts.start_from_latent_avg:
        codes = codes + net.latent_avg.to(codes.device).unsqueeze(0)
    if codes.shape[1] == 18 and is_cars:
        codes = codes[:, :16, :]
    return codes


def build_net(size=256, seed=0, dtype=torch.float32, device="cuda", vgg_seed=1234,
              with_vgg=True, encoder="linear"):
    """Seeded synthetic pSp bundle (+ VGG) — no checkpoints exist offline.
    ``encoder``: "e4e" (IR-SE50 Encoder4Editing, the reference's encoder) or "linear" (the
    SURVEY.md §7 stand-in)."""
    gp = make_generator_weights(size, seed=seed)
    if encoder == "e4e":
        ep = make_e4e_weights(size, seed=seed + 1)
    elif encoder == "linear":
        ep = make_encoder_weights(size, seed=seed + 1)
    else:
        raise ValueError("encoder: 'e4e' or 'linear'")
    net = PSPNet(Encoder(ep, size, device=device, dtype=dtype),
                 Decoder(gp, size, dtype=dtype, device=device),
                 ep["latent_avg"].to(device), ep["start_from_latent_avg"])
    net.params = dict(generator=gp, encoder=ep)
    if with_vgg:
        vs = make_vgg_weights(vgg_seed)
        net.vgg = VGGBase(vs, dtype=dtype, device=device)
        net.params["vgg"] = vs
    return net


def psp_params_from_checkpoint(ckpt):
    """Generator and e4e encoder parameter dicts from a pSp / e4e checkpoint (a path or an already
    loaded dict), as ``utils/model_utils.py:7-35`` + pSp.load_weights split it: ``state_dict``
    keys ``encoder.*`` / ``decoder.*``, ``latent_avg``, ``opts``. Loaded with
    ``torch.load(weights_only=True)`` (nothing in the file is executed)."""
    if not isinstance(ckpt, dict):
        ckpt = torch.load(ckpt, map_location="cpu", weights_only=True)
    sd = ckpt["state_dict"]
    enc = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    dec = {k[len("decoder."):]: v for k, v in sd.items() if k.startswith("decoder.")}
    if not enc or not dec:
        raise ValueError("checkpoint state_dict needs encoder.* and decoder.* keys")
    opts = ckpt.get("opts", {}) or {}
    enc["latent_avg"] = ckpt["latent_avg"].reshape(-1, STYLE_DIM).float()
    enc["start_from_latent_avg"] = bool(opts.get("start_from_latent_avg", True))
    enc["kind"] = "e4e"
    return dec, enc, opts


def build_net_from_checkpoint(ckpt, size=None, dtype=torch.float32, device="cuda", vgg=None):
    """``setup_model(checkpoint_path)`` (utils/model_utils.py:7-18) on the device kernels: the
    e4e encoder + StyleGAN2 decoder of one checkpoint (+ an optional VGG state dict)."""
    dec, enc, opts = psp_params_from_checkpoint(ckpt)
    size = int(size or opts.get("stylegan_size", 1024))
    net = PSPNet(Encoder(enc, size, device=device, dtype=dtype),
                 Decoder(dec, size, dtype=dtype, device=device),
                 enc["latent_avg"].to(device), enc["start_from_latent_avg"])
    if vgg is not None:
        net.vgg = VGGBase(vgg, dtype=dtype, device=device)
    return net
