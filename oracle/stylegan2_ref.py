"""CPU oracle: StyleGAN2 synthesis (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

**Parity unpinned.** The reference calls an un-vendored rosinality-style generator
(``net.decoder([w+], input_is_latent=True, randomize_noise=False, return_latents=True)``,
``code/attack/attack_main2.py:619-621``; ``SFGenerator_hook`` at ``code/style_fusion_simple.py:51``).
This module restates that published algorithm in the reference's own per-sample formulation
(per-sample modulated weights + grouped conv / grouped transposed conv + FIR blur), which is
structurally different from the product's factorised kernels, so agreement is meaningful:

* ModulatedConv2d: w = (1/sqrt(Cin k²)) · W · s[n,ci]; demod = rsqrt(Σ w² + 1e-8); grouped conv,
  or for ``upsample``: grouped conv_transpose2d(stride 2) then Blur = upfirdn2d(k=[1,3,3,1]⊗[1,3,3,1]
  normalised × 4, pad (1,1)).
* style s = EqualLinear(w) = w · (A/sqrt(512))ᵀ + b_A.
* StyledConv = ModulatedConv2d → NoiseInjection (x + strength·noise) → FusedLeakyReLU
  (leaky_relu(x + b, 0.2)·sqrt 2).
* ToRGB = 1×1 modulated conv without demod + bias + upfirdn2d(skip, up=2, pad (2,1)).
"""
import math

import torch
import torch.nn.functional as F

from . import forcing

BLUR_1D = [1.0, 3.0, 3.0, 1.0]


def make_kernel(k1d, dtype=torch.float32):
    k = torch.tensor(k1d, dtype=dtype)
    k = k[None, :] * k[:, None]
    return k / k.sum()


def upfirdn2d(x, kernel, up=1, down=1, pad=(0, 0)):
    """Zero-insert upsample by ``up``, pad (pad0, pad1) on both axes, correlate with the flipped
    kernel, then keep every ``down``-th sample (rosinality op/upfirdn2d native semantics)."""
    n, c, h, w = x.shape
    kh, kw = kernel.shape
    p0, p1 = pad
    out = x.reshape(n * c, 1, h, w)
    if up > 1:
        z = out.new_zeros(n * c, 1, h * up, w * up)
        z[:, :, ::up, ::up] = out
        out = z
    out = F.pad(out, [max(p0, 0), max(p1, 0), max(p0, 0), max(p1, 0)])
    if p0 < 0 or p1 < 0:
        hh, ww = out.shape[2], out.shape[3]
        out = out[:, :, max(-p0, 0):hh - max(-p1, 0), max(-p0, 0):ww - max(-p1, 0)]
    wk = torch.flip(kernel, [0, 1]).to(out.dtype).view(1, 1, kh, kw)
    out = F.conv2d(out, wk)
    out = out[:, :, ::down, ::down]
    return out.reshape(n, c, out.shape[2], out.shape[3])


def style_affine(p, prefix, w):
    a = p[prefix + ".modulation.weight"].to(w.dtype)
    b = p[prefix + ".modulation.bias"].to(w.dtype)
    return F.linear(w, a * (1.0 / math.sqrt(a.shape[1])), b)


def modulated_conv2d(p, prefix, x, w, demodulate=True, upsample=False, s=None):
    """``s``: the layer's style vector given directly (style_vector path), else A·w + b."""
    weight = p[prefix + ".weight"].to(x.dtype)  # (1, out, in, k, k)
    _, cout, cin, k, _ = weight.shape
    n = x.shape[0]
    style = (style_affine(p, prefix, w) if s is None else s.to(x.dtype)).view(n, 1, cin, 1, 1)
    scale = 1.0 / math.sqrt(cin * k * k)
    wt = scale * weight * style
    if demodulate:
        demod = torch.rsqrt(wt.pow(2).sum([2, 3, 4]) + 1e-8)
        wt = wt * demod.view(n, cout, 1, 1, 1)
    h, ww = x.shape[2], x.shape[3]
    if upsample:
        xin = x.reshape(1, n * cin, h, ww)
        wt = wt.view(n, cout, cin, k, k).transpose(1, 2).reshape(n * cin, cout, k, k)
        out = F.conv_transpose2d(xin, wt, padding=0, stride=2, groups=n)
        out = out.view(n, cout, out.shape[2], out.shape[3])
        blur = make_kernel(BLUR_1D, x.dtype) * 4.0  # upsample_factor ** 2
        out = upfirdn2d(out, blur, pad=(1, 1))
    else:
        xin = x.reshape(1, n * cin, h, ww)
        out = F.conv2d(xin, wt.view(n * cout, cin, k, k), padding=k // 2, groups=n)
        out = out.view(n, cout, out.shape[2], out.shape[3])
    return out


# Teacher-forced LeakyReLU branches (tests only): {styled-conv prefix: bool tensor (NCHW)}, the
# device run's positive set per layer (see vgg_ref.forced_masks).
_FORCED = None


class forced_masks:
    def __init__(self, masks):
        self.masks = masks

    def __enter__(self):
        global _FORCED
        _FORCED = self.masks
        return self

    def __exit__(self, *exc):
        global _FORCED
        _FORCED = None


def styled_conv(p, prefix, x, w, noise, upsample=False, s=None):
    out = modulated_conv2d(p, prefix + ".conv", x, w, demodulate=True, upsample=upsample, s=s)
    out = out + p[prefix + ".noise.weight"].to(x.dtype) * noise.to(x.dtype)
    b = p[prefix + ".activate.bias"].to(x.dtype)
    pre = out + b.view(1, -1, 1, 1)
    if _FORCED is not None and prefix in _FORCED:
        forcing.relu_site("g." + prefix, _FORCED[prefix], pre)
        return torch.where(_FORCED[prefix], pre, 0.2 * pre) * math.sqrt(2.0)
    return F.leaky_relu(pre, 0.2) * math.sqrt(2.0)


def to_rgb(p, prefix, x, w, skip=None, s=None):
    out = modulated_conv2d(p, prefix + ".conv", x, w, demodulate=False, s=s)
    out = out + p[prefix + ".bias"].to(x.dtype)
    if skip is not None:
        up = make_kernel(BLUR_1D, x.dtype) * 4.0
        out = out + upfirdn2d(skip, up, up=2, pad=(2, 1))
    return out


def synthesis(p, latent, size):
    """Generator.forward with input_is_latent=True, randomize_noise=False, w+ of (N, n_latent, 512).
    Returns the image (N, 3, size, size)."""
    n = latent.shape[0]
    dt = latent.dtype
    log_size = int(math.log2(size))
    noises = [p[f"noises.noise_{i}"].to(dt) for i in range((log_size - 2) * 2 + 1)]
    out = p["input.input"].to(dt).repeat(n, 1, 1, 1)
    out = styled_conv(p, "conv1", out, latent[:, 0], noises[0])
    skip = to_rgb(p, "to_rgb1", out, latent[:, 1])
    i = 1
    for k in range(log_size - 2):
        out = styled_conv(p, f"convs.{2 * k}", out, latent[:, i], noises[2 * k + 1], upsample=True)
        out = styled_conv(p, f"convs.{2 * k + 1}", out, latent[:, i + 1], noises[2 * k + 2])
        skip = to_rgb(p, f"to_rgbs.{k}", out, latent[:, i + 2], skip)
        i += 2
    return skip


def mapping(p, z, n_mlp=8, lr_mul=0.01):
    """rosinality Generator.style: PixelNorm then n_mlp × EqualLinear(512, 512, lr_mul,
    activation='fused_lrelu'): x ← lrelu(x·(W·lr_mul/√512)ᵀ + b·lr_mul, 0.2)·√2."""
    x = z * torch.rsqrt(torch.mean(z * z, dim=1, keepdim=True) + 1e-8)
    for i in range(1, n_mlp + 1):
        w = p[f"style.{i}.weight"].to(z.dtype) * (lr_mul / math.sqrt(z.shape[1]))
        b = p[f"style.{i}.bias"].to(z.dtype) * lr_mul
        x = F.leaky_relu(x @ w.t() + b, 0.2) * math.sqrt(2)
    return x


def truncate(w, mean, psi):
    """Generator.forward truncation: mean + psi·(w − mean)."""
    return mean + psi * (w - mean)


def style_vectors(p, latent, size):
    """Per-layer modulation styles s for a W+ latent, in generator forward order (conv1, to_rgb1,
    then per resolution: up-conv, conv, to_rgb) — the 'style vector' of SFGenerator
    (style_fusion_simple.py:126-142, return_style_vector=True)."""
    log_size = int(math.log2(size))
    out = [style_affine(p, "conv1.conv", latent[:, 0]), style_affine(p, "to_rgb1.conv", latent[:, 1])]
    i = 1
    for k in range(log_size - 2):
        out.append(style_affine(p, f"convs.{2 * k}.conv", latent[:, i]))
        out.append(style_affine(p, f"convs.{2 * k + 1}.conv", latent[:, i + 1]))
        out.append(style_affine(p, f"to_rgbs.{k}.conv", latent[:, i + 2]))
        i += 2
    return out


def synthesis_from_styles(p, styles, size):
    """SFGenerator(style_vector=s) (style_fusion_simple.py:146-153): the synthesis driven by given
    per-layer styles (order of style_vectors)."""
    n = styles[0].shape[0]
    dt = styles[0].dtype
    log_size = int(math.log2(size))
    noises = [p[f"noises.noise_{i}"].to(dt) for i in range((log_size - 2) * 2 + 1)]
    out = p["input.input"].to(dt).repeat(n, 1, 1, 1)
    out = styled_conv(p, "conv1", out, None, noises[0], s=styles[0])
    skip = to_rgb(p, "to_rgb1", out, None, s=styles[1])
    j = 2
    for k in range(log_size - 2):
        out = styled_conv(p, f"convs.{2 * k}", out, None, noises[2 * k + 1], upsample=True,
                          s=styles[j])
        out = styled_conv(p, f"convs.{2 * k + 1}", out, None, noises[2 * k + 2], s=styles[j + 1])
        skip = to_rgb(p, f"to_rgbs.{k}", out, None, skip, s=styles[j + 2])
        j += 3
    return skip

