"""CPU oracle: the encoder behind ``net.encoder`` (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Two encoders:

* ``encode``     — the synthetic linear stand-in:
                   E(x) = W_E·vec(avgpool(x))/sqrt(768) + b_E → (N, n_latent, 512), avgpool reducing
                   a 256² image to 16². The build's own definition; parity unpinned.
* ``e4e_encode`` — e4e ``Encoder4Editing(50, 'ir_se', opts)`` as the reference builds it
                   (``code/utils/model_utils.py:24``, called as ``net.encoder(x)`` at
                   ``code/attack/attack_main2.py:597,622`` and ``interpolation.py:757-781``).
                   The module is an UN-VENDORED dependency (omertov/encoder4editing
                   ``models/encoders/psp_encoders.py`` + ``helpers.py``: ``get_blocks``,
                   ``bottleneck_IR_SE``, ``SEModule``, ``GradualStyleBlock``, ``_upsample_add``;
                   ``EqualLinear`` from its stylegan2 ``model.py``; no version pin in the
                   reference). Its published algorithm is restated with torch functional ops in
                   eval mode (BatchNorm running statistics, eps 1e-5). **Parity unpinned**: no
                   reference test or fixture holds encoder outputs.
"""
import math

import torch
import torch.nn.functional as F

from . import forcing

BN_EPS = 1e-5
# Teacher-forced activation masks (tests only): {key: bool tensor (NCHW)}. Under forced_masks the
# positive set of a PReLU / LeakyReLU is taken from the given mask instead of the sign of its own
# fp64 pre-activation, so the oracle's backward follows the same piecewise-linear branch as the
# device run (a pre-activation within rounding of 0 may take either branch). Keys: "in" (input
# layer PReLU), "body.{i}" (unit i's PReLU), "body.{i}.se" (its SE block's ReLU, (N, C/16, 1, 1)),
# "styles.{i}.{j}" (head i's j-th LeakyReLU(0.01)).
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


def _leaky(x, slope, key):
    """PReLU (per-channel tensor slope) / LeakyReLU (float slope), optionally mask-forced."""
    m = _FORCED.get(key) if _FORCED is not None else None
    if m is None:
        return F.prelu(x, slope) if torch.is_tensor(slope) else F.leaky_relu(x, slope)
    s = slope.view(1, -1, 1, 1) if torch.is_tensor(slope) else slope
    forcing.relu_site("e4e." + key, m, x)
    return torch.where(m.to(x.device), x, s * x)
E4E_STAGES = [(64, 64, 3), (64, 128, 4), (128, 256, 14), (256, 512, 3)]  # helpers.get_blocks(50)
COARSE, MIDDLE = 3, 7


def encode(e, x):
    n, _, h, _ = x.shape
    v = F.avg_pool2d(x, h // 16).reshape(n, -1)
    w = e["enc.weight"].to(x.dtype)
    lat = F.linear(v, w * (1.0 / math.sqrt(w.shape[1])), e["enc.bias"].to(x.dtype))
    return lat.view(n, -1, 512)


def _units():
    out = []
    for cin, depth, n in E4E_STAGES:
        out.append((cin, depth, 2))
        out += [(depth, depth, 1)] * (n - 1)
    return out


def _bn(p, pre, x):
    t = lambda k: p[f"{pre}.{k}"].to(x.dtype)  # noqa: E731
    return F.batch_norm(x, t("running_mean"), t("running_var"), t("weight"), t("bias"),
                        training=False, eps=BN_EPS)


def _w(p, k, x):
    return p[k].to(x.dtype)


def bottleneck_ir_se(p, pre, x, cin, depth, stride):
    """helpers.bottleneck_IR_SE.forward: res_layer(x) + shortcut_layer(x)."""
    if cin == depth:
        sc = F.max_pool2d(x, 1, stride)  # MaxPool2d(1, stride)
    else:
        sc = F.conv2d(x, _w(p, pre + ".shortcut_layer.0.weight", x), stride=stride)
        sc = _bn(p, pre + ".shortcut_layer.1", sc)
    r = _bn(p, pre + ".res_layer.0", x)
    r = F.conv2d(r, _w(p, pre + ".res_layer.1.weight", x), stride=1, padding=1)
    r = _leaky(r, _w(p, pre + ".res_layer.2.weight", x), pre)
    r = F.conv2d(r, _w(p, pre + ".res_layer.3.weight", x), stride=stride, padding=1)
    r = _bn(p, pre + ".res_layer.4", r)
    # SEModule(depth, 16)
    s = F.adaptive_avg_pool2d(r, 1)
    s = _leaky(F.conv2d(s, _w(p, pre + ".res_layer.5.fc1.weight", x)), 0.0, pre + ".se")
    s = torch.sigmoid(F.conv2d(s, _w(p, pre + ".res_layer.5.fc2.weight", x)))
    return r * s + sc


def gradual_style_block(p, pre, x, spatial):
    """GradualStyleBlock(512, 512, spatial): log2(spatial) × (conv3×3 s2 + LeakyReLU(0.01)),
    view(-1, 512), EqualLinear(512, 512, lr_mul=1)."""
    for j in range(int(math.log2(spatial))):
        x = F.conv2d(x, _w(p, f"{pre}.convs.{2 * j}.weight", x), _w(p, f"{pre}.convs.{2 * j}.bias", x),
                     stride=2, padding=1)
        x = _leaky(x, 0.01, f"{pre}.{j}")
    x = x.reshape(-1, 512)
    w = _w(p, pre + ".linear.weight", x)
    return F.linear(x, w * (1.0 / math.sqrt(w.shape[1])), _w(p, pre + ".linear.bias", x))


def _upsample_add(x, y):
    return F.interpolate(x, size=y.shape[-2:], mode="bilinear", align_corners=True) + y


def e4e_features(p, x):
    """Input layer + IR-SE50 body; returns (c1, c2, c3) (Encoder4Editing.forward, i = 6, 20, 23)."""
    x = F.conv2d(x, _w(p, "input_layer.0.weight", x), padding=1)
    x = _bn(p, "input_layer.1", x)
    x = _leaky(x, _w(p, "input_layer.2.weight", x), "in")
    c = {}
    for i, (cin, depth, stride) in enumerate(_units()):
        x = bottleneck_ir_se(p, f"body.{i}", x, cin, depth, stride)
        if i in (6, 20, 23):
            c[i] = x
    return c[6], c[20], c[23]


def e4e_encode(p, x, style_count):
    """Encoder4Editing.forward at ProgressiveStage.Inference (every delta active): w (N, S, 512) =
    styles[0](c3) repeated, w[:, i] += styles[i](features_i) with features c3 / p2 / p1."""
    c1, c2, c3 = e4e_features(p, x)
    w0 = gradual_style_block(p, "styles.0", c3, 16)
    w = w0.unsqueeze(1).repeat(1, style_count, 1)
    feats = c3
    p2 = None
    deltas = [torch.zeros_like(w0)]
    for i in range(1, style_count):
        if i == COARSE:
            p2 = _upsample_add(c3, F.conv2d(c2, _w(p, "latlayer1.weight", c2),
                                            _w(p, "latlayer1.bias", c2)))
            feats = p2
        elif i == MIDDLE:
            feats = _upsample_add(p2, F.conv2d(c1, _w(p, "latlayer2.weight", c1),
                                               _w(p, "latlayer2.bias", c1)))
        sp = 16 if i < COARSE else (32 if i < MIDDLE else 64)
        deltas.append(gradual_style_block(p, f"styles.{i}", feats, sp))
    return w + torch.stack(deltas, dim=1)


def apply(ep, xp, size):
    """``net.encoder(x')`` for either encoder dict (``kind`` "e4e" → e4e_encode)."""
    if ep.get("kind") == "e4e":
        return e4e_encode(ep, xp, 2 * int(math.log2(size)) - 2)
    return encode(ep, xp)
