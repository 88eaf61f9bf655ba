"""CPU oracle: VGG16 trunk with four feature taps (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Restates ``code/vgg.py``:
* forward ``code/vgg.py:44-64``: conv1_1→relu (tap), conv1_2→relu (tap), pool1, conv2_1, conv2_2,
  pool2 (the tap the reference names ``conv3_2`` is the pool2 output, ``vgg.py:53-54``), conv3_1..3,
  pool3 with ``ceil_mode=True`` (``vgg.py:24``), conv4_1, conv4_2→relu (tap).
* weight loading ``code/vgg.py:66-76``: the first 26 tensors of the checkpoint, positionally.
"""
import torch
import torch.nn.functional as F

from . import forcing

LAYERS = ["conv1_1", "conv1_2", "conv2_1", "conv2_2", "conv3_1", "conv3_2", "conv3_3",
          "conv4_1", "conv4_2"]


def load_positional(state_dict):
    """vgg.py:70-74 — take checkpoint tensors in order, weight then bias per conv."""
    vals = list(state_dict.values())
    params = {}
    for i, name in enumerate(LAYERS):
        params[name] = (vals[2 * i], vals[2 * i + 1])
    return params


# Teacher-forced branches (tests only): a list of {key: bool tensor (NCHW)} consumed one per
# vgg_forward call. Keys: the conv names (ReLU positive set) and "pool1" / "pool2" / "pool3" (the
# one-hot argmax of every 2×2 window at the pool's input resolution). Under forcing the oracle
# follows the device run's branch wherever a pre-activation or a window's maximum is within
# rounding of a tie; the function is the same piecewise-linear one.
_FORCED = None


class forced_masks:
    def __init__(self, per_call):
        self.per_call = list(per_call)

    def __enter__(self):
        global _FORCED
        _FORCED = self.per_call
        return self

    def __exit__(self, *exc):
        global _FORCED
        _FORCED = None


def vgg_forward(params, image):
    """vgg.py:44-64. Returns (conv1_1, conv1_2, conv3_2[=pool2 output], conv4_2)."""
    forced = _FORCED.pop(0) if _FORCED else None

    def conv(name, x):
        w, b = params[name]
        y = F.conv2d(x, w.to(x.dtype), b.to(x.dtype), padding=1)
        if forced is not None:
            forcing.relu_site("vgg." + name, forced[name], y)
            return torch.where(forced[name], y, torch.zeros_like(y))
        return F.relu(y)

    def pool(name, x, ceil_mode=False):
        if forced is not None:  # the forced window maxima: a sum over each window of x·one-hot
            forcing.pool_site("vgg." + name, forced[name], x, ceil_mode)
            xm = torch.where(forced[name], x, torch.zeros_like(x))
            return F.avg_pool2d(xm, 2, 2, ceil_mode=ceil_mode, divisor_override=1)
        return F.max_pool2d(x, 2, 2, ceil_mode=ceil_mode)

    out = conv("conv1_1", image)
    c11 = out
    out = conv("conv1_2", out)
    c12 = out
    out = pool("pool1", out)
    out = conv("conv2_1", out)
    out = conv("conv2_2", out)
    out = pool("pool2", out)
    c32 = out
    out = conv("conv3_1", out)
    out = conv("conv3_2", out)
    out = conv("conv3_3", out)
    out = pool("pool3", out, ceil_mode=True)
    out = conv("conv4_1", out)
    out = conv("conv4_2", out)
    return c11, c12, c32, out


def branch_masks(params, image):
    """The ReLU positive sets and pool-window argmax one-hots (first maximum in row-major window
    order, ceil-mode windows padded with −inf) that vgg_forward takes on ``image`` in image's own
    dtype — e.g. the branches of a torch CPU fp32 run, for forced_masks."""
    m, out = {}, image
    pools = {"conv1_2": ("pool1", False), "conv2_2": ("pool2", False), "conv3_3": ("pool3", True)}
    with torch.no_grad():
        for name in LAYERS:
            w, b = params[name]
            pre = F.conv2d(out, w.to(out.dtype), b.to(out.dtype), padding=1)
            m[name] = pre > 0
            out = F.relu(pre)
            if name in pools:
                pn, ceil = pools[name]
                N, C, H, W = out.shape
                xp = F.pad(out, (0, W % 2, 0, H % 2), value=float("-inf"))
                Hp, Wp = xp.shape[2], xp.shape[3]
                win = xp.reshape(N, C, Hp // 2, 2, Wp // 2, 2).permute(0, 1, 2, 4, 3, 5)
                oh = F.one_hot(win.reshape(N, C, Hp // 2, Wp // 2, 4).argmax(-1), 4).bool()
                oh = oh.reshape(N, C, Hp // 2, Wp // 2, 2, 2).permute(0, 1, 2, 4, 3, 5)
                m[pn] = oh.reshape(N, C, Hp, Wp)[:, :, :H, :W]
                out = F.max_pool2d(out, 2, 2, ceil_mode=ceil)
    return m


def tap_mse_grad(params, image, targets):
    """Input gradient of Σ_k MSE(tap_k(image), target_k) (mean reduction, as interpolation.py:766)."""
    x = image.clone().requires_grad_(True)
    taps = vgg_forward(params, x)
    loss = sum(F.mse_loss(t, tt) for t, tt in zip(taps, targets))
    (g,) = torch.autograd.grad(loss, x)
    return loss.detach(), g
