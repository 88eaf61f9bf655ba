"""CPU oracle: VGG16 trunk with four feature taps (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Restates ``code/vgg.py``:
* forward ``code/vgg.py:44-64``: conv1_1→relu (tap), conv1_2→relu (tap), pool1, conv2_1, conv2_2,
  pool2 (the tap the reference names ``conv3_2`` is the pool2 output, ``vgg.py:53-54``), conv3_1..3,
  pool3 with ``ceil_mode=True`` (``vgg.py:24``), conv4_1, conv4_2→relu (tap).
* weight loading ``code/vgg.py:66-76``: the first 26 tensors of the checkpoint, positionally.
"""
import torch
import torch.nn.functional as F

LAYERS = ["conv1_1", "conv1_2", "conv2_1", "conv2_2", "conv3_1", "conv3_2", "conv3_3",
          "conv4_1", "conv4_2"]


def load_positional(state_dict):
    """vgg.py:70-74 — take checkpoint tensors in order, weight then bias per conv."""
    vals = list(state_dict.values())
    params = {}
    for i, name in enumerate(LAYERS):
        params[name] = (vals[2 * i], vals[2 * i + 1])
    return params


def vgg_forward(params, image):
    """vgg.py:44-64. Returns (conv1_1, conv1_2, conv3_2[=pool2 output], conv4_2)."""
    def conv(name, x):
        w, b = params[name]
        return F.relu(F.conv2d(x, w.to(x.dtype), b.to(x.dtype), padding=1))

    out = conv("conv1_1", image)
    c11 = out
    out = conv("conv1_2", out)
    c12 = out
    out = F.max_pool2d(out, 2, 2)
    out = conv("conv2_1", out)
    out = conv("conv2_2", out)
    out = F.max_pool2d(out, 2, 2)
    c32 = out
    out = conv("conv3_1", out)
    out = conv("conv3_2", out)
    out = conv("conv3_3", out)
    out = F.max_pool2d(out, 2, 2, ceil_mode=True)
    out = conv("conv4_1", out)
    out = conv("conv4_2", out)
    return c11, c12, c32, out


def tap_mse_grad(params, image, targets):
    """Input gradient of Σ_k MSE(tap_k(image), target_k) (mean reduction, as interpolation.py:766)."""
    x = image.clone().requires_grad_(True)
    taps = vgg_forward(params, x)
    loss = sum(F.mse_loss(t, tt) for t, tt in zip(taps, targets))
    (g,) = torch.autograd.grad(loss, x)
    return loss.detach(), g
