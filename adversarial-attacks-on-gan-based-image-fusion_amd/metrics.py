"""Fusion-evaluation metrics of the reference on device kernels.

Mirrors code/attack/interpolation.py:
* ``cal_SSMI(original_image, distorted_image)`` (:903-919): SSIM of the rgb2gray images with
  skimage.metrics.structural_similarity's defaults — ``mia_ssim`` (csrc/metrics.hip);
* ``cal_result(original_f, adv_f_all)`` (:1076-1091): per adversarial fusion i, the pixel MSE to
  the original fusion (``mia_mse_sum``), the sum of the four VGG-tap MSEs (the VGG trunk on
  device, code/vgg.py:44-64) and the SSIM; returned as the reference's three dicts.

``data_range`` = 2.0 by default: skimage < 0.20 used the float dtype range (−1, 1) when it was not
given, as in the reference call (later skimage versions require it explicitly).
"""
import torch

from . import ops


def _dev(t):
    """Host tensors are copied to the current GPU once (as attack() does); no CPU path."""
    return t if t.is_cuda else t.to(torch.device("cuda", torch.cuda.current_device()))


def ssim(ref, imgs, data_range=2.0):
    """ref (3,H,W) or (1,3,H,W), imgs (N,3,H,W): fp32 CUDA tensors → SSIM per image (N,) fp32."""
    ref = ref.reshape(3, ref.shape[-2], ref.shape[-1]).float().contiguous()
    if imgs.dim() == 3:
        imgs = imgs.unsqueeze(0)
    imgs = imgs.float().contiguous()
    N, C, H, W = imgs.shape
    if C != 3 or tuple(ref.shape) != (3, H, W):
        raise ValueError("ssim: RGB images of one size expected")
    work = torch.empty(ops.ssim_workspace_numel(N, H, W), dtype=torch.float64, device=imgs.device)
    out = torch.empty(N, dtype=torch.float32, device=imgs.device)
    ops.ssim(ref, imgs, data_range, work, out)
    return out


def cal_SSMI(original_image, distorted_image, data_range=2.0):  # noqa: N802 (reference name)
    """interpolation.py:903-919: (3,H,W) images → SSIM (float)."""
    if tuple(original_image.shape) != tuple(distorted_image.shape):
        raise ValueError("Both images must have the same dimensions and shape.")
    return float(ssim(_dev(original_image), _dev(distorted_image), data_range)[0])


def _mse_rows(a, b):
    """Per-row mean squared difference of two (n, …) fp32 tensors (mia_mse_sum)."""
    n = a.shape[0]
    loss = torch.zeros(n, dtype=torch.float32, device=a.device)
    ops.mse_sum(a.contiguous(), b.contiguous(), loss, coef=1.0 / (a.numel() // n))
    return loss


def cal_result(original_f, adv_f_all, vgg, data_range=2.0):
    """interpolation.py:1076-1091. original_f (1,3,H,W), adv_f_all (N,3,H,W) in [-1,1]; vgg: the
    VGG trunk (networks.VGGBase / vgg16(), called as vgg(x) → 4 taps). Returns (mse, vgg, ssim)
    dicts keyed by image index, like the reference."""
    x0 = _dev(original_f).float().reshape(1, *original_f.shape[-3:])
    xs = _dev(adv_f_all).float().contiguous()
    N = xs.shape[0]
    mse = _mse_rows(x0.expand(N, -1, -1, -1), xs)
    t0 = vgg(x0)
    ts = vgg(xs)
    vg = torch.zeros(N, dtype=torch.float32, device=xs.device)
    for a, b in zip(t0, ts):
        vg += _mse_rows(a.expand(N, *a.shape[1:]), b)
    ss = ssim(x0, xs, data_range)
    mse, vg, ss = mse.tolist(), vg.tolist(), ss.tolist()
    return ({i: mse[i] for i in range(N)}, {i: vg[i] for i in range(N)},
            {i: ss[i] for i in range(N)})
