"""CPU restatement of the reference's fusion-evaluation metrics — TEST INFRASTRUCTURE ONLY (the
checker of gfa_amd.metrics; never imported by the product path).

* cal_SSMI (code/attack/interpolation.py:903-919): skimage.color.rgb2gray then
  skimage.metrics.structural_similarity with its defaults. scikit-image is an un-vendored
  dependency of the reference (imported at interpolation.py:44, no version pin in the repository)
  and is not installed here, so this restates its published algorithm (skimage
  _structural_similarity.py, 0.19-0.22): 7×7 uniform window (scipy.ndimage.uniform_filter, mode
  'reflect'), sample covariance NP/(NP−1), K1 = 0.01, K2 = 0.03, C = (K·data_range)², mean of the
  SSIM map after cropping (win−1)/2 = 3 pixels per side, all in float64. data_range: skimage < 0.20
  took the float dtype range (−1, 1) → 2 when it was not given (the reference does not give it);
  later versions require it. PARITY UNPINNED against skimage itself (no fixture of the reference
  holds an SSIM value); pinned by the closed-form properties in tests/test_oracle.py.
* rgb2gray: 0.2125 R + 0.7154 G + 0.0721 B on float input (no rescaling).
* cal_result (interpolation.py:1076-1091): MSE(original, adv_i), Σ of the 4 VGG-tap MSEs, SSIM.
"""
import numpy as np
from scipy import ndimage

RGB2GRAY = np.array([0.2125, 0.7154, 0.0721])


def rgb2gray(chw):
    """(3, H, W) → (H, W) float64 (skimage.color.rgb2gray on an HWC float image)."""
    a = np.asarray(chw, dtype=np.float64)
    return np.tensordot(RGB2GRAY, a, axes=(0, 0))


def structural_similarity(x, y, data_range=2.0, win_size=7, K1=0.01, K2=0.03):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if x.shape != y.shape:
        raise ValueError("Both images must have the same dimensions and shape.")
    np_ = win_size ** x.ndim
    cov_norm = np_ / (np_ - 1)
    f = lambda a: ndimage.uniform_filter(a, size=win_size, mode="reflect")  # noqa: E731
    ux, uy = f(x), f(y)
    uxx, uyy, uxy = f(x * x), f(y * y), f(x * y)
    vx = cov_norm * (uxx - ux * ux)
    vy = cov_norm * (uyy - uy * uy)
    vxy = cov_norm * (uxy - ux * uy)
    c1, c2 = (K1 * data_range) ** 2, (K2 * data_range) ** 2
    s = ((2 * ux * uy + c1) * (2 * vxy + c2)) / ((ux ** 2 + uy ** 2 + c1) * (vx + vy + c2))
    pad = (win_size - 1) // 2
    return float(s[pad:-pad, pad:-pad].mean())


def cal_ssmi(original_chw, distorted_chw, data_range=2.0):
    """interpolation.py:903-919 on (3, H, W) arrays."""
    return structural_similarity(rgb2gray(original_chw), rgb2gray(distorted_chw), data_range)


def ssim_direct(x, y, data_range=2.0):
    """The same mean SSIM by explicit 7×7 window loops (small images only): the independent
    check of structural_similarity's filter / crop bookkeeping."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    H, W = x.shape
    c1, c2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    tot, cnt = 0.0, 0
    for i in range(3, H - 3):
        for j in range(3, W - 3):
            a = x[i - 3:i + 4, j - 3:j + 4].ravel()
            b = y[i - 3:i + 4, j - 3:j + 4].ravel()
            ux, uy = a.mean(), b.mean()
            vx, vy = a.var(ddof=1), b.var(ddof=1)
            vxy = ((a - ux) * (b - uy)).sum() / 48.0
            tot += ((2 * ux * uy + c1) * (2 * vxy + c2)) / ((ux * ux + uy * uy + c1) * (vx + vy + c2))
            cnt += 1
    return tot / cnt
