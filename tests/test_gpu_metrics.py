"""Fusion-evaluation metrics (gfa_amd.metrics: cal_SSMI / cal_result of interpolation.py:903-919,
1076-1091) on the GPU against the CPU restatement oracle/metrics_ref.py (skimage's algorithm;
parity unpinned against skimage itself, which is absent here)."""
import pytest
import torch

from gfa_amd import metrics, networks
from oracle import metrics_ref

pytestmark = pytest.mark.gpu


def _imgs(N, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    ref = torch.rand(3, H, W, generator=g) * 2 - 1
    imgs = (ref.unsqueeze(0) + 0.25 * torch.randn(N, 3, H, W, generator=g)).clamp(-1, 1)
    imgs[0] = ref  # identical image: SSIM 1
    return ref, imgs


@pytest.mark.parametrize("N,H,W", [(2, 7, 7), (3, 40, 37), (2, 256, 256), (2, 1024, 1024)])
def test_ssim_kernel_matches_oracle(cuda, N, H, W):
    ref, imgs = _imgs(N, H, W, seed=H + W)
    got = metrics.ssim(ref.to(cuda), imgs.to(cuda)).cpu()
    for i in range(N):
        want = metrics_ref.cal_ssmi(ref.numpy(), imgs[i].numpy())
        assert abs(got[i].item() - want) < 2e-5, (i, got[i].item(), want)
    assert abs(got[0].item() - 1.0) < 1e-5
    # ordered per-tile partials (no atomics): bit-identical reruns, and an image's SSIM does not
    # depend on the other images of the call
    assert torch.equal(metrics.ssim(ref.to(cuda), imgs.to(cuda)).cpu(), got)
    alone = metrics.ssim(ref.to(cuda), imgs[N - 1:].to(cuda)).cpu()
    assert torch.equal(alone, got[N - 1:])


def test_cal_ssmi_and_cal_result(cuda):
    """cal_result: per image the pixel MSE, the Σ of the 4 VGG-tap MSEs (the device VGG trunk),
    and the SSIM, as the reference's three dicts."""
    torch.manual_seed(0)
    N, S = 3, 64
    ref, imgs = _imgs(N, S, S, seed=5)
    vgg = networks.vgg16(networks.make_vgg_weights(1234), device=cuda)
    mse, vg, ss = metrics.cal_result(ref.unsqueeze(0), imgs, vgg)
    assert sorted(mse) == list(range(N))
    t0 = vgg(ref.unsqueeze(0).to(cuda))
    ts = vgg(imgs.to(cuda))
    for i in range(N):
        assert abs(mse[i] - ((imgs[i] - ref) ** 2).mean().item()) < 1e-6
        want_vg = sum(((a[0] - b[i]) ** 2).mean().item() for a, b in zip(t0, ts))
        assert abs(vg[i] - want_vg) <= 1e-5 * max(1.0, want_vg)
        assert abs(ss[i] - metrics_ref.cal_ssmi(ref.numpy(), imgs[i].numpy())) < 2e-5
        assert abs(metrics.cal_SSMI(ref, imgs[i]) - ss[i]) < 1e-7
    assert mse[0] == 0.0 and vg[0] == 0.0
