"""On-disk formats of the attack's outputs. Host-side I/O, no kernels.

* Raw tensor dumps — ``attack_main2.py:1097-1111``: ``torch.save`` of the concatenated batches
  under the reference's file names (``.npz`` is the reference's suffix; the content is torch's
  zip-pickle format, not numpy's): adversarial inputs / rec losses / inner features in the
  adversarial directory, their benign counterparts in the benign one. ``load_records`` reads them
  back with ``torch.load(weights_only=True)`` (plain tensors; nothing in the file is executed).
* Image grids — ``torchvision.utils.save_image((x + 1) / 2, path)`` as the reference calls it
  (``attack_main2.py:1025-1028``, ``interpolation.py:386``): make_grid(nrow=8, padding=2,
  pad_value=0) then ``mul(255).add_(0.5).clamp_(0, 255)`` to uint8 and PIL. torchvision is not in
  this image; ``make_grid`` / ``save_image`` restate it.
* Grid reload — ``interpolation.py:1379-1394``: the saved grid read back as a [-1, 1] tensor
  (ToTensor + Normalize(0.5, 0.5)) and cut into tiles at rows 2…S+2, columns i·S+2…i·S+S+2 — the
  reference's offsets, which ignore the 2-pixel separators after the first tile
  (``reference_tiles``); ``grid_tiles`` is the exact inverse of make_grid. (The reference's
  img_transform there also resizes to the decoder size, which would make its crop indices fall
  outside the image; it is not applied.)
* Per-image JPEG — ``attack_main2.py:164-171`` (``save_image(img, save_dir, idx)`` over
  ``utils/common.py:10-17`` tensor2im): (x + 1)/2 clipped to [0, 1], ×255, truncated to uint8,
  ``{idx:05d}.jpg`` or ``{idx}.jpg``.
"""
import math
import os

import numpy as np
import torch

ADV_FILES = ("all_adv_inputs", "all_adv_rec_loss", "all_adv_inner_feature")
BENIGN_FILES = ("all_inputs", "all_rec_loss", "all_inner_feature")


def save_records(adv_savedir, benign_savedir, *, all_adv_inputs, all_inputs, all_adv_rec_loss,
                 all_rec_loss, all_adv_inner_feature=None, all_inner_feature=None):
    """attack_main2.py:1097-1111: each argument is a list of per-batch tensors (concatenated on
    dim 0, as torch.cat(all_x, dim=0)) or one tensor. Inner features are optional (the reference
    collects them from its fusion model)."""
    def cat(v):
        return torch.cat(list(v), dim=0) if isinstance(v, (list, tuple)) else v

    os.makedirs(adv_savedir, exist_ok=True)
    os.makedirs(benign_savedir, exist_ok=True)
    out = {}
    for d, name, v in ((adv_savedir, "all_adv_inputs", all_adv_inputs),
                       (benign_savedir, "all_inputs", all_inputs),
                       (adv_savedir, "all_adv_rec_loss", all_adv_rec_loss),
                       (benign_savedir, "all_rec_loss", all_rec_loss),
                       (adv_savedir, "all_adv_inner_feature", all_adv_inner_feature),
                       (benign_savedir, "all_inner_feature", all_inner_feature)):
        if v is None:
            continue
        path = os.path.join(d, name + ".npz")
        torch.save(cat(v).detach().cpu(), path)
        out[name] = path
    return out


def load_records(directory):
    """{name: tensor} of the record files present in one directory (weights_only loads)."""
    out = {}
    for name in ADV_FILES + BENIGN_FILES:
        path = os.path.join(directory, name + ".npz")
        if os.path.exists(path):
            out[name] = torch.load(path, map_location="cpu", weights_only=True)
    return out


def make_grid(t, nrow=8, padding=2, pad_value=0.0):
    """torchvision.utils.make_grid (normalize=False): tiles row-major, ``padding`` pixels before
    every tile and after the last; one image is returned unpadded; 1-channel → 3-channel."""
    t = t.detach()
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.dim() == 3:
        t = t.unsqueeze(0)
    if t.shape[1] == 1:
        t = torch.cat((t, t, t), 1)
    if t.shape[0] == 1:
        return t.squeeze(0)
    n = t.shape[0]
    xm = min(nrow, n)
    ym = int(math.ceil(n / xm))
    h, w = t.shape[2] + padding, t.shape[3] + padding
    grid = t.new_full((t.shape[1], h * ym + padding, w * xm + padding), pad_value)
    k = 0
    for y in range(ym):
        for x in range(xm):
            if k >= n:
                break
            grid[:, y * h + padding:y * h + padding + t.shape[2],
                 x * w + padding:x * w + padding + t.shape[3]] = t[k]
            k += 1
    return grid


def to_uint8_hwc(grid):
    """torchvision save_image's quantisation: mul(255).add_(0.5).clamp_(0, 255) → uint8, HWC."""
    return grid.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to("cpu", torch.uint8).numpy()


def save_image(t, path, nrow=8, padding=2, pad_value=0.0):
    """torchvision.utils.save_image(t, path) — the reference passes (x + 1) / 2."""
    from PIL import Image
    grid = make_grid(t.detach().cpu().float(), nrow=nrow, padding=padding, pad_value=pad_value)
    Image.fromarray(to_uint8_hwc(grid)).save(path)
    return path


def load_image_tensor(path):
    """ToTensor + Normalize([0.5]*3, [0.5]*3): an image file as a (3, H, W) tensor in [-1, 1]."""
    from PIL import Image
    a = np.asarray(Image.open(path).convert("RGB"), dtype=np.float32) / 255.0
    return (torch.from_numpy(a).permute(2, 0, 1) - 0.5) / 0.5


def reference_tiles(grid, n, size):
    """interpolation.py:1386-1394: tile i = grid[:, 2:size+2, i·size+2 : i·size+size+2] (the
    reference's offsets; exact for tile 0, shifted 2·i pixels left of make_grid's tile i)."""
    return [grid[:, 2:size + 2, i * size + 2:i * size + size + 2].unsqueeze(0) for i in range(n)]


def grid_tiles(grid, n, size, nrow=8, padding=2):
    """Exact inverse of make_grid for n tiles of size × size."""
    if n == 1:
        return [grid.unsqueeze(0)]
    step = size + padding
    return [grid[:, (k // nrow) * step + padding:(k // nrow) * step + padding + size,
                 (k % nrow) * step + padding:(k % nrow) * step + padding + size].unsqueeze(0)
            for k in range(n)]


def tensor2im(var):
    """utils/common.py:10-17: (3, H, W) in [-1, 1] → PIL image (clip, ×255, truncate)."""
    from PIL import Image
    a = var.detach().cpu().permute(1, 2, 0).numpy()
    a = (a + 1) / 2
    a[a < 0] = 0
    a[a > 1] = 1
    return Image.fromarray((a * 255).astype("uint8"))


def save_image_idx(img, save_dir, idx):
    """attack_main2.py:164-171: one image as save_dir/{idx:05d}.jpg (int idx) or {idx}.jpg."""
    name = f"{idx:05d}.jpg" if isinstance(idx, int) else f"{idx}.jpg"
    path = os.path.join(save_dir, name)
    tensor2im(img).save(path)
    return path
