"""Adversarial patch attack: ``code/attack/patch/adversarial_patch.py``.

* ``attack(img, patch, mask, generator, encoder, vgg, ...)`` (:103-160) — the patch optimisation:
  loss = 0·MSE(E(t'),E(x')) − 1·MSE(E(x0'),E(x')) + 0·MSE(t, G(E(x'))) + 0·Σ_k MSE(V_k(G'),V_k(t'))
  (:125), ``patch -= ∇_x loss`` with the FULL-image gradient and step 1 (:127-131), then
  adv = clamp((1−m)·img + m·patch, min(img), max(img)) with tensor-global min / max (:133-134),
  for ``max_count`` iterations (:157). Returns (adv_x, mask, patch, adv_img_rec).
* ``patch_white_box(inputs, mask, adv_patch)`` (``attack_main2.py:413-420``) — paste a trained
  patch: per image clamp((1−m)·x + m·patch, min(x), max(x)).

The circle / square placement (``adversarial_patch_util.circle_transform`` / ``square_transform``,
:45-48) is un-vendored in the reference; callers pass the placed patch and mask (the tensors those
transforms return: the batch's shape). The weight-0 terms contribute 0·g to the gradient, so the
loop runs the encoder forward / backward only (AttackEngine.lat_only); the returned
adv_img_rec = G(E(adv')) of the last iteration's input is computed once. Runs on libmiattack
kernels (mia_patch_update for the update / composite, bit-exact vs torch fp32).
"""
import torch

from . import ops
from .pgd import PATCH_WEIGHTS, AttackEngine, _check_images


def attack(img, patch, mask, net, max_count, target_img=None, vgg=None, loss_scale=None):
    """adversarial_patch.attack on the device. img, patch, mask: (N,3,S,S) (patch / mask as the
    placement transforms return them); net: pSp bundle (net.encoder, net.decoder, optional
    net.vgg). ``patch`` is not modified; the updated patch is returned (the reference updates its
    argument in place). Returns (adv_x, mask, patch, adv_img_rec) on img's device."""
    size = net.decoder.size
    _check_images(img, size, "img")
    for name, t in (("patch", patch), ("mask", mask)):
        if tuple(t.shape) != tuple(img.shape):
            raise ValueError(f"{name} must have img's shape {tuple(img.shape)} (the placement "
                             "transforms return batch-shaped tensors)")
    if max_count < 1 or int(max_count) != max_count:
        raise ValueError("max_count must be an integer >= 1")
    vgg = vgg if vgg is not None else getattr(net, "vgg", None)
    if vgg is None:
        raise ValueError("a VGG feature network is required (the reference builds its targets)")
    dev = net.decoder.device
    f32 = torch.float32
    x0 = img.detach().to(dev, f32).contiguous()
    t = (target_img if target_img is not None else img).detach().to(dev, f32)
    if t.shape[0] == 1 and x0.shape[0] > 1:
        t = t.expand(x0.shape[0], -1, -1, -1)
    t = t.contiguous()
    p = patch.detach().to(dev, f32).clone().contiguous()
    m = mask.detach().to(dev, f32).contiguous()
    eng = AttackEngine(net.encoder.impl, net.decoder.impl, vgg.impl, loss_scale=loss_scale,
                       weights=PATCH_WEIGHTS)
    adv, rec = eng.run_patch(x0, t, p, m, int(max_count))
    d = img.device
    return adv.to(d), mask, p.to(d), rec.to(d)


def patch_white_box(inputs, mask, adv_patch):
    """attack_main2.py:413-420: for each image, clamp((1−m)·x + m·patch, min(x), max(x)).
    mask / adv_patch: one image's shape (3,S,S) or (1,3,S,S), broadcast over the batch."""
    if inputs.dim() != 4:
        raise ValueError("inputs must be (N,3,S,S)")
    dev = inputs.device
    f32 = torch.float32
    one = tuple(inputs.shape[1:])
    for nm, t in (("mask", mask), ("adv_patch", adv_patch)):
        # the (1,3,S,S) mask / patch adversarial_patch.main saves; a batch-shaped (N,3,S,S)
        # placement (the reference would broadcast it to N·N images) is not supported
        if t.numel() != inputs[0].numel() or tuple(t.shape[-3:]) != one:
            raise ValueError(f"{nm} must have shape (3,S,S) or (1,3,S,S) with (3,S,S) = {one}; "
                             f"got {tuple(t.shape)} (batch-shaped masks are not supported)")
    m = mask.detach().to(dev, f32).reshape(one).contiguous()
    p = adv_patch.detach().to(dev, f32).reshape(one).contiguous()
    x = inputs.detach().to(f32).contiguous()
    out = torch.empty_like(x)
    for i in range(x.shape[0]):  # per-image min / max (:417)
        xi = x[i:i + 1]
        ops.patch_update(p, None, xi, m, out[i:i + 1], float(xi.min()), float(xi.max()))
    return out
