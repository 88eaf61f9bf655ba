"""CPU oracle: white-box objective + PGD/FGSM (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

* Objective — ``code/attack/interpolation.py:743-818`` (``optimize_vgg``), per image, every MSE
  with ``reduction='mean'`` (``:766``)::

    L = (10·MSE(E(x'), E(t')) − MSE(E(x'), E(x0')))                       # latent terms
      + (MSE(t, G(E(x'))) + 0.1·Σ_k MSE(V_k(G(E(x'))'), V_k(t')))           # reconstruction terms
      + (10·MSE(x0, x) + Σ_k MSE(V_k(x'), V_k(x0')))                        # input-fidelity terms

  with ' = avg_pool2d(·, S/256) (``:749-750,780-785``). The decoder gets the raw encoder output
  (no latent_avg, ``:780``). Images are independent, so a batch's loss is the SUM of per-image
  losses (each image's gradient equals the reference's batch-1 gradient).
* PGD update — torchattacks ``PGD.forward`` copied in comments at ``interpolation.py:62-96``:
  adv += α·sign(∇cost); δ = clamp(adv − x, −ε, ε); adv = clamp(x + δ, lo, hi). The reference
  minimises L, so cost = −L (the targeted form, ``:83-86``). ε, α are in [0,1] pixel units and the
  tensors live in [-1,1]: e = 2ε, a = 2α, lo/hi = −1/+1.
"""
import contextlib

import numpy as np
import torch
import torch.nn.functional as F

from . import encoder_ref, stylegan2_ref, vgg_ref

LOSS_WEIGHTS = dict(lat_t=10.0, lat_o=-1.0, img_rec_t=1.0, vgg_rec_t=0.1, img_o=10.0, vgg_img=1.0)


def _mse_per_image(a, b):
    return ((a - b) ** 2).reshape(a.shape[0], -1).mean(dim=1)


class Refs:
    """Precomputed (no_grad) targets: interpolation.py:757-764."""

    def __init__(self, gp, vp, ep, x0, t, size):
        with torch.no_grad():
            pf = max(1, size // 256)
            self.x0, self.t = x0, t
            self.x0p = F.avg_pool2d(x0, pf) if pf > 1 else x0
            self.tp = F.avg_pool2d(t, pf) if pf > 1 else t
            self.lat_t = encoder_ref.apply(ep, self.tp, size)
            self.lat_o = encoder_ref.apply(ep, self.x0p, size)
            self.taps_t = vgg_ref.vgg_forward(vp, self.tp)
            self.taps_o = vgg_ref.vgg_forward(vp, self.x0p)


def objective(gp, vp, ep, x, refs, size, weights=LOSS_WEIGHTS, per_image=False):
    """The per-image objective (summed unless ``per_image``). With only the latent terms weighted
    (the patch attack's loss, adversarial_patch.py:125) the generator and VGG terms are 0·(finite)
    = +0 exactly in L and in ∇L, so they are not evaluated."""
    pf = max(1, size // 256)
    xp = F.avg_pool2d(x, pf) if pf > 1 else x
    lat = encoder_ref.apply(ep, xp, size)
    w = weights
    if all(w[k] == 0 for k in ("img_rec_t", "vgg_rec_t", "img_o", "vgg_img")):
        L = (w["lat_t"] * _mse_per_image(refs.lat_t, lat)
             + w["lat_o"] * _mse_per_image(refs.lat_o, lat))
        return L if per_image else L.sum()
    rec = stylegan2_ref.synthesis(gp, lat, size)
    recp = F.avg_pool2d(rec, pf) if pf > 1 else rec
    taps_rec = vgg_ref.vgg_forward(vp, recp)
    taps_x = vgg_ref.vgg_forward(vp, xp)
    l_lat_t = _mse_per_image(refs.lat_t, lat)
    l_lat_o = _mse_per_image(refs.lat_o, lat)
    l_img_rec_t = _mse_per_image(refs.t, rec)
    l_vgg_rec_t = sum(_mse_per_image(a, b) for a, b in zip(taps_rec, refs.taps_t))
    l_img_o = _mse_per_image(refs.x0, x)
    l_vgg_img = sum(_mse_per_image(a, b) for a, b in zip(taps_x, refs.taps_o))
    L = (w["lat_t"] * l_lat_t + w["lat_o"] * l_lat_o + w["img_rec_t"] * l_img_rec_t
         + w["vgg_rec_t"] * l_vgg_rec_t + w["img_o"] * l_img_o + w["vgg_img"] * l_vgg_img)
    return L if per_image else L.sum()


def loss_grad(gp, vp, ep, x, refs, size):
    """∇_x L (summed over images) and the per-image losses."""
    xx = x.detach().clone().requires_grad_(True)
    L = objective(gp, vp, ep, xx, refs, size, per_image=True)
    (g,) = torch.autograd.grad(L.sum(), xx)
    return L.detach(), g


def project_step(adv, x0, g, e, a, lo=-1.0, hi=1.0):
    """interpolation.py:92-94 with cost = −L: adv + a·sign(−g), then the ε-ball and range clamps.
    Scalars are rounded to fp32 first, as torch does for a float32 tensor."""
    a32 = float(np.float32(a))
    e32 = float(np.float32(e))
    adv = adv.detach() + a32 * torch.sign(-g)
    delta = torch.clamp(adv - x0, min=-e32, max=e32)
    return torch.clamp(x0 + delta, min=lo, max=hi).detach()


def pgd(gp, vp, ep, x0, t, size, eps, alpha, steps, random_start=False, start_noise=None,
        dtype=torch.float32, return_grads=False, progress=None):
    """PGD-`steps` in [-1,1] space (FGSM = steps 1, alpha = eps, no random start).

    ``start_noise``: U(-1,1) draws, scaled by e here (host-seeded so the GPU path shares it).
    ``progress``: called with the iteration index after each step (bench.py's liveness lines)."""
    e, a = 2.0 * eps, 2.0 * alpha
    x0 = x0.to(dtype)
    t = t.to(dtype)
    refs = Refs(gp, vp, ep, x0, t, size)
    adv = x0.clone()
    if random_start:
        adv = torch.clamp(adv + float(np.float32(e)) * start_noise.to(dtype), -1.0, 1.0)
    grads = []
    for _ in range(steps):
        _, g = loss_grad(gp, vp, ep, adv, refs, size)
        if return_grads:
            grads.append(g)
        adv = project_step(adv, x0, g, e, a)
        if progress is not None:
            progress(len(grads) if return_grads else None)
    return (adv, grads) if return_grads else adv


def adam_attack(gp, vp, ep, x0, t, size, steps, lr=0.01, betas=(0.9, 0.999), eps=1e-8,
                dtype=torch.float32, return_trace=False):
    """``optimize_vgg`` literal mode (interpolation.py:743-843): ``Adam([img], lr)`` descending
    L for ``steps`` iterations, no ε-ball, no clamp; img starts at x0 (:607-617).
    ``return_trace``: also the per-iteration losses and gradients (checked against the fixture
    generated by running the reference's own optimize_vgg, oracle/gen_golden_objective.py)."""
    x0 = x0.to(dtype)
    refs = Refs(gp, vp, ep, x0, t.to(dtype), size)
    img = x0.clone().requires_grad_(True)
    opt = torch.optim.Adam([img], lr=lr, betas=betas, eps=eps)
    losses, grads = [], []
    for _ in range(steps):
        opt.zero_grad()
        L = objective(gp, vp, ep, img, refs, size)
        L.backward()
        if return_trace:
            losses.append(float(L))
            grads.append(img.grad.detach().clone())
        opt.step()
    if return_trace:
        return img.detach(), losses, grads
    return img.detach()


def cw_attack(gp, vp, ep, x0, t, size, steps, c=1e-4, lr=0.01, dtype=torch.float32,
              flip_step0=None):
    """torchattacks ``CW.forward`` (commented copy at interpolation.py:98-193) composed with the
    GAN objective in [-1,1] image space: adv = tanh(w) (= 2·½(tanh w + 1) − 1), w0 = atanh(x0)
    (x0 clamped to ±(1 − 2⁻²⁰)); per image L2 = ‖(adv − x0)/2‖² (the [0,1]-space MSE sum of
    :132-134); f_n = the objective L_n (no logits: κ does not apply); cost = Σ L2 + c·Σ f;
    Adam(lr) on w; best-L2 tracking where "success" = L_n(adv) < L_n(x0) (the objective improved on
    the clean image: the GAN analogue of "misclassified", :154-163); early stop every steps//10
    when the cost rises (:166-170).

    ``flip_step0`` (test aid, bool per image): invert the step-0 success decision of those images.
    At step 0 adv = tanh(atanh(x0)) ≈ x0, so "f < f0" compares two equal objectives up to rounding
    and either outcome is a valid fp32 result; the tests run both branches of such a tie."""
    x0 = x0.to(dtype)
    refs = Refs(gp, vp, ep, x0, t.to(dtype), size)
    with torch.no_grad():
        f0 = objective(gp, vp, ep, x0, refs, size, per_image=True)
    lim = 1.0 - 2.0 ** -20
    w = torch.atanh(x0.clamp(-lim, lim)).detach().requires_grad_(True)
    best = x0.clone()
    best_l2 = torch.full((x0.shape[0],), 1e10, dtype=dtype)
    prev = 1e10
    opt = torch.optim.Adam([w], lr=lr)
    for step in range(steps):
        adv = torch.tanh(w)
        cur_l2 = (((adv - x0) / 2) ** 2).reshape(x0.shape[0], -1).sum(dim=1)
        f = objective(gp, vp, ep, adv, refs, size, per_image=True)
        cost = cur_l2.sum() + c * f.sum()
        opt.zero_grad()
        cost.backward()
        opt.step()
        with torch.no_grad():
            succ = f < f0
            if step == 0 and flip_step0 is not None:
                succ = succ ^ flip_step0.to(torch.bool)
            mask = (succ & (best_l2 > cur_l2)).to(dtype)
            best_l2 = mask * cur_l2 + (1 - mask) * best_l2
            m4 = mask.view(-1, 1, 1, 1)
            best = m4 * adv + (1 - m4) * best
        if step % max(steps // 10, 1) == 0:
            if cost.item() > prev:
                return best
            prev = cost.item()
    return best


PATCH_WEIGHTS = dict(lat_t=0.0, lat_o=-1.0, img_rec_t=0.0, vgg_rec_t=0.0, img_o=0.0, vgg_img=0.0)


def patch_attack(gp, vp, ep, img, patch, mask, t, size, max_count, dtype=torch.float32,
                 grad_ctx=None):
    """code/attack/patch/adversarial_patch.py:103-160 (``attack``), batch semantics kept:
    refs under no_grad (:108-112); adv = (1−m)·img + m·patch (:114, no clamp); per iteration the
    loss 0·l_lat_t − 1·l_lat_o + 0·l_img + 0·l_lpips with batch-mean MSEs (:117-125) — the
    objective below with PATCH_WEIGHTS is the per-image form; the batch-mean MSE of the reference
    is the per-image mean averaged over the batch, so its gradient is this one ÷ N —
    backward, patch −= grad (:127-131), adv = clamp((1−m)·img + m·patch, min(img), max(img))
    (:133-134). Returns (adv, patch, rec) with rec = G(E(adv')) of the last iteration's input.
    ``grad_ctx`` (tests): a context-manager factory entered around each gradient evaluation only
    (e.g. encoder_ref.forced_masks of a device run), not around the target precompute."""
    img, patch, mask, t = (z.to(dtype) for z in (img, patch, mask, t))
    refs = Refs(gp, vp, ep, img, t, size)
    patch = patch.clone()
    adv = (1 - mask) * img + mask * patch
    lo, hi = torch.min(img), torch.max(img)
    n = img.shape[0]
    rec = None
    for it in range(max_count):
        x = adv.detach().requires_grad_(True)
        with (grad_ctx() if grad_ctx is not None else contextlib.nullcontext()):
            L = objective(gp, vp, ep, x, refs, size, weights=PATCH_WEIGHTS, per_image=True)
            (g,) = torch.autograd.grad(L.sum() / n, x)
        with torch.no_grad():
            if it == max_count - 1:  # adv_img_rec: the last iteration's reconstruction
                pf = max(1, size // 256)
                xp = F.avg_pool2d(adv, pf) if pf > 1 else adv
                rec = stylegan2_ref.synthesis(gp, encoder_ref.apply(ep, xp, size), size)
            patch = patch - g
            adv = torch.clamp((1 - mask) * img + mask * patch, lo, hi)
    return adv.detach(), patch.detach(), rec
