"""Adversarial patch attack (code/attack/patch/adversarial_patch.py:103-160,
attack_main2.py:413-420) on the GPU against oracle.attack_ref.patch_attack / torch fp32 ops."""
import numpy as np
import pytest
import torch

import gfa_amd
from gfa_amd import networks, ops
from gpu_helpers import e4e_masks, seeded, to64
from oracle import attack_ref, encoder_ref, vgg_ref

pytestmark = pytest.mark.gpu


def _square(N, S, side, y0, x0):
    """The tensors square_transform returns (un-vendored): a batch-shaped 0/1 mask and a patch of
    U(-1,1) inside it."""
    m = torch.zeros(N, 3, S, S)
    m[:, :, y0:y0 + side, x0:x0 + side] = 1.0
    p = seeded(41, (N, 3, S, S)) * m
    return p, m


@pytest.mark.parametrize("frac_mask", [False, True])
def test_patch_update_bit_exact(cuda, frac_mask):
    """mia_patch_update vs adversarial_patch.py:131-134 in torch fp32 (separately rounded ops)."""
    N, S = 3, 40
    img = seeded(1, (N, 3, S, S))
    g = seeded(2, (N, 3, S, S)) * 1e-2
    patch, mask = _square(N, S, 12, 5, 9)
    if frac_mask:
        mask = (seeded(3, mask.shape) + 1) / 2
    lo, hi = float(img.min()), float(img.max())
    want_p = patch - g
    want = torch.clamp((1 - mask) * img + mask * want_p, lo, hi)
    pd, adv = patch.to(cuda), torch.empty(N, 3, S, S, device=cuda)
    ops.patch_update(pd, g.to(cuda), img.to(cuda), mask.to(cuda), adv, lo, hi)
    torch.cuda.synchronize()
    assert torch.equal(pd.cpu(), want_p) and torch.equal(adv.cpu(), want)
    # patch_white_box: one shared patch / mask, per-image min / max (attack_main2.py:413-420)
    p1, m1 = patch[:1], mask[:1]
    want = torch.cat([torch.clamp((1 - m1) * img[i] + m1 * p1, img[i].min(), img[i].max())
                      for i in range(N)])
    got = gfa_amd.patch_white_box(img.to(cuda), m1.to(cuda), p1.to(cuda)).cpu()
    assert torch.equal(got, want)


def _params(net):
    p = net.params
    return p["generator"], vgg_ref.load_positional(p["vgg"]), p["encoder"]


def test_patch_attack_vs_oracle_linear_encoder(cuda):
    """3 iterations at 32² with the linear stand-in encoder (no activation branches): the
    patch's total change and the final images vs the fp64 oracle."""
    S, N, it = 32, 2, 3
    net = networks.build_net(S, seed=3, device=cuda)
    img = seeded(5, (N, 3, S, S)) * 0.9
    patch, mask = _square(N, S, 10, 4, 7)
    adv, m, p, rec = gfa_amd.patch_attack(img.to(cuda), patch.to(cuda), mask.to(cuda), net, it)
    gp, vp, ep = to64(_params(net))
    a_ref, p_ref, r_ref = attack_ref.patch_attack(gp, vp, ep, img.double(), patch.double(),
                                                  mask.double(), img.double(), S, it,
                                                  dtype=torch.float64)
    dp, dp_ref = p.cpu().double() - patch.double(), p_ref - patch.double()
    rel = ((dp - dp_ref).norm() / dp_ref.norm()).item()
    print(f"patch change vs oracle: rel {rel:.2e}, |Δpatch| {dp_ref.abs().max():.3e}")
    assert dp_ref.abs().max() > 0 and rel < 1e-4
    assert (adv.cpu().double() - a_ref).abs().max() < 1e-5
    assert (rec.cpu().double() - r_ref).abs().max() < 1e-4
    assert torch.equal(m.cpu(), mask)
    lo, hi = img.min(), img.max()
    assert adv.min() >= lo and adv.max() <= hi


def test_patch_attack_e4e_first_step_branch_forced(cuda):
    """One iteration at 256² with the e4e encoder (the reference's network): the patch update vs
    the fp64 oracle on the device run's encoder branches (encoder_ref.forced_masks)."""
    S, N = 256, 1
    net = networks.build_net(S, seed=0, device=cuda, encoder="e4e")
    img = seeded(6, (N, 3, S, S)) * 0.9
    patch, mask = _square(N, S, 64, 100, 30)
    # the branches of the gradient pass's own forward (the 3rd encoder forward: prepare encodes
    # t and x0 first; the final rec pass re-encodes the same composite)
    enc = net.encoder.impl
    seen = []
    fwd = enc.forward_nhwc

    def capture(xin, ws, tag="e"):
        lat = fwd(xin, ws, tag)
        seen.append(e4e_masks(enc))
        return lat
    enc.forward_nhwc = capture
    try:
        _, _, p, _ = gfa_amd.patch_attack(img.to(cuda), patch.to(cuda), mask.to(cuda), net, 1)
    finally:
        del enc.forward_nhwc
    assert len(seen) == 4, len(seen)
    masks = seen[2]
    gp, vp, ep = to64(_params(net))
    _, p_ref, _ = attack_ref.patch_attack(gp, vp, ep, img.double(), patch.double(),
                                          mask.double(), img.double(), S, 1, dtype=torch.float64,
                                          grad_ctx=lambda: encoder_ref.forced_masks(masks))
    dp, dp_ref = p.cpu().double() - patch.double(), p_ref - patch.double()
    rel = ((dp - dp_ref).norm() / dp_ref.norm()).item()
    print(f"e4e patch step vs oracle: rel {rel:.2e}")
    assert rel < 1e-4


# ---- against the reference's own code (tests/golden/patch_golden.npz, oracle/gen_golden_patch.py)

def test_patch_white_box_matches_reference_output(cuda):
    """gfa_amd.patch_white_box on the fixture's inputs (3 images at 64², a soft-edged mask) is
    bit-identical to the reference's own patch_white_box (attack_main2.py:413-433) output."""
    import os
    from conftest import GOLDEN
    pg = np.load(os.path.join(GOLDEN, "patch_golden.npz"))
    x, m, p = (torch.from_numpy(pg[f"wb/{k}"]) for k in ("inputs", "mask", "patch"))
    got = gfa_amd.patch_white_box(x.to(cuda), m.to(cuda), p.to(cuda)).cpu()
    assert torch.equal(got, torch.from_numpy(pg["wb/out"]))


def test_patch_attack_matches_reference_attack(cuda):
    """gfa_amd.patch_attack (fp32, e4e, 256², 2 images, 3 iterations) vs the reference's own
    adversarial_patch.attack run in fp64 with the oracle networks: the patch's change inside the
    mask (Δpatch ≈ 3e-3) within 2e-3 in norm (unforced e4e branches: activations within fp32
    rounding of 0 may take the other PReLU branch), the adversarial image within 1e-5 and the
    reconstruction within 1e-3 max-abs, all projections within 1e-3."""
    import os
    import golden_inputs as gi
    from conftest import GOLDEN
    pg = np.load(os.path.join(GOLDEN, "patch_golden.npz"))
    P = gi.PATCH
    net = networks.build_net(gi.SIZE, seed=gi.SEEDS["gen"], device=cuda, encoder="e4e",
                             vgg_seed=gi.SEEDS["vgg"])
    img, patch, mask, tgt = gi.patch_inputs()
    adv, m, p, rec = gfa_amd.patch_attack(img.to(cuda), patch.to(cuda), mask.to(cuda), net,
                                          P["max_count"], target_img=tgt.to(cuda))
    ys, xs = slice(P["y0"], P["y0"] + P["side"]), slice(P["x0"], P["x0"] + P["side"])
    p, adv, rec = p.cpu().double(), adv.cpu().double(), rec.cpu().double()
    dp = p[:, :, ys, xs] - patch.double()[:, :, ys, xs]
    dp_ref = torch.from_numpy(pg["patch/region"]).double() - patch.double()[:, :, ys, xs]
    rel = ((dp - dp_ref).norm() / dp_ref.norm()).item()
    print(f"patch change vs reference attack: rel {rel:.2e} (|Δ| {dp_ref.abs().max():.2e})")
    assert dp_ref.abs().max() > 1e-3 and rel < 2e-3
    assert (adv[:, :, ys, xs] - torch.from_numpy(pg["adv/region"]).double()).abs().max() < 1e-5
    assert (adv[gi.SLICE] - torch.from_numpy(pg["adv/slice"])).abs().max() < 1e-5
    assert (rec[gi.SLICE] - torch.from_numpy(pg["rec/slice"])).abs().max() < 1e-3
    probes = gi.projections(gi.SIZE, P["n"])
    for nm, t in (("adv", adv), ("rec", rec)):
        got = torch.tensor([float((q * t).sum()) for q in probes])
        ref = torch.from_numpy(pg[f"{nm}/proj"])
        assert ((got - ref).abs().max() / ref.abs().max()).item() < 1e-3, nm
    assert torch.equal(m.cpu(), mask)
