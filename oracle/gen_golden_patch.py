"""Pin the patch attack, patch_white_box and the partial-fusion sweep to the REFERENCE's own code
(build container only; TEST INFRASTRUCTURE, see oracle/__init__).

    python oracle/gen_golden_patch.py     # writes tests/golden/{patch,fusion}_golden.npz

Like ``gen_golden_objective.py``, each function is taken out of its reference file with ``ast``
and executed unchanged through ``oracle/refexec.py`` — NOT a sandbox: a manual step in the build
container (``MIA_EXEC_REFERENCE=1``) — with the oracle's networks (fp64) where the reference fills
in un-vendored modules:

* ``attack`` — ``code/attack/patch/adversarial_patch.py:94-160`` (the patch optimisation:
  ``patch -= ∇loss`` with loss = −MSE(E(x0'), E(x')), composite + clamp to the batch's
  min / max). ``generator`` → ``oracle.stylegan2_ref.synthesis`` (``.size`` 256), ``encoder`` →
  ``oracle.encoder_ref.apply`` (e4e), ``vgg`` → ``oracle.vgg_ref.vgg_forward``; ``Variable`` is
  ``torch.autograd.Variable``; ``args.max_count`` = 3, ``args.save_img`` False. Recorded: the
  final patch / adversarial image / reconstruction (strided slices + fp64 projections, the patch
  region in full) and the 'Loss:%.5f' lines the function appends to ``w_loss.txt``.
* ``patch_white_box`` — ``code/attack/attack_main2.py:413-433`` in fp32 (elementwise: the device
  result must be bit-identical); recorded in full at 64².
* ``partial_adv_fusion_arithmetic`` + ``interpolation`` — ``code/attack/interpolation.py:921-977``
  and ``:658-669`` with ``drawer`` → an oracle drawer whose ``generate_img(w, latents_type="w")``
  is the church generator (256², 14 layers, ``make_generator_weights(256, seed=0)``, W repeated
  over the layers, truncation 1 — ``style_fusion_simple.py:128-139``); the globals the function
  reads from its module (``batch_idx``, ``args``, ``drawer``) are supplied. Recorded: the M + 1
  fused images (slices + projections).

Inputs come from ``tests/golden_inputs.py`` (seeded). Only outputs are stored.
"""
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gfa_import  # noqa: E402,F401
from gfa_amd.weights import make_generator_weights  # noqa: E402
from golden_inputs import (FUSION, PATCH, SIZE, SLICE, fusion_latents, networks,  # noqa: E402
                           patch_inputs, projections)
from oracle import encoder_ref, refexec, stylegan2_ref, vgg_ref  # noqa: E402

REF = "/root/reference/code"
PATCH_FILE = os.path.join(REF, "attack", "patch", "adversarial_patch.py")
MAIN2_FILE = os.path.join(REF, "attack", "attack_main2.py")
INTERP_FILE = os.path.join(REF, "attack", "interpolation.py")
OUT_PATCH = os.path.join(ROOT, "tests", "golden", "patch_golden.npz")
OUT_FUSION = os.path.join(ROOT, "tests", "golden", "fusion_golden.npz")
WB_SIZE, WB_N = 64, 3


class _Generator:
    def __init__(self, gp, size=SIZE):
        self.gp, self.size = gp, size

    def __call__(self, styles, input_is_latent=False, randomize_noise=True, return_latents=False):
        assert input_is_latent and not randomize_noise and return_latents
        return stylegan2_ref.synthesis(self.gp, styles[0], self.size), styles[0]


def _proj(t, probes):
    return np.array([float((p * t.double()).sum()) for p in probes])


def gen_patch():
    gp, vp, ep = networks("e4e")
    img, patch, mask, tgt = (t.double() for t in patch_inputs())
    P = PATCH
    with tempfile.TemporaryDirectory() as workdir:
        ns = refexec.execute(PATCH_FILE, ["attack"], workdir, Variable=torch.autograd.Variable)
        args = types.SimpleNamespace(max_count=P["max_count"], save_img=False)
        p = patch.clone()
        adv, m, p_out, rec = ns["attack"](
            img, p, mask, _Generator(gp), lambda x: encoder_ref.apply(ep, x, SIZE),
            lambda x: tuple(vgg_ref.vgg_forward(vp, x)), "cpu", args, tgt, workdir, 0, 0)
        losses = [float(s.split(":")[1])
                  for s in open(os.path.join(workdir, "w_loss.txt")).read().split()]
    assert len(losses) == P["max_count"]
    probes = projections(SIZE, P["n"])
    ys, xs = slice(P["y0"], P["y0"] + P["side"]), slice(P["x0"], P["x0"] + P["side"])
    out = {"losses": np.array(losses), **{f"P_{k}": v for k, v in P.items()}}
    for nm, t in (("patch", p_out), ("adv", adv), ("rec", rec)):
        t = t.detach()
        out[f"{nm}/slice"] = t[SLICE].numpy()
        out[f"{nm}/proj"] = _proj(t, probes)
        out[f"{nm}/region"] = t[:, :, ys, xs].float().numpy()
    out["patch/delta_absmax"] = float((p_out.detach() - patch).abs().max())
    print("patch losses", losses, "Δpatch absmax", out["patch/delta_absmax"])
    # patch_white_box (fp32, full)
    g = torch.Generator().manual_seed(611)
    inputs = (torch.rand(WB_N, 3, WB_SIZE, WB_SIZE, generator=g) * 2 - 1) * 0.8
    wb_mask = torch.zeros(1, 3, WB_SIZE, WB_SIZE)
    wb_mask[:, :, 10:30, 20:44] = 1.0
    wb_mask[:, :, 30:34, 20:44] = 0.5  # a soft edge
    wb_patch = (torch.rand(1, 3, WB_SIZE, WB_SIZE, generator=g) * 2.4 - 1.2) * (wb_mask > 0)
    with tempfile.TemporaryDirectory() as workdir:
        ns = refexec.execute(MAIN2_FILE, ["patch_white_box"], workdir)
        wb = ns["patch_white_box"](inputs, wb_mask, wb_patch)
    out.update({"wb/inputs": inputs.numpy(), "wb/mask": wb_mask.numpy(),
                "wb/patch": wb_patch.numpy(), "wb/out": wb.numpy()})
    np.savez_compressed(OUT_PATCH, **out)
    print("wrote", OUT_PATCH, os.path.getsize(OUT_PATCH), "bytes")


class _OracleDrawer:
    """StyleFusionSimple('church') restated on the oracle generator: generate_img of a W latent
    (1, 512) → (image, [image]) (the feature list's last entry; the sweep never reads it)."""

    def __init__(self, gp, n_latent=14):
        self.gp, self.n_latent = gp, n_latent

    def generate_img(self, base_latent, latents_type="z"):
        assert latents_type == "w" and tuple(base_latent.shape) == (1, 512)
        w = base_latent.unsqueeze(1).repeat(1, self.n_latent, 1)
        img = stylegan2_ref.synthesis(self.gp, w, SIZE)
        return img, [img]


def gen_fusion():
    gp = {k: v.double() for k, v in make_generator_weights(SIZE, seed=0).items()}
    W, Wa = (t.double() for t in fusion_latents())
    M = FUSION["m"]
    with tempfile.TemporaryDirectory() as workdir:
        ns = refexec.execute(INTERP_FILE, ["interpolation", "partial_adv_fusion_arithmetic"],
                             workdir, batch_idx=0, drawer=_OracleDrawer(gp),
                             args=types.SimpleNamespace(save_img=False))
        inputs = torch.zeros(M, 3, 8, 8)
        with torch.no_grad():
            fused = ns["partial_adv_fusion_arithmetic"](workdir, inputs, inputs + 1, W, Wa)
    assert tuple(fused.shape) == (M + 1, 3, SIZE, SIZE)
    probes = projections(SIZE, M + 1)
    out = {"fused/slice": fused[SLICE].numpy(), "fused/proj": _proj(fused, probes),
           **{f"F_{k}": v for k, v in FUSION.items()}}
    np.savez_compressed(OUT_FUSION, **out)
    print("wrote", OUT_FUSION, os.path.getsize(OUT_FUSION), "bytes")


def main():
    torch.set_num_threads(os.cpu_count() or 1)
    which = sys.argv[1:] or ["patch", "fusion"]
    if "fusion" in which:
        gen_fusion()
    if "patch" in which:
        gen_patch()


if __name__ == "__main__":
    main()
