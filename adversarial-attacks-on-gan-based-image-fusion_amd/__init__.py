"""MI355X-native adversarial-perturbation engine for GAN image fusion (import name ``gfa_amd``).

Hot path: PGD/FGSM through encoder → StyleGAN2 synthesis → VGG feature loss → ∇ pixels →
sign-project, all on hand-written gfx950 HIP kernels in ``libmiattack.so`` (C ABI:
``include/miattack.h``). Public API:

    from gfa_amd import attack, build_net, StyleFusionSimple
    net = build_net(256)                       # seeded synthetic pSp + VGG
    adv = attack(net, imgs, eps=8/255, steps=20, target=t)

Submodules import lazily so the package can be imported (and the library inspected) on a host
without a GPU; any compute call without the library or a GPU raises.
"""
__all__ = ["attack", "fgsm", "build_net", "vgg16", "get_latents", "StyleFusionSimple",
           "interpolation", "partial_adv_fusion_arithmetic", "attack_distributed",
           "patch_attack", "patch_white_box"]


def __getattr__(name):
    if name in ("attack", "fgsm", "AttackEngine"):
        from . import pgd as _a
        return getattr(_a, name)
    if name in ("build_net", "vgg16", "get_latents", "PSPNet", "Decoder", "Encoder", "VGGBase",
                "MappingNet"):
        from . import networks as _n
        return getattr(_n, name)
    if name in ("StyleFusionSimple", "interpolation", "partial_adv_fusion_arithmetic"):
        from . import style_fusion_simple as _f
        return getattr(_f, name)
    if name in ("patch_attack", "patch_white_box"):
        from . import patch as _p
        return _p.attack if name == "patch_attack" else _p.patch_white_box
    if name == "attack_distributed":
        from .dist import attack_distributed
        return attack_distributed
    raise AttributeError(name)
