"""Seeded inputs and probes of the committed golden fixtures (tests/golden/*.npz). The fixture
generators under oracle/ import these, and the tests regenerate the same inputs from them, so the
GPU box never imports a generator script."""
import torch

SIZE = 256
SEEDS = dict(x0=501, t=502, gen=0, vgg=1234, enc=1)
SLICE = (slice(None), slice(None), slice(None, None, 4), slice(None, None, 4))
N_PROJ = 4


def projections(size, n=1):
    """Seeded ±1 probe tensors: Σ probe·v (fp64) pins a whole tensor in 4 numbers."""
    g = torch.Generator().manual_seed(777)
    return [(torch.randint(0, 2, (n, 3, size, size), generator=g) * 2 - 1).double()
            for _ in range(N_PROJ)]


def networks(kind, dtype=torch.float64, size=SIZE):
    """The oracle parameter dicts (generator, VGG positional, encoder) of the fixtures, seeded
    (``gfa_amd.weights``): ``kind`` 'e4e' or 'linear' picks the encoder."""
    import gfa_import  # noqa: F401
    from gfa_amd.weights import (make_e4e_weights, make_encoder_weights, make_generator_weights,
                                 make_vgg_weights)
    from oracle import vgg_ref
    gp = {k: v.to(dtype) for k, v in make_generator_weights(size, seed=SEEDS["gen"]).items()}
    vp = {k: (w.to(dtype), b.to(dtype))
          for k, (w, b) in vgg_ref.load_positional(make_vgg_weights(SEEDS["vgg"])).items()}
    raw = (make_e4e_weights(size, seed=SEEDS["enc"]) if kind == "e4e"
           else make_encoder_weights(size, seed=SEEDS["enc"]))
    ep = {k: (v.to(dtype) if torch.is_tensor(v) else v) for k, v in raw.items()}
    return gp, vp, ep


def seeded_pair(size=SIZE):
    g = torch.Generator().manual_seed(SEEDS["x0"])
    x0 = torch.rand(1, 3, size, size, generator=g) * 2 - 1
    g = torch.Generator().manual_seed(SEEDS["t"])
    t = torch.rand(1, 3, size, size, generator=g) * 2 - 1
    return x0, t


# the patch-attack fixture (tests/golden/patch_golden.npz, oracle/gen_golden_patch.py)
PATCH = dict(n=2, side=48, y0=40, x0=96, max_count=3, seed_img=601, seed_patch=602, seed_tgt=603)


def patch_inputs(size=SIZE):
    """(img, patch, mask, target) of the patch fixture: two seeded images in [-0.9, 0.9], a square
    patch of U(-1,1) in a 0/1 mask (the batch-shaped tensors square_transform returns)."""
    P = PATCH
    g = torch.Generator().manual_seed(P["seed_img"])
    img = (torch.rand(P["n"], 3, size, size, generator=g) * 2 - 1) * 0.9
    m = torch.zeros(P["n"], 3, size, size)
    m[:, :, P["y0"]:P["y0"] + P["side"], P["x0"]:P["x0"] + P["side"]] = 1.0
    g = torch.Generator().manual_seed(P["seed_patch"])
    patch = (torch.rand(P["n"], 3, size, size, generator=g) * 2 - 1) * m
    g = torch.Generator().manual_seed(P["seed_tgt"])
    tgt = torch.rand(P["n"], 3, size, size, generator=g) * 2 - 1
    return img, patch, m, tgt


# the partial-fusion fixture (tests/golden/fusion_golden.npz): M W latents (1, 512) from seeds
FUSION = dict(m=2, seed_w=701, seed_adv=702, adv_scale=0.05)


def fusion_latents():
    g = torch.Generator().manual_seed(FUSION["seed_w"])
    W = torch.randn(FUSION["m"], 512, generator=g) * 0.5
    g = torch.Generator().manual_seed(FUSION["seed_adv"])
    Wa = W + FUSION["adv_scale"] * torch.randn(W.shape, generator=g)
    return W, Wa
