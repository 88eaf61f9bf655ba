"""Fusion entry point: ``StyleFusionSimple`` and the arithmetic fusion, on the device networks.

Mirrors ``code/style_fusion_simple.py:25-177``: the same constructor,
method names, argument meaning and return shapes, over this package's StyleGAN2 (SynthesisNet +
MappingNet) instead of the un-vendored ``SFGenerator_hook``. The semantic-part blender
(``SFHierarchy*`` + fusion nets, :73-80) is an un-vendored dependency whose weights are not
available offline: only the ``"all"`` part is supported, which is what the reference's arithmetic
fusion uses (``interpolation.py:658-669``); asking for fusion nets raises.

Style vectors are lists of per-layer fp32 (N, Cin) tensors in generator forward order (conv1,
to_rgb1, then per resolution: up-conv, conv, to_rgb). ``s_to_image`` returns ``(img, features)``
where features are the StyledConv activations (NCHW views of the device buffers, compute dtype).
"""
import torch

from .networks import Decoder
from .weights import STYLE_DIM, make_generator_weights, n_latent_for
from .workspace import Workspace

# style_fusion_simple.py:28-39
STYLEGAN_TYPES = {"ffhq": (1024, 18, 0.7), "car": (512, 16, 0.5), "church": (256, 14, 0.5)}

# semantic parts of generate_img (style_fusion_simple.py:89-104); only "all" can be blended here
_SWAPS = [("hair", ["bg_hair_clothes", "hair"]),
          ("face", ["face", "eyes", "skin_mouth", "mouth", "skin", "shirt"]),
          ("background", ["background", "background_top", "background_bottom", "bg"]),
          ("all", ["all"]), ("mouth", ["skin_mouth", "face"]), ("eyes", ["eyes", "face"]),
          ("wheels", ["wheels"]), ("car", ["car", "body", "wheels", "car_body"]),
          ("bg_top", ["background_top"]), ("bg_bottom", ["background_bottom"])]


def _load_generator(stylegan_weights, GAN, size, seed):
    """g_ema state dict from a checkpoint path (weights_only load), a dict, a GAN module, or —
    with neither (no checkpoints offline) — seeded synthetic weights of the right size."""
    if GAN is not None:
        return {k: v.detach().cpu() for k, v in GAN.state_dict().items()}
    if isinstance(stylegan_weights, dict):
        return stylegan_weights.get("g_ema", stylegan_weights)
    if stylegan_weights:
        ckpt = torch.load(stylegan_weights, map_location="cpu", weights_only=True)
        return ckpt["g_ema"] if "g_ema" in ckpt else ckpt
    return make_generator_weights(size, seed=seed)


class StyleFusionSimple:
    def __init__(self, stylegan_type, stylegan_weights, fusion_nets_weights, device, GAN=None, *,
                 dtype=torch.float32, seed=0, n_mean_latent=4096):
        if stylegan_type not in STYLEGAN_TYPES:
            raise ValueError(f"stylegan_type must be one of {sorted(STYLEGAN_TYPES)}")
        if fusion_nets_weights:
            raise NotImplementedError(
                "SFHierarchy fusion nets (style_fusion_simple.py:73-80) are an un-vendored "
                "dependency; only the 'all' blend (arithmetic fusion) is available")
        self.stylegan_type = stylegan_type
        self.stylegan_size, self.stylegan_layers, self.truncation = STYLEGAN_TYPES[stylegan_type]
        self.device = torch.device(device)
        params = _load_generator(stylegan_weights, GAN, self.stylegan_size, seed)
        self.original_net = Decoder(params, self.stylegan_size, dtype=dtype, device=self.device)
        assert self.original_net.n_latent == self.stylegan_layers == n_latent_for(self.stylegan_size)
        if self.original_net.mapping is None:
            raise ValueError("the generator weights lack the mapping MLP (style.{1..8}.*)")
        self.mean_latent = self.original_net.mapping.mean_latent(n_mean_latent, seed=seed)
        self._ws = Workspace(self.device)

    # ---- latents ------------------------------------------------------------------------------
    def seed_to_z(self, seed):
        """style_fusion_simple.py:106-109: the seed[1]-th draw after seeding with seed[0]
        (host torch.Generator, so draws are identical on every platform)."""
        g = torch.Generator().manual_seed(int(seed[0]))
        z = torch.randn((int(seed[1]) + 1, 1, STYLE_DIM), generator=g)
        return z[int(seed[1])].to(self.device)

    def z_to_w_plus(self, z):
        """:117-121: mapping, truncation toward mean_latent, repeated over the layers."""
        w = self.original_net.mapping(z)
        w = self.original_net._truncate(w, self.truncation, self.mean_latent)
        return w.unsqueeze(1).repeat(1, self.stylegan_layers, 1)

    def w_plus_to_s(self, w_plus, truncation):
        """:123-126: style vectors of W+ (after truncation toward mean_latent)."""
        w_plus = w_plus.to(self.device, torch.float32).contiguous()
        w_plus = self.original_net._truncate(w_plus, truncation, self.mean_latent).contiguous()
        return self.original_net.impl.style_vectors(w_plus, self._ws)

    def z_to_s(self, z):
        """:111-114."""
        return self.w_plus_to_s(self.z_to_w_plus(z), truncation=1)

    def general_latent_to_s(self, l, latent_type):
        """:128-139 (same assertions)."""
        assert latent_type in ["z", "w", "w+", "s"]
        if latent_type == "z":
            assert l.size() == (1, 512)
            return self.z_to_s(l)
        if latent_type in ("w", "w+"):
            assert l.size() == (1, 512) or l.size() == (1, self.stylegan_layers, 512)
            if l.dim() == 2:
                return self.w_plus_to_s(l.unsqueeze(0).repeat(1, self.stylegan_layers, 1), 1)
            return self.w_plus_to_s(l, truncation=1)
        return l

    # ---- images -------------------------------------------------------------------------------
    def s_to_image(self, s):
        """:141-153: (img (N,3,S,S) fp32, StyledConv features)."""
        G = self.original_net.impl
        img = G.forward_styles(s, self._ws).clone()
        feats = [L["_pre"].permute(0, 3, 1, 2) for L in G.convs]
        return img, feats

    def w_plus_to_image(self, w_plus):
        return self.s_to_image(self.w_plus_to_s(w_plus, truncation=1))

    def z_to_image(self, z):
        return self.s_to_image(self.z_to_s(z))

    def s_dict_to_image(self, s_dict):
        """:163-165 with the 'all' blender (the only part without fusion nets)."""
        extra = set(s_dict) - {"all"}
        if extra:
            raise NotImplementedError(f"parts {sorted(extra)} need SFHierarchy fusion nets")
        return self.s_to_image(s_dict["all"])

    def w_plus_dict_to_image(self, w_plus_dict, truncation=1):
        return self.s_dict_to_image({k: self.w_plus_to_s(v, truncation=truncation)
                                     for k, v in w_plus_dict.items()})

    def z_dict_to_image(self, z_dict):
        return self.s_dict_to_image({k: self.z_to_s(v) for k, v in z_dict.items()})

    def generate_img(self, base_latent, latents_type="z", hair=None, face=None, background=None,
                     all=None, mouth=None, eyes=None, wheels=None, car=None, bg_top=None,
                     bg_bottom=None):
        """:82-104: base latent for every active part, then per-part swaps."""
        s_dict = {"all": self.general_latent_to_s(base_latent, latents_type)}
        parts = dict(hair=hair, face=face, background=background, all=all, mouth=mouth, eyes=eyes,
                     wheels=wheels, car=car, bg_top=bg_top, bg_bottom=bg_bottom)
        for name, keys in _SWAPS:
            value = parts[name]
            if value is None:
                continue
            for k in keys:
                s_dict[k] = self.general_latent_to_s(value, latents_type)
        return self.s_dict_to_image(s_dict)


def interpolation(drawer, all_latents, feature_idx=-1):
    """Arithmetic fusion (interpolation.py:658-669): the image of the mean W latent, the image of
    every latent, and the chosen feature of each. Returns (I_fused, I_all, features)."""
    avg = all_latents.mean(dim=0, keepdim=True) if all_latents.shape[0] > 1 else all_latents
    I_fused, _ = drawer.generate_img(avg, latents_type="w")
    I_all, feats = [], []
    for i in range(all_latents.shape[0]):
        img, inner = drawer.generate_img(all_latents[i].unsqueeze(0), latents_type="w")
        I_all.append(img)
        feats.append(inner[feature_idx].float().clone())
    return I_fused, torch.cat(I_all, dim=0), torch.cat(feats, dim=0)


def partial_adv_fusion_arithmetic(drawer, inputs, adv_inputs, all_latents, all_adv_latents):
    """Partial-fusion sweep (interpolation.py:921-977): for j = 0 … M−1 the arithmetic fusion with
    only latent j replaced by its adversarial one, then with all of them replaced. Returns the
    M + 1 fused images (M+1, 3, S, S) in that order. The image files of ``args.save_img`` are I/O
    and out of scope; ``inputs`` / ``adv_inputs`` only feed those files in the reference, so they
    are checked for shape and otherwise unused."""
    M = all_adv_latents.shape[0]
    if tuple(all_latents.shape) != tuple(all_adv_latents.shape):
        raise ValueError("all_latents and all_adv_latents must have the same shape")
    if inputs is not None and adv_inputs is not None and inputs.shape[0] != adv_inputs.shape[0]:
        raise ValueError("inputs and adv_inputs must hold the same images")
    out = []
    for j in range(M + 1):
        if j < M:
            lat = all_latents.clone()
            lat[j] = all_adv_latents[j]
        else:
            lat = all_adv_latents.clone()
        fused, _, _ = interpolation(drawer, lat, feature_idx=-1)
        out.append(fused)
    return torch.cat(out, dim=0)
