"""Seeded synthetic weights for the three networks on the attack path.

There are no checkpoints offline, so every network is built from a seed on the
host (CPU, ``torch.Generator``) and copied to the device. The same dicts feed the product path and
the CPU oracle, so parity tests compare like with like.

Names follow the state-dict keys of the modules the reference calls:

* StyleGAN2 generator (rosinality ``model.py`` API, used as ``net.decoder`` at
  ``code/attack/attack_main2.py:619-621`` and as ``SFGenerator_hook`` at
  ``code/style_fusion_simple.py:51``): ``input.input``, ``conv1.*``, ``to_rgb1.*``, ``convs.{i}.*``,
  ``to_rgbs.{i}.*``, ``noises.noise_{i}``, and the mapping MLP ``style.{1..8}.*`` (used only by the
  fusion entry point's z → W path, ``style_fusion_simple.py:110-119``; the attack calls the
  decoder with ``input_is_latent=True``, ``attack_main2.py:619``).
* VGG16 trunk (``code/vgg.py:12-39``): positional list of 13 convs, loaded like
  ``VGGBase.load_pretrained_layers`` (``code/vgg.py:66-76``).
* Encoder: e4e ``Encoder4Editing(50, 'ir_se')`` (``code/utils/model_utils.py:24``; state-dict keys
  of that module: ``input_layer.*``, ``body.{i}.*``, ``styles.{i}.*``, ``latlayer{1,2}.*``), or the
  deterministic linear stand-in of SURVEY.md §7 step 1 (``enc.*``).
"""
import math

import torch

STYLE_DIM = 512
N_MLP = 8          # rosinality Generator(n_mlp=8) (style_fusion_simple.py:51: SFGenerator_hook(.., 8))
LR_MLP = 0.01      # EqualLinear lr_mul of the mapping layers


def generator_channels(channel_multiplier=2):
    """rosinality Generator.channels for channel_multiplier."""
    cm = channel_multiplier
    return {4: 512, 8: 512, 16: 512, 32: 512, 64: 256 * cm, 128: 128 * cm, 256: 64 * cm,
            512: 32 * cm, 1024: 16 * cm}


def n_latent_for(size):
    """n_latent = 2*log2(size) - 2 (14/16/18 for 256/512/1024: style_fusion_simple.py:31,35,39)."""
    log_size = int(math.log2(size))
    assert 2 ** log_size == size and size >= 8
    return log_size * 2 - 2


def generator_layout(size, channel_multiplier=2):
    """Per-layer description of the synthesis network.

    Returns (convs, torgbs): lists of dicts. Each conv: name, cin, cout, res (output resolution),
    up (bool), latent (index into w+), noise (index of noises.noise_i). Each torgb: name, cin,
    res, latent, has_skip. Order and latent/noise indexing follow rosinality Generator.forward
    (latent[:,0] → conv1, latent[:,1] → to_rgb1, then (i, i+1, i+2) per resolution).
    """
    ch = generator_channels(channel_multiplier)
    log_size = int(math.log2(size))
    convs = [dict(name="conv1", cin=ch[4], cout=ch[4], res=4, up=False, latent=0, noise=0)]
    torgbs = [dict(name="to_rgb1", cin=ch[4], res=4, latent=1, has_skip=False)]
    in_ch = ch[4]
    li = 1
    ci = 0
    for i in range(3, log_size + 1):
        r = 2 ** i
        out_ch = ch[r]
        convs.append(dict(name=f"convs.{ci}", cin=in_ch, cout=out_ch, res=r, up=True, latent=li,
                          noise=2 * (i - 3) + 1))
        convs.append(dict(name=f"convs.{ci + 1}", cin=out_ch, cout=out_ch, res=r, up=False,
                          latent=li + 1, noise=2 * (i - 3) + 2))
        torgbs.append(dict(name=f"to_rgbs.{(ci) // 2}", cin=out_ch, res=r, latent=li + 2,
                           has_skip=True))
        ci += 2
        li += 2
        in_ch = out_ch
    return convs, torgbs


def make_generator_weights(size, seed=0, channel_multiplier=2, noise_weight=0.1,
                           bias_std=0.1):
    """Seeded rosinality-layout generator weights (fp32, CPU).

    Initialisation follows rosinality (weights ~ N(0,1), runtime equalised-lr scaling; modulation
    bias = 1). Conv/ToRGB biases and noise strengths are made non-zero (bias_std, noise_weight) so
    every term of the synthesis contributes.
    """
    g = torch.Generator().manual_seed(int(seed))
    ch = generator_channels(channel_multiplier)
    convs, torgbs = generator_layout(size, channel_multiplier)
    p = {}
    p["input.input"] = torch.randn(1, ch[4], 4, 4, generator=g)

    def modconv(prefix, cin, cout, k):
        p[prefix + ".weight"] = torch.randn(1, cout, cin, k, k, generator=g)
        p[prefix + ".modulation.weight"] = torch.randn(cin, STYLE_DIM, generator=g)
        p[prefix + ".modulation.bias"] = torch.ones(cin) + 0.1 * torch.randn(cin, generator=g)

    for c in convs:
        modconv(c["name"] + ".conv", c["cin"], c["cout"], 3)
        p[c["name"] + ".noise.weight"] = torch.full((1,), float(noise_weight))
        p[c["name"] + ".activate.bias"] = bias_std * torch.randn(c["cout"], generator=g)
    for t in torgbs:
        modconv(t["name"] + ".conv", t["cin"], 3, 1)
        p[t["name"] + ".bias"] = bias_std * torch.randn(1, 3, 1, 1, generator=g)
    log_size = int(math.log2(size))
    for i in range((log_size - 2) * 2 + 1):
        r = 2 ** ((i + 5) // 2)
        p[f"noises.noise_{i}"] = torch.randn(1, 1, r, r, generator=g)
    # mapping MLP (own stream, so the synthesis weights above do not depend on it): EqualLinear
    # stores weight ~ N(0,1)/lr_mul; the bias (0 at rosinality init) is made non-zero here
    gm = torch.Generator().manual_seed(int(seed) + 7919)
    for i in range(1, N_MLP + 1):
        p[f"style.{i}.weight"] = torch.randn(STYLE_DIM, STYLE_DIM, generator=gm) / LR_MLP
        p[f"style.{i}.bias"] = bias_std * torch.randn(STYLE_DIM, generator=gm) / LR_MLP
    return p


# VGG16 feature convs in order (code/vgg.py:12-33); the first 9 are run by VGGBase.forward.
VGG_CONVS = [("conv1_1", 3, 64), ("conv1_2", 64, 64), ("conv2_1", 64, 128), ("conv2_2", 128, 128),
             ("conv3_1", 128, 256), ("conv3_2", 256, 256), ("conv3_3", 256, 256),
             ("conv4_1", 256, 512), ("conv4_2", 512, 512), ("conv4_3", 512, 512),
             ("conv5_1", 512, 512), ("conv5_2", 512, 512), ("conv5_3", 512, 512)]
VGG_USED = 9


def make_vgg_weights(seed=0, n_convs=13):
    """Seeded He-normal VGG16 conv weights, positional order (as a pretrained VGG16 state dict).

    Keys are ``features.{idx}.weight/bias`` with torchvision VGG16 indices; ``VGGBase``-style
    loading is positional (code/vgg.py:70-74), so only the order matters.
    """
    g = torch.Generator().manual_seed(int(seed))
    sd = {}
    idx = 0
    feat_idx = [0, 2, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28]
    for (name, cin, cout), fi in zip(VGG_CONVS[:n_convs], feat_idx):
        std = math.sqrt(2.0 / (cin * 9))
        sd[f"features.{fi}.weight"] = torch.randn(cout, cin, 3, 3, generator=g) * std
        sd[f"features.{fi}.bias"] = 0.05 * torch.randn(cout, generator=g)
        idx += 1
    return sd


ENC_POOL_RES = 16  # the synthetic encoder sees a 16x16 average-pooled image (3*16*16 = 768)


def make_encoder_weights(size, seed=0, start_from_latent_avg=True):
    """Synthetic linear encoder weights (stand-in for e4e).

    E(x) = W_E · vec(avgpool(x, 256/16)) / sqrt(768) + b_E, reshaped to (N, n_latent, 512).
    ``latent_avg`` is exposed for ``get_latents`` (attack_main2.py:137-146) but, like the
    reference's optimize_vgg (interpolation.py:780), the attack objective does not add it.
    """
    g = torch.Generator().manual_seed(int(seed))
    nl = n_latent_for(size)
    d_in = 3 * ENC_POOL_RES * ENC_POOL_RES
    return {
        "enc.weight": torch.randn(nl * STYLE_DIM, d_in, generator=g),
        "enc.bias": 0.1 * torch.randn(nl * STYLE_DIM, generator=g),
        "latent_avg": 0.1 * torch.randn(nl, STYLE_DIM, generator=g),
        "start_from_latent_avg": bool(start_from_latent_avg),
    }


# ---- e4e: Encoder4Editing(50, 'ir_se') ------------------------------------------------------------
E4E_STAGES = [(64, 64, 3), (64, 128, 4), (128, 256, 14), (256, 512, 3)]  # get_blocks(50)
E4E_SE_REDUCTION = 16
E4E_COARSE, E4E_MIDDLE = 3, 7  # Encoder4Editing.coarse_ind / middle_ind


def e4e_units():
    """bottleneck_IR_SE units of the IR-SE50 body in order: (in_channel, depth, stride)
    (get_block: the first unit of a stage has stride 2, the others 1)."""
    units = []
    for cin, depth, n in E4E_STAGES:
        units.append((cin, depth, 2))
        units += [(depth, depth, 1)] * (n - 1)
    return units


def e4e_style_spatial(i):
    """GradualStyleBlock spatial size of style i: 16 (coarse, from c3), 32 (middle, from p2) or 64
    (fine, from p1)."""
    return 16 if i < E4E_COARSE else (32 if i < E4E_MIDDLE else 64)


def make_e4e_weights(size, seed=0, start_from_latent_avg=True):
    """Seeded Encoder4Editing(50, 'ir_se') state dict (eval-mode BatchNorm running statistics
    included) for a generator of output size ``size`` (style_count = n_latent). Scales keep the
    24-unit residual stack O(1): He-normal convs, BatchNorm γ of the residual branch ≈ 0.3,
    PReLU slopes ≈ 0.25 (PyTorch's init; kept > 0 here — the encoder also takes slopes ≤ 0,
    tests/test_gpu_e4e.py::test_e4e_negative_prelu_slopes_vs_forced_oracle)."""
    g = torch.Generator().manual_seed(int(seed))
    p = {}

    def bn(prefix, c, gamma=1.0):
        p[prefix + ".weight"] = gamma * (1.0 + 0.1 * torch.randn(c, generator=g))
        p[prefix + ".bias"] = 0.1 * torch.randn(c, generator=g)
        p[prefix + ".running_mean"] = 0.1 * torch.randn(c, generator=g)
        p[prefix + ".running_var"] = 0.5 + torch.rand(c, generator=g)

    def conv(name, cout, cin, k, gain=2.0):
        p[name] = torch.randn(cout, cin, k, k, generator=g) * math.sqrt(gain / (cin * k * k))

    def prelu(name, c):
        p[name] = (0.25 + 0.05 * torch.randn(c, generator=g)).clamp_min(0.05)

    conv("input_layer.0.weight", 64, 3, 3)
    bn("input_layer.1", 64)
    prelu("input_layer.2.weight", 64)
    for i, (cin, depth, stride) in enumerate(e4e_units()):
        pre = f"body.{i}"
        if cin != depth:
            conv(pre + ".shortcut_layer.0.weight", depth, cin, 1, gain=1.0)
            bn(pre + ".shortcut_layer.1", depth)
        bn(pre + ".res_layer.0", cin)
        conv(pre + ".res_layer.1.weight", depth, cin, 3)
        prelu(pre + ".res_layer.2.weight", depth)
        conv(pre + ".res_layer.3.weight", depth, depth, 3)
        bn(pre + ".res_layer.4", depth, gamma=0.3)
        cr = depth // E4E_SE_REDUCTION
        conv(pre + ".res_layer.5.fc1.weight", cr, depth, 1, gain=1.0)
        conv(pre + ".res_layer.5.fc2.weight", depth, cr, 1, gain=1.0)
    for i in range(n_latent_for(size)):
        sp = e4e_style_spatial(i)
        for j in range(int(math.log2(sp))):
            conv(f"styles.{i}.convs.{2 * j}.weight", STYLE_DIM, STYLE_DIM, 3)
            p[f"styles.{i}.convs.{2 * j}.bias"] = 0.05 * torch.randn(STYLE_DIM, generator=g)
        p[f"styles.{i}.linear.weight"] = torch.randn(STYLE_DIM, STYLE_DIM, generator=g)
        p[f"styles.{i}.linear.bias"] = 0.1 * torch.randn(STYLE_DIM, generator=g)
    for name, cin in (("latlayer1", 256), ("latlayer2", 128)):
        conv(name + ".weight", STYLE_DIM, cin, 1, gain=1.0)
        p[name + ".bias"] = 0.05 * torch.randn(STYLE_DIM, generator=g)
    p["latent_avg"] = 0.1 * torch.randn(n_latent_for(size), STYLE_DIM, generator=g)
    p["start_from_latent_avg"] = bool(start_from_latent_avg)
    p["kind"] = "e4e"
    return p
