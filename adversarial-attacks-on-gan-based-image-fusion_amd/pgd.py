"""PGD / FGSM attack on GAN image fusion: the public ``attack(net, imgs, eps, steps)`` entry point.

Semantics:
* objective — ``optimize_vgg`` (code/attack/interpolation.py:743-818), per image, MSE means:
    L = 10·MSE(E(x'),E(t')) − MSE(E(x'),E(x0')) + MSE(t, G(E(x'))) + 0.1·Σ_k MSE(V_k(G'), V_k(t'))
        + 10·MSE(x0, x) + Σ_k MSE(V_k(x'), V_k(x0'))          (' = avg_pool2d(·, S/256))
  The decoder receives the raw encoder output (no latent_avg, interpolation.py:780).
* update — torchattacks PGD (commented copy at interpolation.py:62-96), descending L
  (cost = −L, the targeted form :83-86): x ← clamp(x0 + clamp(x + a·sign(−∇L) − x0, −e, e), −1, 1),
  with e = 2ε, a = 2α because ε, α are given in [0,1] pixel units and the tensors live in [-1,1].
  FGSM = one step with α = ε and no random start.

Execution: every step runs on libmiattack kernels (no autograd, no torch compute ops):
encoder → synthesis → VGG(rec') fwd/bwd → VGG(x') fwd/bwd → synthesis bwd → encoder bwd →
fused gradient-assembly + sign-project kernel. Images are independent, so the batch is processed
together (per-image MSE means; a batch's gradient equals the reference's per-image gradients).
The loss is never materialised on the device unless ``return_info`` asks for it: PGD needs only
sign(∇L), so there is no per-step host synchronisation.
"""
import numpy as np
import torch

from . import ops
from .vgg import CPAD
from .weights import ENC_POOL_RES, STYLE_DIM
from .workspace import Workspace

LOSS_WEIGHTS = dict(lat_t=10.0, lat_o=-1.0, img_rec_t=1.0, vgg_rec_t=0.1, img_o=10.0, vgg_img=1.0)
DEFAULT_LOSS_SCALE = {torch.float32: 1.0, torch.float16: 2.0 ** 16, torch.bfloat16: 2.0 ** 16}


def _f32(v):
    return float(np.float32(v))


class AttackEngine:
    """Owns the device networks and the step workspace for one (batch, size, dtype)."""

    def __init__(self, encoder, synth, vgg, loss_scale=None, weights=LOSS_WEIGHTS):
        self.E, self.G, self.V = encoder, synth, vgg
        self.size = synth.size
        self.dtype = synth.dtype
        if vgg.dtype != self.dtype:
            raise ValueError("VGG and generator must share the compute dtype")
        self.R = min(self.size, 256)  # the objective pools to 256² (attack_main2.py:590-591)
        self.pf = self.size // self.R
        self.ws = Workspace(synth.device)
        self.loss_scale = float(loss_scale if loss_scale is not None
                                else DEFAULT_LOSS_SCALE[self.dtype])
        self.w = dict(weights)
        R = self.R
        self.tap_numel = [64 * R * R, 64 * R * R, 128 * (R // 4) ** 2,
                          512 * ops.pool_out(R // 4, True) ** 2]
        lam = self.loss_scale
        S2 = 3 * self.size * self.size
        nl = self.G.n_latent * STYLE_DIM
        self.c_lat_t = lam * self.w["lat_t"] * 2.0 / nl
        self.c_lat_o = lam * self.w["lat_o"] * 2.0 / nl
        self.c_img_rec = lam * self.w["img_rec_t"] * 2.0 / S2
        self.c_img_o = lam * self.w["img_o"] * 2.0 / S2
        self.c_vgg_rec = [lam * self.w["vgg_rec_t"] * 2.0 / n for n in self.tap_numel]
        self.c_vgg_x = [lam * self.w["vgg_img"] * 2.0 / n for n in self.tap_numel]

    # ------------------------------------------------------------------------------------------
    def _vgg_input(self, img, name):
        N = img.shape[0]
        y = self.ws.get(name, (N, self.R, self.R, CPAD), self.dtype)
        return ops.image_to_nhwc(img, y, self.pf, CPAD)

    def prepare(self, x0, t):
        """Targets under no_grad (interpolation.py:757-764): E(t'), E(x0'), VGG taps of t', x0'."""
        ws = self.ws
        N = x0.shape[0]
        self.N = N
        self.x0 = x0
        self.t = t
        self.lat_t = ws.get("ref.lat_t", (N, self.G.n_latent, STYLE_DIM), torch.float32)
        self.lat_t.copy_(self.E.forward(t, ws))
        self.lat_o = ws.get("ref.lat_o", (N, self.G.n_latent, STYLE_DIM), torch.float32)
        self.lat_o.copy_(self.E.forward(x0, ws))
        self.taps_t, self.taps_o = [], []
        for img, dst, nm in ((t, self.taps_t, "t"), (x0, self.taps_o, "o")):
            a = self.V.forward(self._vgg_input(img, "ref.in"), ws, "")
            for k, tap in enumerate(self.V.taps(a)):
                keep = ws.get(f"ref.tap{nm}{k}", tap.shape, self.dtype)
                keep.copy_(tap)
                dst.append(keep)

    def gradient(self, x):
        """One forward/backward of the objective at x. Leaves (g_vgg_x, g_enc) for the update and
        returns them; both are scaled by loss_scale."""
        ws, G, V, E = self.ws, self.G, self.V, self.E
        N = x.shape[0]
        lat = E.forward(x, ws)
        rec = G.forward(lat, ws)
        self.rec = rec
        # reconstruction path: VGG(rec') vs VGG(t'), pixel MSE vs t
        a = V.forward(self._vgg_input(rec, "in.rec"), ws, "")
        g_rv = V.backward(a, self.taps_t, self.c_vgg_rec, ws, "r")
        g_img = ws.get("g.img", rec.shape, torch.float32)
        ops.image_grad(rec, self.t, g_rv, g_img, self.pf, self.c_img_rec)
        # input path: VGG(x') vs VGG(x0')
        a = V.forward(self._vgg_input(x, "in.x"), ws, "")
        g_xv = V.backward(a, self.taps_o, self.c_vgg_x, ws, "x")
        # latent terms, synthesis backward, encoder backward
        g_lat = ws.get("g.lat", lat.shape, torch.float32)
        ops.mse_grad_f32(lat, self.lat_t, g_lat, self.c_lat_t)
        ops.mse_grad_f32(lat, self.lat_o, g_lat, self.c_lat_o, accumulate=True)
        G.backward(g_img, g_lat, ws)
        g_enc = E.backward(g_lat, ws)
        return g_xv, g_enc

    def step(self, x, a, e):
        g_xv, g_enc = self.gradient(x)
        ops.pgd_update(x, self.x0, g_xv, g_enc, self.pf, ENC_POOL_RES, self.c_img_o, _f32(a),
                       _f32(e))
        return x

    def full_gradient(self, x):
        """∇_x L (unscaled, fp32 NCHW) assembled from the pieces — a diagnostic for tests."""
        g_xv, g_enc = self.gradient(x)
        N, S, pf = x.shape[0], self.size, self.pf
        k = S // ENC_POOL_RES
        g = self.c_img_o * (x - self.x0)
        gv = g_xv[..., :3].permute(0, 3, 1, 2).float()
        g = g + gv.repeat_interleave(pf, 2).repeat_interleave(pf, 3) / (pf * pf)
        g = g + g_enc.repeat_interleave(k, 2).repeat_interleave(k, 3) / (k * k)
        return g / self.loss_scale

    def loss(self, x):
        """Per-image objective value (fp32, host) — diagnostics only (syncs)."""
        ws, G, V, E = self.ws, self.G, self.V, self.E
        N = x.shape[0]
        out = torch.zeros(8, N, device=x.device)
        lat = E.forward(x, ws)
        rec = G.forward(lat, ws)
        nl = G.n_latent * STYLE_DIM
        ops.mse_sum(lat, self.lat_t, out[0])
        ops.mse_sum(lat, self.lat_o, out[1])
        ops.mse_sum(rec, self.t, out[2])
        ops.mse_sum(x, self.x0, out[4])
        a = V.forward(self._vgg_input(rec, "in.rec"), ws, "")
        for k, tap in enumerate(V.taps(a)):
            tmp = torch.zeros(N, device=x.device)
            ops.mse_sum(tap, self.taps_t[k], tmp)
            out[3] += tmp / self.tap_numel[k]
        a = V.forward(self._vgg_input(x, "in.x"), ws, "")
        for k, tap in enumerate(V.taps(a)):
            tmp = torch.zeros(N, device=x.device)
            ops.mse_sum(tap, self.taps_o[k], tmp)
            out[5] += tmp / self.tap_numel[k]
        S2 = 3 * self.size * self.size
        w = self.w
        L = (w["lat_t"] * out[0] / nl + w["lat_o"] * out[1] / nl + w["img_rec_t"] * out[2] / S2
             + w["vgg_rec_t"] * out[3] + w["img_o"] * out[4] / S2 + w["vgg_img"] * out[5])
        return L.cpu()

    def run(self, x0, t, steps, eps, alpha, random_start=False, start_noise=None):
        """PGD-steps from x0 toward the objective; returns the adversarial images (new tensor)."""
        e, a = 2.0 * eps, 2.0 * alpha
        self.prepare(x0, t)
        x = self.ws.get("adv", x0.shape, torch.float32)
        x.copy_(x0)
        if random_start:
            if start_noise is None:
                raise ValueError("random_start needs start_noise (host-seeded U(-1,1))")
            ops.random_start(x, x0, start_noise, _f32(e))
        for _ in range(steps):
            self.step(x, a, e)
        return x.clone()


def _check_images(imgs, size, name):
    if not torch.is_tensor(imgs) or imgs.dim() != 4 or imgs.shape[1] != 3:
        raise ValueError(f"{name} must be an (N,3,H,W) tensor")
    if imgs.shape[2] != size or imgs.shape[3] != size:
        raise ValueError(f"{name} must be {size}x{size} (net.decoder.size)")
    if not imgs.is_floating_point():
        raise ValueError(f"{name} must be floating point")


def attack(net, imgs, eps, steps, *, target=None, vgg=None, alpha=2 / 255, random_start=False,
           seed=0, norm="linf", loss="gan_vgg", loss_scale=None, return_info=False):
    """Craft adversarial images against the GAN fusion pipeline.

    net     pSp-like bundle: net.encoder, net.decoder (.size), net.latent_avg, net.opts
            (built by ``gfa_amd.networks.build_net``); may also carry ``net.vgg``.
    imgs    (N,3,S,S) float tensor in [-1,1] (reference normalisation, transforms_config.py:29-31),
            on CPU or GPU; not modified.
    eps     L∞ radius in [0,1] pixel units (8/255 in the reference's PGD call, interpolation.py:1343).
    steps   PGD iterations (1 with alpha=eps and random_start=False is FGSM).
    target  white-box target image(s) (N or 1, 3, S, S) — the ``img_target`` of optimize_vgg.
    Returns the adversarial images on the input's device (fp32), and a dict if return_info.
    """
    if norm != "linf" or loss != "gan_vgg":
        raise ValueError("only norm='linf', loss='gan_vgg' are implemented")
    size = net.decoder.size
    _check_images(imgs, size, "imgs")
    if target is None:
        target = getattr(net, "default_target", None)
    if target is None:
        raise ValueError("a white-box target image is required (optimize_vgg img_target)")
    if target.dim() == 4 and target.shape[0] == 1 and imgs.shape[0] > 1:
        target = target.expand(imgs.shape[0], -1, -1, -1)
    _check_images(target, size, "target")
    if target.shape[0] != imgs.shape[0]:
        raise ValueError("target batch must be 1 or match imgs")
    if not (eps > 0 and alpha > 0) or steps < 0 or int(steps) != steps:
        raise ValueError("need eps > 0, alpha > 0, integer steps >= 0")
    if float(imgs.min()) < -1.0 or float(imgs.max()) > 1.0:
        raise ValueError("imgs must lie in [-1, 1]")
    vgg = vgg if vgg is not None else getattr(net, "vgg", None)
    if vgg is None:
        raise ValueError("a VGG feature network is required (optimize_vgg's vgg)")
    dev = net.decoder.device
    x0 = imgs.detach().to(dev, torch.float32).contiguous()
    t = target.detach().to(dev, torch.float32).contiguous()
    eng = AttackEngine(net.encoder.impl, net.decoder.impl, vgg.impl, loss_scale=loss_scale)
    noise = None
    if random_start:
        g = torch.Generator().manual_seed(int(seed))
        noise = (torch.rand(x0.shape, generator=g) * 2 - 1).to(dev)
    adv = eng.run(x0, t, int(steps), float(eps), float(alpha), random_start, noise)
    adv = adv.to(imgs.device)
    if return_info:
        info = dict(loss=eng.loss(adv.to(dev)), steps=int(steps), eps=eps, alpha=alpha,
                    dtype=str(eng.dtype), loss_scale=eng.loss_scale)
        return adv, info
    return adv


def fgsm(net, imgs, eps, **kw):
    """FGSM = one PGD step with α = ε and no random start."""
    kw.pop("alpha", None)
    kw.pop("random_start", None)
    return attack(net, imgs, eps, 1, alpha=eps, random_start=False, **kw)


def algorithmic_flops_per_image_step(synth, vgg):
    """G fwd ×3 (fwd, dgrad, style-grad) + VGG ×4 (two calls, fwd + dgrad)."""
    return 3 * synth.flops_fwd_per_image + 4 * vgg.flops_fwd_per_image

