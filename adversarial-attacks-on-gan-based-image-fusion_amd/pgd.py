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
# the patch attack's loss (code/attack/patch/adversarial_patch.py:125): only −MSE(E(x0'), E(x'))
PATCH_WEIGHTS = dict(lat_t=0.0, lat_o=-1.0, img_rec_t=0.0, vgg_rec_t=0.0, img_o=0.0, vgg_img=0.0)
# Gradient (loss) scale per compute dtype. fp16: its range tops out at 65504, and the e4e
# encoder's backward from the latent terms (weight 10·2/(n_latent·512) per element) reaches
# 1e3–1e4 × λ… at λ = 2^16 whole images overflowed to inf/NaN (3 of 8 at 256², measured); at
# λ ≤ 2^12 none did and the gradient's sign agreed with fp32 on 99.98 % of the significant
# pixels, at λ = 2^8 too — 2^8 keeps 16× headroom. bf16 has fp32's exponent range: no scaling.
# An overflow that still happens is caught (per-image non-finite flags, read once per attack):
# the engine divides λ by RESCALE and re-runs the attack, at most MAX_RESCALES times.
DEFAULT_LOSS_SCALE = {torch.float32: 1.0, torch.float16: 2.0 ** 8, torch.bfloat16: 1.0}
RESCALE, MAX_RESCALES = 16.0, 4
RUN_OK, RUN_RESCALE, RUN_FATAL = 0, 1, 2  # per-run status, MAX-reduced over the ranks


def rescale_consensus(status, group=None):
    """The job-wide status of one attack run: the MAX of every rank's (OK < RESCALE < FATAL).
    Without a process group (single process) the local status."""
    if group is None:
        return status
    import torch.distributed as dist
    dev = (torch.device("cpu") if dist.get_backend(group) == "gloo"
           else torch.device("cuda", torch.cuda.current_device()))
    t = torch.tensor([int(status)], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def idle_rank_consensus(group):
    """A rank with an empty shard takes part in the attack's status rounds (one all-reduce per
    run of the ranks that attack) until they finish or fail together."""
    while True:
        st = rescale_consensus(RUN_OK, group)
        if st == RUN_OK:
            return
        if st == RUN_FATAL:
            raise FloatingPointError("non-finite gradient on another rank")


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
        self.w = dict(weights)
        # latent terms only (the patch attack): the generator and VGG terms carry weight 0, so
        # their gradient is 0·g and the step runs the encoder forward / backward alone
        self.lat_only = all(self.w[k] == 0 for k in ("img_rec_t", "vgg_rec_t", "img_o",
                                                     "vgg_img"))
        R = self.R
        self.tap_numel = [64 * R * R, 64 * R * R, 128 * (R // 4) ** 2,
                          512 * ops.pool_out(R // 4, True) ** 2]
        self.rescales = 0  # loss-scale reductions of the last attack (overflow re-runs)
        self.set_loss_scale(loss_scale if loss_scale is not None
                            else DEFAULT_LOSS_SCALE[self.dtype])

    def set_loss_scale(self, lam):
        """λ: every gradient coefficient carries it (fp16 range); the projections and the Adam /
        C&W updates divide it back out (sign(λ·g) = sign(g))."""
        self.loss_scale = lam = float(lam)
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
        self.nonfinite = ops.zero_(ws.get("nonfinite", (N,), torch.int32))
        self.lat_t = ws.get("ref.lat_t", (N, self.G.n_latent, STYLE_DIM), torch.float32)
        self.lat_t.copy_(self._encode(t, "ref.in")[0])
        self.lat_o = ws.get("ref.lat_o", (N, self.G.n_latent, STYLE_DIM), torch.float32)
        self.lat_o.copy_(self._encode(x0, "ref.in")[0])
        self.taps_t, self.taps_o = [], []
        for img, dst, nm in ((t, self.taps_t, "t"), (x0, self.taps_o, "o")):
            a = self.V.forward(self._vgg_input(img, "ref.in"), ws, "")
            for k, tap in enumerate(self.V.taps(a)):
                keep = ws.get(f"ref.tap{nm}{k}", tap.shape, self.dtype)
                keep.copy_(tap)
                dst.append(keep)

    def _encode(self, img, name):
        """E(img'). The e4e encoder reads the VGG input tensor x' (N,R,R,8) (both networks see
        avg_pool2d(img, S/256), attack_main2.py:597,622); returns (lat, x' or None)."""
        if getattr(self.E, "input_nhwc", False):
            xin = self._vgg_input(img, name)
            return self.E.forward_nhwc(xin, self.ws), xin
        return self.E.forward(img, self.ws), None

    def _loss_terms(self, which, out, *tensors):
        """out[n] += the per-image objective terms of one stage (unscaled weights, MSE means)."""
        w, nl = self.w, self.G.n_latent * STYLE_DIM
        S2 = 3 * self.size * self.size
        if which == "lat":
            lat, = tensors
            ops.mse_sum(lat, self.lat_t, out, w["lat_t"] / nl)
            ops.mse_sum(lat, self.lat_o, out, w["lat_o"] / nl)
        elif which == "rec":
            rec, a = tensors
            ops.mse_sum(rec, self.t, out, w["img_rec_t"] / S2)
            for k, tap in enumerate(self.V.taps(a)):
                ops.mse_sum(tap, self.taps_t[k], out, w["vgg_rec_t"] / self.tap_numel[k])
        else:
            x, a = tensors
            ops.mse_sum(x, self.x0, out, w["img_o"] / S2)
            for k, tap in enumerate(self.V.taps(a)):
                ops.mse_sum(tap, self.taps_o[k], out, w["vgg_img"] / self.tap_numel[k])

    def gradient(self, x, loss=None):
        """One forward/backward of the objective at x. Leaves (g_vgg_x, g_enc) for the update and
        returns them; both are scaled by loss_scale. ``loss`` (fp32 [N], zeroed by the caller)
        receives the per-image objective at x from the same forward pass (no host sync)."""
        ws, G, V, E = self.ws, self.G, self.V, self.E
        if self.lat_only:
            return self._gradient_lat(x, loss)
        lat, xin = self._encode(x, "in.x")
        rec = G.forward(lat, ws)
        self.rec = rec
        if loss is not None:
            self._loss_terms("lat", loss, lat)
        # reconstruction path: VGG(rec') vs VGG(t'), pixel MSE vs t
        a = V.forward(self._vgg_input(rec, "in.rec"), ws, "")
        if loss is not None:
            self._loss_terms("rec", loss, rec, a)
        g_rv = V.backward(a, self.taps_t, self.c_vgg_rec, ws, "r")
        g_img = ws.get("g.img", rec.shape, torch.float32)
        ops.image_grad(rec, self.t, g_rv, g_img, self.pf, self.c_img_rec)
        # input path: VGG(x') vs VGG(x0')
        a = V.forward(xin if xin is not None else self._vgg_input(x, "in.x"), ws, "")
        if loss is not None:
            self._loss_terms("x", loss, x, a)
        g_xv = V.backward(a, self.taps_o, self.c_vgg_x, ws, "x")
        # latent terms, synthesis backward, encoder backward
        g_lat = ws.get("g.lat", lat.shape, torch.float32)
        ops.mse_grad_f32(lat, self.lat_t, g_lat, self.c_lat_t)
        ops.mse_grad_f32(lat, self.lat_o, g_lat, self.c_lat_o, accumulate=True)
        G.backward(g_img, g_lat, ws)
        if xin is not None:  # e4e: ∂L/∂x' joins the VGG input-path gradient (same x')
            E.backward_nhwc(g_lat, ws, g_xv, accumulate=True)
            return g_xv, None
        return g_xv, E.backward(g_lat, ws)

    def _gradient_lat(self, x, loss=None):
        """gradient() when only the latent terms carry weight: E forward, the two latent MSE
        gradients, E backward (no generator, no VGG). Same return convention."""
        ws, E = self.ws, self.E
        lat, xin = self._encode(x, "in.x")
        if loss is not None:
            self._loss_terms("lat", loss, lat)
        g_lat = ws.get("g.lat", lat.shape, torch.float32)
        ops.mse_grad_f32(lat, self.lat_t, g_lat, self.c_lat_t)
        ops.mse_grad_f32(lat, self.lat_o, g_lat, self.c_lat_o, accumulate=True)
        N = x.shape[0]
        g_xv = ops.zero_(ws.get("g.xv0", (N, self.R, self.R, CPAD), self.dtype))
        if xin is not None:
            E.backward_nhwc(g_lat, ws, g_xv, accumulate=True)
            return g_xv, None
        return g_xv, E.backward(g_lat, ws)

    def run_patch(self, img, t, patch, mask, max_count):
        """The adversarial-patch loop (code/attack/patch/adversarial_patch.py:103-160) on the
        engine's loss weights (PATCH_WEIGHTS for the reference's loss): adv = (1−m)·img + m·patch;
        max_count times: g = ∇_adv L, patch −= g (the full-image gradient, step 1), adv =
        clamp((1−m)·img + m·patch, min(img), max(img)). `patch` (img's shape, fp32) is updated in
        place, as the reference's. Returns (adv, rec) with rec = G(E(adv')) of the last
        iteration's input (the reference's adv_img_rec).

        A loss-scale overflow (fp16) lowers λ and re-runs the whole loop from the caller's
        patch, like PGD / Adam / C&W (the raw-gradient step would otherwise have written NaN /
        Inf into the patch)."""
        patch0 = patch.clone()

        def once():
            patch.copy_(patch0)
            return self._run_patch(img, t, patch, mask, max_count)
        return self._with_rescale(once)

    def _run_patch(self, img, t, patch, mask, max_count):
        ws = self.ws
        f32 = torch.float32
        self.prepare(img, t)
        lo, hi = float(img.min()), float(img.max())  # torch.min / torch.max of the batch (:134)
        adv = ws.get("adv", img.shape, f32)
        ops.patch_update(patch, None, img, mask, adv, -float("inf"), float("inf"))  # :111 no clamp
        last = ws.get("patch.last", img.shape, f32)
        g = ws.get("g.full", img.shape, f32)
        for it in range(int(max_count)):
            if it == max_count - 1:
                last.copy_(adv)
            g_xv, g_enc = self.gradient(adv)
            # the reference's MSEs are batch means (nn.MSELoss over the whole batch, :116): the
            # raw-gradient step scales with 1/N, unlike the sign steps of PGD
            ops.grad_assemble(adv, self.x0, g_xv, g_enc, g, self.pf, ENC_POOL_RES, self.c_img_o,
                              1.0 / (self.loss_scale * img.shape[0]), nonfinite=self.nonfinite)
            ops.patch_update(patch, g, img, mask, adv, lo, hi)
        lat, _ = self._encode(last if max_count > 0 else adv, "in.x")
        return adv.clone(), self.G.forward(lat, ws).clone()

    def step(self, x, a, e):
        g_xv, g_enc = self.gradient(x)
        ops.pgd_update(x, self.x0, g_xv, g_enc, self.pf, ENC_POOL_RES, self.c_img_o, _f32(a),
                       _f32(e), nonfinite=self.nonfinite)
        return x

    def overflowed(self):
        """Images whose gradient had a non-finite element since prepare() (one host sync)."""
        return self.nonfinite.nonzero().flatten().tolist()

    def _with_rescale(self, run_once, group=None):
        """Run an attack; if any image's gradient overflowed, lower λ and run it again (fp16).
        A non-finite gradient at λ that cannot be lowered (fp32 / bf16, or after MAX_RESCALES)
        raises: sign(NaN) = 0 would otherwise leave those pixels silently unattacked.

        ``group`` (attack_distributed): the decision is taken by every rank together — each
        rank's status (OK / RESCALE / FATAL) is MAX-all-reduced after every run, so all shards
        re-run at the same λ (the result does not depend on the world size) and a fatal overflow
        raises on every rank instead of leaving the others blocked in the final all-gather."""
        self.rescales = 0
        while True:
            out = run_once()
            bad = self.overflowed()
            status = (RUN_OK if not bad else RUN_RESCALE
                      if self.dtype == torch.float16 and self.rescales < MAX_RESCALES
                      else RUN_FATAL)
            status = rescale_consensus(status, group)
            if status == RUN_OK:
                return out
            if status == RUN_FATAL:
                raise FloatingPointError(
                    f"non-finite gradient for images {bad[:8]}"
                    + ("" if bad else " on another rank")
                    + f" (dtype {self.dtype}, loss scale {self.loss_scale:g}): check the weights "
                    "/ inputs, or run fp32")
            self.set_loss_scale(self.loss_scale / RESCALE)
            self.rescales += 1

    def full_gradient(self, x):
        """∇_x L (unscaled, fp32 NCHW) at x."""
        g = self.ws.get("g.full", x.shape, torch.float32)
        g_xv, g_enc = self.gradient(x)
        ops.grad_assemble(x, self.x0, g_xv, g_enc, g, self.pf, ENC_POOL_RES, self.c_img_o,
                          1.0 / self.loss_scale)
        return g.clone()

    def objective(self, x, out):
        """Per-image objective at x into out (fp32 [N], +=): forward passes only."""
        ws, G, V, E = self.ws, self.G, self.V, self.E
        lat, xin = self._encode(x, "in.x")
        rec = G.forward(lat, ws)
        self._loss_terms("lat", out, lat)
        a = V.forward(self._vgg_input(rec, "in.rec"), ws, "")
        self._loss_terms("rec", out, rec, a)
        a = V.forward(xin if xin is not None else self._vgg_input(x, "in.x"), ws, "")
        self._loss_terms("x", out, x, a)
        return out

    def loss(self, x):
        """Per-image objective value (fp32, host) — diagnostics (syncs)."""
        out = self.ws.get("loss.diag", (x.shape[0],), torch.float32)
        ops.zero_(out)
        return self.objective(x, out).cpu()

    def _full_grad(self, x, g, loss=None):
        """g ← ∇_x L (loss-scaled, fp32 NCHW) by the gradient-assembly kernel."""
        g_xv, g_enc = self.gradient(x, loss)
        ops.grad_assemble(x, self.x0, g_xv, g_enc, g, self.pf, ENC_POOL_RES, self.c_img_o,
                          nonfinite=self.nonfinite)
        return g

    def run_adam(self, x0, t, steps, lr=0.01, betas=(0.9, 0.999), eps=1e-8, group=None):
        """``optimize_vgg`` literal mode (interpolation.py:743-843): Adam(lr) on the pixels,
        descending L, no ε-ball or clamp. The gradient carries the loss scale λ, so Adam's eps is
        scaled by λ too (m̂/(√v̂ + λ·eps) on λ·g ≡ m̂/(√v̂ + eps) on g)."""
        return self._with_rescale(lambda: self._run_adam(x0, t, steps, lr, betas, eps), group)

    def _run_adam(self, x0, t, steps, lr, betas, eps):
        self.prepare(x0, t)
        ws = self.ws
        x = ws.get("adv", x0.shape, torch.float32)
        x.copy_(x0)
        m = ops.zero_(ws.get("adam.m", x0.shape, torch.float32))
        v = ops.zero_(ws.get("adam.v", x0.shape, torch.float32))
        g = ws.get("g.full", x0.shape, torch.float32)
        for it in range(1, steps + 1):
            self._full_grad(x, g)
            ops.adam_step(x, g, m, v, lr, betas[0], betas[1], eps * self.loss_scale, it)
        return x.clone()

    def run_cw(self, x0, t, steps, c=1e-4, lr=0.01, betas=(0.9, 0.999), eps=1e-8, group=None,
               early_stop=True):
        """torchattacks C&W L2 (interpolation.py:98-193) composed with the GAN objective, in
        [-1,1] space: adv = tanh(w); cost = Σ‖(adv − x0)/2‖² + c·Σ L_n(adv); Adam(lr) on w;
        best-L2 tracking with success = L_n(adv) < L_n(x0); early stop every steps//10 when the
        cost rises (one host sync there). See oracle.attack_ref.cw_attack. ``early_stop=False``
        runs every iteration (a fixed-work timing; not the reference's semantics)."""
        return self._with_rescale(
            lambda: self._run_cw(x0, t, steps, c, lr, betas, eps, early_stop), group)

    def _run_cw(self, x0, t, steps, c, lr, betas, eps, early_stop=True):
        self.prepare(x0, t)
        ws = self.ws
        N = x0.shape[0]
        f32 = torch.float32
        f0 = ops.zero_(ws.get("cw.f0", (N,), f32))
        self.objective(x0, f0)
        w = ops.cw_init(x0, ws.get("cw.w", x0.shape, f32))
        adv = ws.get("adv", x0.shape, f32)
        best = ws.get("cw.best", x0.shape, f32)
        best.copy_(x0)
        best_l2 = ws.get("cw.best_l2", (N,), f32)
        best_l2.fill_(1e10)
        m = ops.zero_(ws.get("adam.m", x0.shape, f32))
        v = ops.zero_(ws.get("adam.v", x0.shape, f32))
        g = ws.get("g.full", x0.shape, f32)
        gw = ws.get("cw.gw", x0.shape, f32)
        f = ws.get("cw.f", (N,), f32)
        sq = ws.get("cw.sq", (N,), f32)
        prev = 1e10
        every = max(steps // 10, 1)
        self.cw_steps_run = 0  # iterations executed (early stop), for bench.py's report
        for step in range(steps):
            self.cw_steps_run = step + 1
            ops.cw_tanh(w, adv)
            ops.zero_(f)
            self._full_grad(adv, g, loss=f)
            ops.cw_grad(adv, x0, g, gw, c, 1.0 / self.loss_scale)
            ops.adam_step(w, gw, m, v, lr, betas[0], betas[1], eps, step + 1)
            ops.zero_(sq)
            ops.mse_sum(adv, x0, sq)
            ops.cw_select(adv, best, sq, best_l2, f, f0, 0.25)
            if early_stop and step % every == 0:
                cost = 0.25 * float(sq.cpu().double().sum()) + c * float(f.cpu().double().sum())
                if cost > prev:
                    break
                prev = cost
        return best.clone()

    def run(self, x0, t, steps, eps, alpha, random_start=False, start_noise=None, group=None):
        """PGD-steps from x0 toward the objective; returns the adversarial images (new tensor)."""
        return self._with_rescale(
            lambda: self._run_pgd(x0, t, steps, eps, alpha, random_start, start_noise), group)

    def _run_pgd(self, x0, t, steps, eps, alpha, random_start, start_noise):
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


NORMS = ("linf", "adam", "l2_cw")


def make_start_noise(shape, seed):
    """The random-start draw: host-seeded U(-1,1) of the FULL batch shape (scaled by e in the
    kernel); ``attack_distributed`` slices it per shard so every world size sees the same noise."""
    g = torch.Generator().manual_seed(int(seed))
    return torch.rand(shape, generator=g) * 2 - 1


def attack(net, imgs, eps, steps, *, target=None, vgg=None, alpha=0.01, random_start=False,
           seed=0, start_noise=None, norm="linf", loss="gan_vgg", loss_scale=None, lr=0.01,
           cw_c=1e-4, return_info=False, group=None):
    """Craft adversarial images against the GAN fusion pipeline.

    net     pSp-like bundle: net.encoder, net.decoder (.size), net.latent_avg, net.opts
            (built by ``gfa_amd.networks.build_net``); may also carry ``net.vgg``.
    imgs    (N,3,S,S) float tensor in [-1,1] (reference normalisation, transforms_config.py:29-31),
            on CPU or GPU; not modified.
    eps     L∞ radius in [0,1] pixel units (8/255 in the reference's PGD call, interpolation.py:1343).
    steps   iterations (PGD: 1 with alpha=eps and random_start=False is FGSM).
    alpha   PGD step in [0,1] pixel units; default 0.01 = the reference's PGD call
            (interpolation.py:1343; torchattacks' own default is 2/255).
    start_noise  optional host U(-1,1) tensor of imgs' shape for random_start (default: drawn
            from ``seed`` by ``make_start_noise(imgs.shape, seed)``).
    target  white-box target image(s) (N or 1, 3, S, S) — the ``img_target`` of optimize_vgg.
    norm    'linf'  — torchattacks PGD rule (interpolation.py:62-96) on the objective;
            'adam'  — optimize_vgg literal (interpolation.py:743-843): Adam(lr) on the pixels,
                      no ε-ball (eps is ignored and may be None);
            'l2_cw' — torchattacks C&W L2 (interpolation.py:98-193) with f = the objective,
                      c = cw_c, Adam(lr) in tanh space (eps ignored; see AttackEngine.run_cw).
    group   process group of a data-parallel job (``dist.attack_distributed``): the fp16
            loss-scale re-run decision is all-reduced over it so every shard runs at one λ.
    Returns the adversarial images on the input's device (fp32), and a dict if return_info.
    """
    if norm not in NORMS:
        raise ValueError(f"norm must be one of {NORMS}")
    if loss != "gan_vgg":
        raise ValueError("only loss='gan_vgg' (the optimize_vgg objective) is implemented")
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
    if steps < 0 or int(steps) != steps:
        raise ValueError("need integer steps >= 0")
    if norm == "linf" and not (eps is not None and eps > 0 and alpha > 0):
        raise ValueError("PGD needs eps > 0 and alpha > 0")
    if norm != "linf" and not lr > 0:
        raise ValueError("lr must be > 0")
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
        if start_noise is None:
            start_noise = make_start_noise(tuple(x0.shape), seed)
        if tuple(start_noise.shape) != tuple(x0.shape):
            raise ValueError("start_noise must have the shape of imgs")
        noise = start_noise.to(dev, torch.float32).contiguous()
    if norm == "linf":
        adv = eng.run(x0, t, int(steps), float(eps), float(alpha), random_start, noise,
                      group=group)
    elif norm == "adam":
        adv = eng.run_adam(x0, t, int(steps), lr=float(lr), group=group)
    else:
        adv = eng.run_cw(x0, t, int(steps), c=float(cw_c), lr=float(lr), group=group)
    adv = adv.to(imgs.device)
    if return_info:
        info = dict(loss=eng.loss(adv.to(dev)), steps=int(steps), eps=eps, alpha=alpha, norm=norm,
                    dtype=str(eng.dtype), loss_scale=eng.loss_scale, rescales=eng.rescales)
        return adv, info
    return adv


def fgsm(net, imgs, eps, **kw):
    """FGSM = one PGD step with α = ε and no random start."""
    kw.pop("alpha", None)
    kw.pop("random_start", None)
    return attack(net, imgs, eps, 1, alpha=eps, random_start=False, **kw)


def algorithmic_flops_per_image_step(synth, vgg, encoder=None):
    """GEMM work one PGD iteration needs per image: G ×2 (forward + input gradient) + VGG ×4
    (two calls, forward + input gradient each) + the e4e encoder ×2 (forward + input gradient)
    when it is the real one (the linear stand-in's FLOPs are excluded).

    SURVEY.md §8d counted G ×3 with a separate style-gradient GEMM. The kernels never form the
    per-sample weight gradient: ∂L/∂s[n][ci] = Σ_p x[n,p,ci]·(Wᵀg)[n,p,ci] is a dot product
    over the dgrad output the input gradient computes anyway (2·H·W·Cin FLOP per layer, the
    `sdot` epilogue), so crediting it as a third GEMM would overstate the work by ~13 %."""
    enc = 2 * getattr(encoder, "flops_fwd_per_image", 0) if encoder is not None else 0
    return 2 * synth.flops_fwd_per_image + 4 * vgg.flops_fwd_per_image + enc

