"""Shared builders for the GPU parity tests (not a test module)."""
import torch

from gfa_amd import pgd
from gfa_amd.vgg import VGGNet
from gfa_amd.weights import (make_e4e_weights, make_encoder_weights, make_generator_weights,
                             make_vgg_weights)


def nchw(t):
    return t.permute(0, 3, 1, 2).double().cpu()


def seeded(seed, shape):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * 2 - 1


def engine(size, dtype, cuda, encoder="e4e", gen_seed=0, enc_seed=1, vgg_seed=1234):
    """AttackEngine over the reference's three networks (seeded random init) and the oracle's
    parameter dicts for the same weights."""
    from gfa_amd.e4e import E4EEncoder
    from gfa_amd.encoder import SyntheticEncoder
    from gfa_amd.stylegan2 import SynthesisNet
    from oracle import vgg_ref
    gp = make_generator_weights(size, seed=gen_seed)
    ep = (make_e4e_weights(size, seed=enc_seed) if encoder == "e4e"
          else make_encoder_weights(size, seed=enc_seed))
    vs = make_vgg_weights(vgg_seed)
    enc = (E4EEncoder(ep, size, dtype=dtype, device=cuda) if encoder == "e4e"
           else SyntheticEncoder(ep, size, device=cuda))
    eng = pgd.AttackEngine(enc, SynthesisNet(gp, size, dtype=dtype, device=cuda),
                           VGGNet(vs, dtype=dtype, device=cuda))
    return eng, (gp, vgg_ref.load_positional(vs), ep)


def to64(params):
    gp, vp, ep = params
    return ({k: v.double() for k, v in gp.items()},
            {k: (w.double(), b.double()) for k, (w, b) in vp.items()},
            {k: (v.double() if torch.is_tensor(v) else v) for k, v in ep.items()})


def e4e_masks(enc):
    """The device run's PReLU / LeakyReLU branch per activation (the sign of the tensor the
    backward masks with: the stored activation, whose sign is the pre-activation's for slopes ≥ 0,
    or — a layer with a negative PReLU slope, round 6 — the stored pre-activation), keyed as
    oracle.encoder_ref.forced_masks expects. Reflects the encoder's most recent forward."""
    m = {"in": nchw(enc._m0) > 0}
    for i, U in enumerate(enc.units):
        m[f"body.{i}"] = nchw(U["_m1"]) > 0
        m[f"body.{i}.se"] = (U["_u"] > 0).cpu()[:, :, None, None]  # relu(fc1(avg)), (N, C/16)
    for i, hd in enumerate(enc.heads):
        for j, a in enumerate(hd["_acts"]):
            m[f"styles.{i}.{j}"] = nchw(a) > 0
    return m


def g_masks(G, ws, n=None):
    """The device generator's LeakyReLU branch per StyledConv (sign of the stored activation
    g.pre{i}), keyed by the oracle's styled-conv prefixes (conv1, convs.0, convs.1, …)."""
    m = {}
    i = 0
    while f"g.pre{i}" in ws._bufs:
        a = nchw(ws._bufs[f"g.pre{i}"]) > 0
        m["conv1" if i == 0 else f"convs.{i - 1}"] = a if n is None else a[:n]
        i += 1
    return m


def pool_onehot(x):
    """One-hot of the first maximum of every 2×2 window (row-major order, ceil-mode padding with
    −inf), the tie rule of maxpool2_bwd_kernel (pointwise.hip)."""
    N, C, H, W = x.shape
    xp = torch.nn.functional.pad(x, (0, W % 2, 0, H % 2), value=float("-inf"))
    Hp, Wp = xp.shape[2], xp.shape[3]
    win = xp.reshape(N, C, Hp // 2, 2, Wp // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(
        N, C, Hp // 2, Wp // 2, 4)
    oh = torch.nn.functional.one_hot(win.argmax(-1), 4).bool()
    oh = oh.reshape(N, C, Hp // 2, Wp // 2, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(N, C, Hp, Wp)
    return oh[:, :, :H, :W]


def vgg_masks(a, n=None):
    """The device VGG forward's branches (ReLU positive sets from the stored post-ReLU outputs,
    pool window argmaxes from the pool inputs), keyed as oracle.vgg_ref.forced_masks expects."""
    sl = (lambda t: t) if n is None else (lambda t: t[:n])
    m = {}
    for k, name in (("c11", "conv1_1"), ("c12", "conv1_2"), ("c21", "conv2_1"), ("c22", "conv2_2"),
                    ("c31", "conv3_1"), ("c32", "conv3_2"), ("c33", "conv3_3"), ("c41", "conv4_1"),
                    ("c42", "conv4_2")):
        m[name] = sl(nchw(a[k]) > 0)
    for k, name in (("c12", "pool1"), ("c22", "pool2"), ("c33", "pool3")):
        m[name] = sl(pool_onehot(nchw(a[k])))
    return m


class capture_vgg:
    """Records vgg_masks() of every device VGG forward while active (the gradient pass runs the
    reconstruction path first, then the input path, as the oracle objective does)."""

    def __init__(self, V, n=None):
        self.V, self.n, self.masks = V, n, []

    def __enter__(self):
        self._fwd = self.V.forward

        def fwd(x, ws, tag):
            a = self._fwd(x, ws, tag)
            self.masks.append(vgg_masks(a, self.n))
            return a
        self.V.forward = fwd
        return self

    def __exit__(self, *exc):
        self.V.forward = self._fwd


# Forced-branch bound (oracle/forcing.py): every site where the device's branch disagrees with the
# fp64 oracle's own decision must be a near-tie — |pre| ≤ FLIP_TOL[dtype]·max|pre| of its layer
# (pools: max − x[forced] ≤ FLIP_TOL·max|x|) — and such sites at most FLIP_FRAC of all sites.
# fp32: the split arithmetic's ≈ 1e-6 relative activation error (test_fp32_arithmetic_is_fp32_
# accurate) compounded through the e4e / generator / VGG depth stays well inside 1e-5.
FLIP_TOL = {torch.float32: 1e-5}
FLIP_FRAC = 1e-4


class forced_all:
    """Oracle context following every branch of the device's most recent gradient pass: e4e
    PReLU / LeakyReLU / SE ReLU, generator LeakyReLU, VGG ReLU and pool argmax (both VGG passes,
    captured with capture_vgg). ``n``: the first n images only. ``.audit`` records, per forced
    site, the branches that disagree with the oracle's own fp64 decision (oracle/forcing.py);
    ``check()`` bounds them."""

    def __init__(self, eng, vgg_cap, n=None):
        from oracle import encoder_ref, forcing, stylegan2_ref, vgg_ref
        em = e4e_masks(eng.E)
        if n is not None:
            em = {k: v[:n] for k, v in em.items()}
        self.audit = forcing.audit()
        self.dtype = eng.dtype
        self.ctx = [self.audit, encoder_ref.forced_masks(em),
                    stylegan2_ref.forced_masks(g_masks(eng.G, eng.ws, n)),
                    vgg_ref.forced_masks(vgg_cap.masks[-2:])]

    def report(self):
        flips, sites, worst, key = self.audit.summary()
        return (f"forced flips: {flips} of {sites} sites, max |pre| at a flip "
                f"{worst:.2e} of its layer's max" + (f" ({key})" if key else ""))

    def check(self, tol=None, frac=FLIP_FRAC):
        """Assert every forced disagreement is a near-tie and that they are rare; returns
        report()."""
        tol = FLIP_TOL.get(self.dtype, 1e-5) if tol is None else tol
        flips, sites, worst, key = self.audit.summary()
        assert sites > 0, "no forced site was evaluated"
        bad = [r for r in self.audit.records if r["flips"] and r["rel_gap"] > tol]
        assert not bad, ("forced branches that are not near-ties: "
                         + ", ".join(f"{r['key']}: {r['flips']} flips, gap {r['rel_gap']:.2e}"
                                     for r in bad[:8]))
        assert flips <= frac * sites, self.report()
        return self.report()

    def __enter__(self):
        for c in self.ctx:
            c.__enter__()
        return self

    def __exit__(self, *exc):
        for c in reversed(self.ctx):
            c.__exit__(*exc)


def grad_stats(got, ref, big_frac=1e-2):
    """(‖Δ‖/‖ref‖, max|Δ|/max|ref|, sign agreement where |ref| > big_frac·max|ref|)."""
    got, ref = got.double().cpu(), ref.double().cpu()
    nrm = ((got - ref).norm() / ref.norm()).item()
    mx = ((got - ref).abs().max() / ref.abs().max()).item()
    big = ref.abs() > big_frac * ref.abs().max()
    agree = (torch.sign(got[big]) == torch.sign(ref[big])).float().mean().item()
    return nrm, mx, agree


def free():
    """Release the caching allocator's blocks between the large tests (callers drop their
    engines first)."""
    import gc
    gc.collect()
    torch.cuda.empty_cache()
