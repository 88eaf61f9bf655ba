"""Audit of the teacher-forced oracle branches (TEST INFRASTRUCTURE ONLY, see oracle/__init__).

Under ``vgg_ref / stylegan2_ref / encoder_ref.forced_masks`` the fp64 oracle follows the device
run's branch at every ReLU / LeakyReLU / PReLU / SE-ReLU and at every 2×2 pool window. Forcing is
only legitimate where the device's branch could come from rounding: a site whose fp64
pre-activation sits at a tie (|pre| ≈ 0) or a window whose two largest inputs are within rounding
of each other. A device bug that flips branches (a wrong mask recovered from a stored activation,
a sign error in a ``pre = a / lrelu'(a)`` recovery) would otherwise be absorbed by the forcing.

While ``audit()`` is active, every forced site records how many of its branches disagree with
the oracle's own fp64 decision at the same point of the (forced) computation and the largest
|pre| (or window margin) among them, relative to the layer's max |pre| (or max |input|). The
tests assert that every disagreement is a near-tie and that they are rare."""
import torch
import torch.nn.functional as F

AUDIT = None


class audit:
    """Collect the per-site records of every forced evaluation inside the block."""

    def __init__(self):
        self.records = []

    def __enter__(self):
        global AUDIT
        AUDIT = self.records
        return self

    def __exit__(self, *exc):
        global AUDIT
        AUDIT = None

    def summary(self):
        """(disagreeing sites, sites, worst relative gap over all disagreements, its key)."""
        flips = sum(r["flips"] for r in self.records)
        sites = sum(r["sites"] for r in self.records)
        worst, key = 0.0, None
        for r in self.records:
            if r["flips"] and r["rel_gap"] >= worst:
                worst, key = r["rel_gap"], r["key"]
        return flips, sites, worst, key


def _record(key, flip, gap, scale):
    n = int(flip.sum())
    g = float(gap[flip].abs().max()) if n else 0.0
    s = float(scale)
    AUDIT.append(dict(key=key, sites=flip.numel(), flips=n, max_gap=g, scale=s,
                      rel_gap=g / s if s > 0 else (0.0 if g == 0 else float("inf"))))


def relu_site(key, forced, pre):
    """A forced positive set ``forced`` at pre-activation ``pre`` (oracle's own branch: pre > 0)."""
    if AUDIT is None:
        return
    with torch.no_grad():
        p = pre.detach()
        own = p > 0
        flip = forced.to(p.device) != own
        # pre == 0 exactly: both branches give 0 — not a flip of the function
        flip &= p != 0
        _record(key, flip, p, p.abs().max())


def pool_site(key, forced_onehot, x, ceil_mode=False):
    """A forced one-hot argmax per 2×2 window at pool input ``x``: a window disagrees when the
    forced position does not hold the window's fp64 maximum; its gap is max − x[forced]."""
    if AUDIT is None:
        return
    with torch.no_grad():
        xd = x.detach()
        sel = F.avg_pool2d(torch.where(forced_onehot, xd, torch.zeros_like(xd)), 2, 2,
                           ceil_mode=ceil_mode, divisor_override=1)
        mx = F.max_pool2d(xd, 2, 2, ceil_mode=ceil_mode)
        gap = mx - sel
        _record(key, gap > 0, gap, xd.abs().max())
