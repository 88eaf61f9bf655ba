"""VGG16 feature trunk on libmiattack kernels (forward + input gradient of the tap-MSE loss).

Mirrors ``code/vgg.py``: ``VGGBase.forward`` (:44-64) returns (conv1_1, conv1_2, conv3_2, conv4_2),
where the tap the reference names ``conv3_2`` is the pool2 output (:53-54) and pool3 uses
``ceil_mode=True`` (:24). Weights load positionally from a VGG16 checkpoint, first 26 tensors
(``load_pretrained_layers`` :66-76). Only conv1_1..conv4_2 run (:44-64); conv4_3..conv7 exist in
the reference module but never execute, so they are not materialised here.

Layout: NHWC in the compute dtype; the 3-channel input is padded to 8 channels (zeros) so every
conv operand row is a whole number of 16-byte vectors.
"""
import torch

from . import layouts, ops
from .weights import VGG_CONVS, VGG_USED

CPAD = 8  # input channel padding
TAP_NAMES = ("conv1_1", "conv1_2", "conv3_2", "conv4_2")


def load_vgg_state(pth_or_sd):
    """vgg.py:66-76 — positional: the checkpoint's tensors in order (weight, bias per conv)."""
    if isinstance(pth_or_sd, dict):
        sd = pth_or_sd
    else:
        sd = torch.load(pth_or_sd, map_location="cpu", weights_only=True)
    vals = list(sd.values())
    if len(vals) < 2 * VGG_USED:
        raise ValueError(f"VGG checkpoint has {len(vals)} tensors, need ≥ {2 * VGG_USED}")
    out = {}
    for i, (name, cin, cout) in enumerate(VGG_CONVS[:VGG_USED]):
        w, b = vals[2 * i], vals[2 * i + 1]
        if tuple(w.shape) != (cout, cin, 3, 3) or tuple(b.shape) != (cout,):
            raise ValueError(f"{name}: unexpected shapes {tuple(w.shape)} {tuple(b.shape)}")
        out[name] = (w.float(), b.float())
    return out


class VGGNet:
    def __init__(self, pth_or_sd, dtype=torch.float32, device="cuda"):
        self.dtype = dtype
        self.device = torch.device(device)
        params = load_vgg_state(pth_or_sd)
        self.layers = {}
        for name, cin, cout in VGG_CONVS[:VGG_USED]:
            w, b = params[name]
            cp = CPAD if cin < CPAD else cin
            self.layers[name] = dict(
                cin=cp, cout=cout,
                wf=layouts.fwd_matrix(w, dtype, cin_pad=cp).contiguous().to(self.device),
                wd=layouts.dgrad_matrix(w, dtype, cin_pad=cp).contiguous().to(self.device),
                bias=b.contiguous().to(self.device))
        # conv MACs per 256² image (15.82 GMAC)
        self.flops_fwd_per_image = 2 * sum(
            9 * cin * cout * r * r for (n, cin, cout), r in zip(
                VGG_CONVS[:VGG_USED], [256, 256, 128, 128, 64, 64, 64, 32, 32]))

    def _conv(self, name, x, y):
        L = self.layers[name]
        N, H, W, _ = x.shape
        fl = 2 * N * H * W * 9 * (3 if name == "conv1_1" else L["cin"]) * L["cout"]
        return ops.conv3x3(x, L["wf"], y, cout=L["cout"], bias=L["bias"], act_out=ops.ACT_RELU,
                           flops=fl)

    def forward(self, x, ws, tag):
        """x: (N,R,R,8) NHWC. Returns dict of the saved activations (taps included)."""
        N, R = x.shape[0], x.shape[1]
        T = self.dtype
        g = lambda n, r, c: ws.get(f"v{tag}.{n}", (N, r, r, c), T)  # noqa: E731
        R2, R4 = R // 2, R // 4
        R8 = ops.pool_out(R4, True)
        a = {"x": x}
        a["c11"] = self._conv("conv1_1", x, g("c11", R, 64))
        a["c12"] = self._conv("conv1_2", a["c11"], g("c12", R, 64))
        a["p1"] = ops.maxpool2_fwd(a["c12"], g("p1", R2, 64))
        a["c21"] = self._conv("conv2_1", a["p1"], g("c21", R2, 128))
        a["c22"] = self._conv("conv2_2", a["c21"], g("c22", R2, 128))
        a["p2"] = ops.maxpool2_fwd(a["c22"], g("p2", R4, 128))
        a["c31"] = self._conv("conv3_1", a["p2"], g("c31", R4, 256))
        a["c32"] = self._conv("conv3_2", a["c31"], g("c32", R4, 256))
        a["c33"] = self._conv("conv3_3", a["c32"], g("c33", R4, 256))
        a["p3"] = ops.maxpool2_fwd(a["c33"], g("p3", R8, 256), ceil_mode=True)
        a["c41"] = self._conv("conv4_1", a["p3"], g("c41", R8, 512))
        a["c42"] = self._conv("conv4_2", a["c41"], g("c42", R8, 512))
        return a

    @staticmethod
    def taps(a):
        """The four reference taps: (conv1_1, conv1_2, conv3_2 [= pool2 output], conv4_2)."""
        return a["c11"], a["c12"], a["p2"], a["c42"]

    def backward(self, a, targets, coefs, ws, tag):
        """∂/∂x of Σ_k coefs[k]/2·‖tap_k − targets[k]‖² (coefs already include 2/numel and the
        loss weight). Returns (N,R,R,8) in the compute dtype."""
        t11, t12, tp2, t42 = targets
        c1, c2, c3, c4 = coefs
        T = self.dtype
        x = a["x"]
        N, R = x.shape[0], x.shape[1]

        def buf(k, like):
            return ws.get(f"vg.{k}", like.shape, T)  # shared by both VGG passes

        L = self.layers
        g = ops.tap_grad(a["c42"], t42, buf("c42", a["c42"]), c4, mask=True)
        g = ops.conv3x3(g, L["conv4_2"]["wd"], buf("c41", a["c41"]), cout=512, mask_a=a["c41"])
        g = ops.conv3x3(g, L["conv4_1"]["wd"], buf("p3", a["p3"]), cout=256)
        g = ops.maxpool2_bwd(a["c33"], g, buf("c33", a["c33"]), ceil_mode=True, mask=True)
        g = ops.conv3x3(g, L["conv3_3"]["wd"], buf("c32", a["c32"]), cout=256, mask_a=a["c32"])
        g = ops.conv3x3(g, L["conv3_2"]["wd"], buf("c31", a["c31"]), cout=256, mask_a=a["c31"])
        g = ops.conv3x3(g, L["conv3_1"]["wd"], buf("p2", a["p2"]), cout=128, tap_a=a["p2"],
                        tap_t=tp2, tap_coef=c3)
        g = ops.maxpool2_bwd(a["c22"], g, buf("c22", a["c22"]), mask=True)
        g = ops.conv3x3(g, L["conv2_2"]["wd"], buf("c21", a["c21"]), cout=128, mask_a=a["c21"])
        g = ops.conv3x3(g, L["conv2_1"]["wd"], buf("p1", a["p1"]), cout=64)
        g = ops.maxpool2_bwd(a["c12"], g, buf("c12", a["c12"]), tap_t=t12, tap_coef=c2, mask=True)
        g = ops.conv3x3(g, L["conv1_2"]["wd"], buf("c11", a["c11"]), cout=64, tap_a=a["c11"],
                        tap_t=t11, tap_coef=c1, mask_a=a["c11"])
        gx = ws.get(f"vg{tag}.x", (N, R, R, CPAD), T)
        ops.conv3x3(g, L["conv1_1"]["wd"], gx, cout=CPAD, flops=2 * N * R * R * 9 * 64 * 3)
        return gx
