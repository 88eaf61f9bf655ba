"""StyleGAN2 synthesis network on libmiattack kernels: forward and input/style backward.

Behind the reference's ``net.decoder`` slot: ``decoder([w+], input_is_latent=True,
randomize_noise=False, return_latents=True) -> (img, latents)`` (code/attack/attack_main2.py:619-621,
code/attack/interpolation.py:780-782) and ``decoder.size`` (attack_main2.py:590). The network is the
rosinality generator (un-vendored dependency, see oracle/stylegan2_ref.py) with the mapping MLP
omitted (the attack always passes W+ latents).

Layout in HBM: every feature map is NHWC in the compute dtype. Each StyledConv stores only its
activation ``a = lrelu(pre)·√2`` with ``pre = demod·conv(x̃) + noise_w·noise + bias`` (one tensor
per layer, written by the producing epilogue), so the next conv's A-operand prologue is a single
multiply by the style. The backward recovers ``pre = a / lrelu'(a)`` (same sign) where it needs it.
The image/skip path (3 channels) is fp32 NCHW. Styles, demod coefficients and their gradients are
fp32 [N][C].

Backward computes ∂L/∂w+ only (no weight gradients: the pixel gradient does not need them,
SURVEY.md §2.1 note). Per StyledConv, with g_pre = ∂L/∂pre:
    gy = g_pre·demod;  gx̃ = dgrad(gy);  ∂x = gx̃·s;  ∂s = Σ_p gx̃·x − s·Σ_co (Σ_p g_pre·o)·demod²·Wsq
where o = pre − noise_w·noise − bias = demod·conv(x̃) and Wsq[co][ci] = Σ_k (scale·W)².
"""
import math

import torch

from . import layouts, ops
from .ops import ACT_LRELU_S2, ACT_NONE
from .weights import STYLE_DIM, generator_layout, n_latent_for

UP_K = list(layouts.BLUR_F)  # separable ToRGB skip up-sampler (Upsample(blur_kernel), factor 2)
# fp16 / bf16 StyledConv forwards at resolution ≥ WMOD_MIN_RES run on per-image modulated +
# demodulated weights (ops.conv3x3_modw: rosinality's own weight path) instead of modulating the
# input halo in LDS once per channel block: at 128² / 256² an image's weight matrix is read by
# ≥ 128 patch blocks of one XCD (L2-resident), and the halo kernel drops its modulation pass and
# the demod in its epilogue. Below it (≤ 32 patches per image, 512 channels) the per-image
# matrices would not stay in L2. 0 disables (A/B: MIA_G_WMOD_RES).
WMOD_MIN_RES = int(__import__("os").environ.get("MIA_G_WMOD_RES", "128"))


class SynthesisNet:
    def __init__(self, params, size, dtype=torch.float32, device="cuda", channel_multiplier=2,
                 up_mode="subpixel"):
        if up_mode not in ("subpixel", "fused"):
            raise ValueError("up_mode: 'subpixel' (convT phases + blur) or 'fused' (4-phase 3×3)")
        self.up_mode = up_mode
        self.size = int(size)
        self.n_latent = n_latent_for(self.size)
        self.dtype = dtype
        self.device = torch.device(device)
        convs, torgbs = generator_layout(self.size, channel_multiplier)
        dev, f32 = self.device, torch.float32

        def style_params(prefix, cin):
            a = params[prefix + ".modulation.weight"].double() / math.sqrt(STYLE_DIM)
            return (a.to(f32).contiguous().to(dev),
                    params[prefix + ".modulation.bias"].to(f32).contiguous().to(dev))

        self.convs = []
        for c in convs:
            pre = c["name"]
            w = params[pre + ".conv.weight"][0].double()  # (cout, cin, 3, 3)
            cin, cout = c["cin"], c["cout"]
            scale = 1.0 / math.sqrt(cin * 9)
            ws = w * scale
            L = dict(c)
            if c["up"] and up_mode == "subpixel":
                L["wph"] = [m.contiguous().to(dev)
                            for m in layouts.upconv_subpixel_matrices(ws, dtype)]
                if cin % 64 == 0 and cout % 32 == 0:  # halo up-conv tiles of 64 / 32 channels
                    L["wup"] = layouts.upconv_halo_matrix(ws, dtype).contiguous().to(dev)
                L["wd"] = layouts.upconv_dgrad_matrix(ws, dtype).contiguous().to(dev)
            elif c["up"]:
                ph = layouts.upconv_phases(ws)
                L["wf"] = layouts.fwd_matrix(ph, dtype).contiguous().to(dev)
                L["wd"] = layouts.dgrad_matrix(ph, dtype).contiguous().to(dev)
            else:
                L["wf"] = layouts.fwd_matrix(ws, dtype).contiguous().to(dev)
                L["wd"] = layouts.dgrad_matrix(ws, dtype).contiguous().to(dev)
            L["wsq"] = (ws ** 2).sum(dim=(2, 3)).to(f32).contiguous().to(dev)  # [cout][cin]
            L["A"], L["Ab"] = style_params(pre + ".conv", cin)
            L["noise"] = params[f"noises.noise_{c['noise']}"].reshape(-1).to(f32).contiguous().to(dev)
            L["noise_w"] = float(params[pre + ".noise.weight"].reshape(-1)[0])
            L["bias"] = params[pre + ".activate.bias"].to(f32).contiguous().to(dev)
            self.convs.append(L)
        self.torgbs = []
        for t in torgbs:
            pre = t["name"]
            w = params[pre + ".conv.weight"][0, :, :, 0, 0].double()  # (3, cin)
            L = dict(t)
            L["wr"] = (w / math.sqrt(t["cin"])).to(f32).contiguous().to(dev)
            L["A"], L["Ab"] = style_params(pre + ".conv", t["cin"])
            L["bias"] = params[pre + ".bias"].reshape(3).to(f32).contiguous().to(dev)
            self.torgbs.append(L)
        const = params["input.input"][0].permute(1, 2, 0).contiguous()  # (4,4,512) NHWC
        self.const = const.to(dtype).to(dev)
        self.flops_fwd_per_image = sum(self._alg_flops(L, 1) for L in self.convs)

    @staticmethod
    def _alg_flops(L, N):
        """Algorithmic FLOPs of one StyledConv GEMM: 3×3 conv at the
        output resolution, or conv_transpose2d at the input resolution for up-convs (the blur
        folded into the 4-phase kernels is extra work the count does not credit)."""
        r = L["res"] // 2 if L["up"] else L["res"]
        return 2 * N * r * r * 9 * L["cin"] * L["cout"]

    # --------------------------------------------------------------------------------------
    def styles(self, lat, ws):
        """s = w+[:, idx]·(A/√512)ᵀ + b for every modulated conv (one grouped GEMM launch for all
        layers); demod for the StyledConvs."""
        N = lat.shape[0]
        nl = self.n_latent
        key = (lat.data_ptr(), N)
        if getattr(self, "_style_key", None) != key:
            plan = ops.GemmPlan()
            for i, L in enumerate(self.convs + self.torgbs):
                cin = L["cin"]
                s = ws.get(f"g.s{i}", (N, cin), torch.float32)
                wrow = lat[:, L["latent"], :]
                plan.add(s, cin, 1, N, cin,
                         [(wrow, nl * STYLE_DIM, 1, L["A"], 1, STYLE_DIM, STYLE_DIM)],
                         bias=L["Ab"])
                L["_s"] = s
            self._style_plan, self._style_key = plan, key
        self._style_plan.run()
        for i, L in enumerate(self.convs + self.torgbs):
            if "wsq" in L:
                d = ws.get(f"g.d{i}", (N, L["cout"]), torch.float32)
                ops.style_demod(L["_s"], L["wsq"], d)
                L["_d"] = d

    def style_order(self):
        """Modulated layers in generator forward order (conv1, to_rgb1, then per resolution:
        up-conv, conv, to_rgb) as indices into convs + torgbs — the order of SFGenerator's style
        vector (style_fusion_simple.py:126-153)."""
        nc = len(self.convs)
        order = [0, nc]
        for k in range(len(self.torgbs) - 1):
            order += [1 + 2 * k, 2 + 2 * k, nc + 1 + k]
        return order

    def style_vectors(self, lat, ws):
        """Per-layer styles s (fp32 (N, Cin) each) for W+ latents, generator forward order."""
        self.styles(lat, ws)
        layers = self.convs + self.torgbs
        return [layers[i]["_s"].clone() for i in self.style_order()]

    def set_styles(self, styles, ws):
        """Install given per-layer styles (generator forward order) and their demodulation."""
        layers = self.convs + self.torgbs
        order = self.style_order()
        if len(styles) != len(order):
            raise ValueError(f"{len(order)} style vectors expected, got {len(styles)}")
        N = styles[0].shape[0]
        for s_in, i in zip(styles, order):
            L = layers[i]
            if tuple(s_in.shape) != (N, L["cin"]):
                raise ValueError(f"style of layer {L['name']}: shape {tuple(s_in.shape)} != "
                                 f"{(N, L['cin'])}")
            s = ws.get(f"g.s{i}", (N, L["cin"]), torch.float32)
            s.copy_(s_in)
            L["_s"] = s
            if "wsq" in L:
                d = ws.get(f"g.d{i}", (N, L["cout"]), torch.float32)
                ops.style_demod(s, L["wsq"], d)
                L["_d"] = d
        self._style_key = None  # the W+ → s plan no longer describes the installed styles

    def forward_styles(self, styles, ws):
        """Image from per-layer styles (SFGenerator style_vector path)."""
        self.set_styles(styles, ws)
        return self._synthesize(styles[0].shape[0], ws)

    def forward(self, lat, ws):
        """lat: (N, n_latent, 512) fp32 → image (N,3,S,S) fp32 (the rosinality ``skip``)."""
        N = lat.shape[0]
        if tuple(lat.shape[1:]) != (self.n_latent, STYLE_DIM) or lat.dtype != torch.float32:
            raise ValueError(f"latent must be (N,{self.n_latent},512) fp32")
        self.styles(lat, ws)
        return self._synthesize(N, ws)

    def _wmod(self, L):
        """Does StyledConv L run on per-image modulated weights (ops.conv3x3_modw)?"""
        r = L["res"]
        return (not L["up"] and self.dtype != torch.float32 and WMOD_MIN_RES
                and r >= WMOD_MIN_RES and r % 16 == 0 and L["cout"] > 64)

    def _synthesize(self, N, ws):
        T = self.dtype
        # one workspace buffer for every layer's per-image weights: they are written and read
        # inside that layer's forward only (no backward reads them), so the layers share it
        wm_numel = max((N * L["wf"].numel() for L in self.convs if self._wmod(L)), default=0)
        wm_buf = ws.get("g.wmod", (wm_numel,), T) if wm_numel else None
        x0 = ws.get("g.const", (N, 4, 4, self.const.shape[-1]), T)
        ops.repeat(self.const, x0, N)
        x = x0
        rgb = None
        ti = 0
        for i, L in enumerate(self.convs):
            r, cout = L["res"], L["cout"]
            pre = ws.get(f"g.pre{i}", (N, r, r, cout), T)
            if L["up"] and self.up_mode == "subpixel":
                t = ws.get(f"g.t{i}", (N, r + 1, r + 1, cout), T)
                ops.upconv_fwd(x, L["wph"], t, cout, style=L["_s"], flops=self._alg_flops(L, N),
                               w_up=L.get("wup"))
                ops.upconv_blur_fwd(t, pre, L["_d"], L["noise"], L["noise_w"], L["bias"],
                                    act_out=ACT_LRELU_S2)
            elif self._wmod(L):
                wm = wm_buf[:N * L["wf"].numel()].view((N,) + tuple(L["wf"].shape))
                ops.conv3x3_modw(x, L["wf"], pre, wm, cout=cout, in_scale=L["_s"],
                                 out_scale=L["_d"], noise=L["noise"], noise_w=L["noise_w"],
                                 bias=L["bias"], act_out=ACT_LRELU_S2,
                                 flops=self._alg_flops(L, N))
            else:
                ops.conv3x3(x, L["wf"], pre, cout=4 * cout if L["up"] else cout,
                            in_scale=L["_s"], out_scale=L["_d"], noise=L["noise"],
                            noise_w=L["noise_w"], bias=L["bias"], act_out=ACT_LRELU_S2,
                            shuffle_out=L["up"], flops=self._alg_flops(L, N))
            L["_x"], L["_pre"] = x, pre  # _pre holds the activation a = lrelu(pre)·√2
            x = pre
            if not L["up"]:  # every non-up conv closes a resolution → ToRGB
                t = self.torgbs[ti]
                out = ws.get(f"g.rgb{ti}", (N, 3, r, r), torch.float32)
                ops.torgb_fwd(pre, t["_s"], t["wr"], t["bias"], rgb, out, act_in=ACT_NONE)
                t["_pre"], t["_skip"] = pre, rgb
                rgb = out
                ti += 1
        return rgb

    # --------------------------------------------------------------------------------------
    def backward(self, g_img, g_lat, ws):
        """g_img = ∂L/∂image (N,3,S,S) fp32; accumulates ∂L/∂w+ into g_lat (N,n_latent,512)."""
        if self.up_mode == "subpixel":
            self._backward_fused(g_img, ws)
        else:
            self._backward_unfused(g_img, ws)
        self._style_backward(g_lat, ws)
        return g_lat

    def _torgb_step(self, i, ti, g_rgb, ws, front=None):
        """ToRGB backward for the (non-up) conv i: writes its activation gradient into "g.ga{i}"
        (not accumulated) and its style gradient; returns the skip-path gradient (or None).
        ``front=(gy, q)`` (topmost conv only): also run conv i's backward front into gy / q."""
        N = g_rgb.shape[0]
        L, t = self.convs[i], self.torgbs[ti]
        r = L["res"]
        gs_t = ops.zero_(ws.get(f"g.gs_rgb{ti}", (N, t["cin"]), torch.float32))
        if front is not None:
            gy, q = front
            ops.torgb_bwd_front(g_rgb, L["_pre"], t["_s"], t["wr"], gy, gs_t, L["_d"], L["noise"],
                                L["noise_w"], L["bias"], q)
        else:
            ga = ws.get(f"g.ga{i}", (N, r, r, L["cout"]), self.dtype)
            ops.torgb_bwd(g_rgb, L["_pre"], t["_s"], t["wr"], ga, gs_t, accumulate=False,
                          act_in=ACT_NONE)
        t["_gs"] = gs_t
        if t["_skip"] is None:
            return None
        g_skip = ws.get(f"g.gskip{ti}", (N, 3, r // 2, r // 2), torch.float32)
        ops.upfirdn2d_bwd(g_rgb, g_skip, UP_K, up=2, pad=(2, 1))
        return g_skip

    def _backward_fused(self, g_img, ws):
        """Top-down; each conv's dgrad epilogue also runs the backward front of the conv below it
        (ToRGB gradient accumulated, lrelu', demod scale and the q = Σ_p g_pre·o reduction:
        mia_conv_args.bab_*); the topmost conv's front is fused into its ToRGB backward
        (mia_torgb_bwd_front)."""
        N = g_img.shape[0]
        T = self.dtype
        last = len(self.convs) - 1
        ti = len(self.torgbs) - 1
        Lt = self.convs[last]
        q = ops.zero_(ws.get(f"g.q{last}", (N, Lt["cout"]), torch.float32))
        gy = ws.get(f"g.gy{last}", (N, Lt["res"], Lt["res"], Lt["cout"]), T)
        g_rgb = self._torgb_step(last, ti, g_img, ws, front=(gy, q))
        ti -= 1
        for i in range(last, -1, -1):
            L = self.convs[i]
            r, cout, cin = L["res"], L["cout"], L["cin"]
            gs = ops.zero_(ws.get(f"g.gs{i}", (N, cin), torch.float32))
            rin = r // 2 if L["up"] else r
            out, bab, acc, q_below = None, None, False, None
            if i > 0:
                Lb = self.convs[i - 1]
                if not Lb["up"]:
                    g_rgb = self._torgb_step(i - 1, ti, g_rgb, ws)  # writes g.ga{i-1}
                    ti -= 1
                    acc = True
                out = ws.get(f"g.ga{i - 1}", (N, rin, rin, cin), T)
                q_below = ops.zero_(ws.get(f"g.q{i - 1}", (N, cin), torch.float32))
                bab = dict(demod=Lb["_d"], noise=Lb["noise"], noise_w=Lb["noise_w"],
                           bias=Lb["bias"], q=q_below)
            if L["up"]:
                gt = ws.get(f"g.gt{i}", (N, r + 1, r + 1, cout), T)
                ops.upconv_blur_bwd(gy, gt)
                if bab is not None:
                    ops.upconv_dgrad_fused(gt, L["wd"], out, cin, L["_x"], L["_s"], gs, bab, acc,
                                           flops=self._alg_flops(L, N))
                else:
                    ops.upconv_dgrad(gt, L["wd"], None, cin, L["_x"], ACT_NONE, L["_s"], gs,
                                     flops=self._alg_flops(L, N))
            else:
                ops.conv3x3(gy, L["wd"], out, cout=cin, out_scale=L["_s"], aux_x=L["_x"],
                            act_aux=ACT_NONE, sdot=gs, accumulate=acc, bab=bab,
                            flops=self._alg_flops(L, N))
            ops.demod_bwd(q, L["_d"], L["wsq"], L["_s"], gs)
            L["_gs"] = gs
            gy, q = out, q_below

    def _backward_unfused(self, g_img, ws):
        """Reference order (fused-phase up-convs): ToRGB → bias_act_bwd → dgrad per conv."""
        N = g_img.shape[0]
        T = self.dtype
        g_rgb = g_img
        ti = len(self.torgbs) - 1
        g_a_next = None  # ∂L/∂act of the current conv's output, written by the conv above
        for i in range(len(self.convs) - 1, -1, -1):
            L = self.convs[i]
            r, cout, cin = L["res"], L["cout"], L["cin"]
            pre = L["_pre"]
            if not L["up"]:
                # ToRGB consumes this conv's activation: add its gradient, route the skip gradient
                t = self.torgbs[ti]
                gs_t = ws.get(f"g.gs_rgb{ti}", (N, t["cin"]), torch.float32)
                ops.zero_(gs_t)
                if g_a_next is None:
                    g_a_next = ws.get(f"g.ga{i}", (N, r, r, cout), T)
                    acc = False
                else:
                    acc = True
                ops.torgb_bwd(g_rgb, pre, t["_s"], t["wr"], g_a_next, gs_t, accumulate=acc,
                              act_in=ACT_NONE)
                t["_gs"] = gs_t
                if t["_skip"] is not None:
                    g_skip = ws.get(f"g.gskip{ti}", (N, 3, r // 2, r // 2), torch.float32)
                    ops.upfirdn2d_bwd(g_rgb, g_skip, UP_K, up=2, pad=(2, 1))
                    g_rgb = g_skip
                ti -= 1
            q = ws.get(f"g.q{i}", (N, cout), torch.float32)
            ops.zero_(q)
            if L["up"]:
                gy = ws.get(f"g.gy{i}", (N, r // 2, r // 2, 4 * cout), T)
            else:
                gy = ws.get(f"g.gy{i}", (N, r, r, cout), T)
            ops.bias_act_bwd(g_a_next, pre, L["noise"], L["noise_w"], L["bias"], L["_d"], gy, q,
                             unshuffle=L["up"], from_act=True)
            gs = ws.get(f"g.gs{i}", (N, cin), torch.float32)
            ops.zero_(gs)
            rin = r // 2 if L["up"] else r
            gx = ws.get(f"g.ga{i - 1}", (N, rin, rin, cin), T) if i > 0 else None
            ops.conv3x3(gy, L["wd"], gx, cout=cin, out_scale=L["_s"], aux_x=L["_x"],
                        act_aux=ACT_NONE, sdot=gs, flops=self._alg_flops(L, N))
            ops.demod_bwd(q, L["_d"], L["wsq"], L["_s"], gs)
            L["_gs"] = gs
            g_a_next = gx

    def _style_backward(self, g_lat, ws):
        N = g_lat.shape[0]
        nl = self.n_latent
        # style affine backward: ∂w+[:, j] += Σ_{layers reading latent j} ∂s · (A/√512); one
        # grouped launch, one group per latent row (≤ 2 layers share a row: ToRGB_i and the next
        # up-conv), so no two blocks write the same output.
        key = (g_lat.data_ptr(), N)
        if getattr(self, "_gstyle_key", None) != key:
            users = {}
            for L in self.convs + self.torgbs:
                users.setdefault(L["latent"], []).append(L)
            plan = ops.GemmPlan()
            for j, Ls in sorted(users.items()):
                segs = [(L["_gs"], L["cin"], 1, L["A"], STYLE_DIM, 1, L["cin"]) for L in Ls]
                plan.add(g_lat[:, j, :], nl * STYLE_DIM, 1, N, STYLE_DIM, segs, beta=1.0)
            self._gstyle_plan, self._gstyle_key = plan, key
        self._gstyle_plan.run()
        return g_lat
