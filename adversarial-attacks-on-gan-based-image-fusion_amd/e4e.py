"""e4e encoder (``Encoder4Editing(50, 'ir_se')``) on libmiattack kernels: forward and input gradient.

Behind the reference's ``net.encoder`` slot: ``net.encoder(x) -> (N, n_latent, 512)``
(code/attack/attack_main2.py:597,622; built at code/utils/model_utils.py:24). The module is an
un-vendored dependency (omertov/encoder4editing ``models/encoders/psp_encoders.py``); its
algorithm is restated in oracle/encoder_ref.py, which the parity tests compare against.

Structure (eval mode):
  input_layer  conv3×3(3→64) · BN · PReLU                                   at R² (R = 256)
  body         24 bottleneck_IR_SE units (IR-SE50: 3/4/14/3 units of 64/128/256/512 ch, the first
               of each stage stride 2):  out = SE(BN2(conv2_s(PReLU(conv1(BN1(x)))))) + shortcut
               shortcut = MaxPool2d(1, s) (= x[::s, ::s]) or BN(conv1×1_s(x))
  FPN          p2 = up(c3) + latlayer1(c2),  p1 = up(p2) + latlayer2(c1)  (bilinear, align_corners)
  styles       14 (18 at 1024²) GradualStyleBlocks: log2(16|32|64) × (conv3×3 s2 + LeakyReLU(0.01))
               → EqualLinear; w[:, 0] = style_0(c3), w[:, i] = style_0(c3) + style_i(c3|p2|p1)

Kernel mapping (include/miattack.h):
  * every conv → the MFMA implicit-GEMM kernels: stride-1 3×3 on the halo kernel, stride-2 3×3 and
    1×1 on the generic kernel via mia_conv2d; their input gradients likewise, the stride-2 adjoint
    as four sub-pixel phase groups in ONE launch (layouts.s2_dgrad_phases);
  * BatchNorm after a conv is folded into its weights + bias (exact); the BN before conv1 (BN1)
    cannot fold (zero padding) and is applied as the second output of the previous unit's
    residual-add kernel (mia_se_apply), its scale folded into conv1's dgrad weights;
  * PReLU / LeakyReLU in the conv epilogue (MIA_ACT_PRELU), their backward as the dgrad epilogue's
    slope mask (mask_a / mask_slope), the SE average pool as the conv epilogue's channel sum
    (csum), the SE MLPs and the rest in csrc/encoder.hip.

Layout: NHWC feature maps in the compute dtype; the input is the VGG input tensor x' (N, R, R, 8)
(the objective feeds the same avg_pool2d(x, S/256) image to both, attack_main2.py:597,622), so the
encoder's input gradient is ADDED to the VGG input-path gradient and the two share one pooling
adjoint in the PGD update. Stored for the backward: per unit a1 = PReLU(conv1), r = BN2(conv2),
the SE vectors u, s; the head activations; nothing else.
"""
import math

import torch

from . import layouts, ops
from .ops import ACT_PRELU

from .vgg import CPAD
from .weights import (E4E_COARSE, E4E_MIDDLE, E4E_SE_REDUCTION, STYLE_DIM, e4e_style_spatial,
                      e4e_units, n_latent_for)

BN_EPS = 1e-5
BATCH_MAX = 16  # groups per mia_conv2d_batched launch
# the style heads' first convs, one launch per FPN source map (mia_conv2d_planes) instead of one
# per head, where a per-head launch has fewer 128×128 output tiles than MERGE_BELOW_TILES (less
# than one wave of blocks on the chip): measured (fp32, 128 images, profiles/r04_layers_*) the
# c3 heads (16² → 8², 256 tiles per head) 15.9 → 12.4 ms per step merged, the p2 heads (1024
# tiles) 63.5 → 63.5, the p1 heads (4096 tiles) 461.7 → 476.4 (the merged launch's 28 column
# tiles per row tile cycle 99 MB of pre-split weights through L2). 0 = never (A/B:
# MIA_E4E_MERGE_HEADS). fp16 / bf16 (round 5, profiles/r05_layers_fp16_merge_ab.txt): the p2
# heads merged 18.7 → 15.2 ms per step, the p1 heads 112.0 → 111.5 (neutral): the 2-byte types
# merge below 2048 tiles (p2 and c3).
MERGE_HEADS = int(__import__("os").environ.get("MIA_E4E_MERGE_HEADS", "1"))
MERGE_BELOW_TILES = 1024
MERGE_BELOW_TILES_2B = 2048


def _bn_fold(p, pre):
    g = p[pre + ".weight"].double()
    v = p[pre + ".running_var"].double()
    scale = g / torch.sqrt(v + BN_EPS)
    return scale, p[pre + ".bias"].double() - p[pre + ".running_mean"].double() * scale


def _s2_out(h):
    return (h - 1) // 2 + 1  # conv 3×3 / 1×1, stride 2, pad 1 / 0


def _g3(w, ho, pad=1):
    return dict(w=w, kh=3, kw=3, pad=(pad, pad), ho=ho, wo=ho)


def _g1(w, ho):
    return dict(w=w, kh=1, kw=1, ho=ho, wo=ho)


def _phase_groups(phases, h_in):
    """mia_conv2d groups of a stride-2 conv's input gradient onto an h_in × h_in grid."""
    out = []
    for w, py, px in phases:
        ho, wo = (h_in - py + 1) // 2, (h_in - px + 1) // 2
        if ho > 0 and wo > 0:
            out.append(dict(w=w, kh=1 + py, kw=1 + px, ho=ho, wo=wo, a=(2, 2), b=(py, px)))
    return out


class E4EEncoder:
    """Device e4e: ``forward_nhwc(x', ws) -> (N, n_latent, 512)`` fp32, ``backward_nhwc(g_lat, ws,
    g_x')`` adds ∂L/∂x' into the given (N, R, R, 8) tensor."""
    input_nhwc = True

    def __init__(self, p, size, dtype=torch.float16, device="cuda"):
        self.size = int(size)
        self.n_latent = n_latent_for(self.size)
        self.R = min(self.size, 256)
        if self.R != 256:  # the style-head pyramid (16², 32², 64² FPN maps) needs a 256² input
            raise ValueError("E4EEncoder: the encoder runs on 256² inputs (pSp resizes to 256; "
                             f"avg_pool2d for larger images): size {self.size} < 256")
        self.dtype = T = dtype
        self.device = dev = torch.device(device)
        self.latent_avg = p["latent_avg"].float().to(dev)
        f32 = torch.float32

        def dd(t):
            return t.to(f32).contiguous().to(dev)

        def mt(t):
            return t.contiguous().to(dev)

        s0, b0 = _bn_fold(p, "input_layer.1")
        w0 = p["input_layer.0.weight"].double() * s0[:, None, None, None]
        self.in_w = mt(layouts.fwd_matrix(w0, T, cin_pad=CPAD))
        self.in_wd = mt(layouts.dgrad_matrix(w0, T, cin_pad=CPAD))
        self.in_b = dd(b0)
        self.in_slope = dd(p["input_layer.2.weight"])
        self.units = []
        for i, (cin, depth, stride) in enumerate(e4e_units()):
            pre = f"body.{i}"
            U = dict(cin=cin, depth=depth, stride=stride, cr=depth // E4E_SE_REDUCTION)
            g1, h1 = _bn_fold(p, pre + ".res_layer.0")
            U["bn1_g"], U["bn1_b"] = dd(g1), dd(h1)
            w1 = p[pre + ".res_layer.1.weight"].double()
            U["w1"] = mt(layouts.fwd_matrix(w1, T))
            U["w1d"] = mt(layouts.dgrad_matrix(w1 * g1[None, :, None, None], T))  # BN1 scale
            U["slope"] = dd(p[pre + ".res_layer.2.weight"])
            g2, h2 = _bn_fold(p, pre + ".res_layer.4")
            w2 = p[pre + ".res_layer.3.weight"].double() * g2[:, None, None, None]
            U["w2"], U["b2"] = mt(layouts.fwd_matrix(w2, T)), dd(h2)
            if stride == 1:
                U["w2d"] = mt(layouts.dgrad_matrix(w2, T))
            else:
                U["w2d"] = [(mt(m), py, px) for m, py, px in layouts.s2_dgrad_phases(w2, T)]
                U["w2dh"] = mt(layouts.s2_dgrad_halo_matrix(w2, T))
            U["se_w1"] = dd(p[pre + ".res_layer.5.fc1.weight"].reshape(U["cr"], depth))
            U["se_w2"] = dd(p[pre + ".res_layer.5.fc2.weight"].reshape(depth, U["cr"]))
            if cin != depth:
                gs, hs = _bn_fold(p, pre + ".shortcut_layer.1")
                wsc = p[pre + ".shortcut_layer.0.weight"].double().reshape(depth, cin) * gs[:, None]
                U["wsc"], U["bsc"] = mt(layouts.conv1x1_matrix(wsc, T)), dd(hs)
                U["wscd"] = mt(layouts.conv1x1_matrix(wsc.t(), T))
            self.units.append(U)
        # The backward takes PReLU'(pre) from the sign of the stored activation, which equals the
        # sign of pre for slopes ≥ 0. A PReLU with a negative slope (allowed in a trained pSp /
        # e4e checkpoint: nn.PReLU slopes are unconstrained) maps both branches to a > 0, so such a
        # layer's conv writes the pre-activation itself (kept as the backward's branch mask) and
        # its activation comes from one mia_prelu_fwd pass (round 6; verdict r05 item 3).
        self.in_neg = bool((self.in_slope < 0).any())
        for U in self.units:
            U["neg"] = bool((U["slope"] < 0).any())
        self.lat_w, self.lat_wd, self.lat_b = [], [], []
        for name in ("latlayer1", "latlayer2"):
            w = p[name + ".weight"].double().reshape(STYLE_DIM, -1)
            self.lat_w.append(mt(layouts.conv1x1_matrix(w, T)))
            self.lat_wd.append(mt(layouts.conv1x1_matrix(w.t(), T)))
            self.lat_b.append(dd(p[name + ".bias"]))
        self.slope001 = torch.full((STYLE_DIM,), 0.01, dtype=f32, device=dev)
        self.heads = []
        inv = 1.0 / math.sqrt(STYLE_DIM)
        for i in range(self.n_latent):
            sp = e4e_style_spatial(i)
            convs = []
            src = "c3" if i < E4E_COARSE else ("p2" if i < E4E_MIDDLE else "p1")
            h = self.R // {"c3": 16, "p2": 8, "p1": 4}[src]  # head input resolution
            for j in range(int(math.log2(sp))):
                w = p[f"styles.{i}.convs.{2 * j}.weight"].double()
                ho = _s2_out(h)
                halo = ops.s2_dgrad_halo_ok(T, ho, STYLE_DIM, STYLE_DIM) and 2 * ho == h
                convs.append(dict(w=mt(layouts.fwd_matrix(w, T)),
                                  wd=[(mt(m), py, px) for m, py, px in
                                      layouts.s2_dgrad_phases(w, T)],
                                  wdh=mt(layouts.s2_dgrad_halo_matrix(w, T)) if halo else None,
                                  b=dd(p[f"styles.{i}.convs.{2 * j}.bias"])))
                h = ho
            self.heads.append(dict(convs=convs, src=src, h0=self.R // {"c3": 16, "p2": 8,
                                                                     "p1": 4}[src],
                                   lw=dd(p[f"styles.{i}.linear.weight"].double() * inv),
                                   lb=dd(p[f"styles.{i}.linear.bias"])))
        # Level batching: every head activation of resolution r lives in ONE stacked buffer
        # (S_r·N, r, r, 512), head i at slot slot[r][i]; the non-first convs of all heads with the
        # same input resolution run as ONE mia_conv2d_batched launch (group = head: its weights,
        # its image range in and out, its bias at channel offset c_off), their input gradients as
        # one batched launch per sub-pixel phase. Per head the 8²…1² convs are a few tiles each
        # with a 144-step K loop, latency-bound: batched, the 14 heads share that latency.
        outs = {}
        for i, hd in enumerate(self.heads):
            r = hd["h0"]
            hd["res"] = []
            for _ in hd["convs"]:
                r = _s2_out(r)
                hd["res"].append(r)
                outs.setdefault(r, []).append(i)
        self.slot = {r: {i: k for k, i in enumerate(sorted(v))} for r, v in outs.items()}
        self.levels = []  # (r_in, r_out, [(head, conv index)], bias cat)
        for r_in in sorted({r for hd in self.heads for r in hd["res"][:-1]}, reverse=True):
            mem = [(i, j) for i, hd in enumerate(self.heads) for j in range(1, len(hd["convs"]))
                   if hd["res"][j - 1] == r_in]
            bcat = torch.cat([self.heads[i]["convs"][j]["b"] for i, j in mem]).contiguous()
            self.levels.append((r_in, _s2_out(r_in), mem, bcat))
        self.slope_cat = torch.full((max(16, self.n_latent) * STYLE_DIM,), 0.01, dtype=f32,
                                    device=dev)
        # the heads whose first conv reads the same FPN map (7 on p1, 4 on p2): their first-conv
        # input gradients run as ONE multi-source launch with the packed matrices concatenated
        # along K (mia_conv_s2_dgrad_halo_multi) — one write of the source gradient instead of
        # one accumulate per head
        self.src_heads = {}
        for src in ("c3", "p2", "p1"):
            idx = [i for i, hd in enumerate(self.heads) if hd["src"] == src]
            if len(idx) > 1 and all(self.heads[i]["convs"][0]["wdh"] is not None for i in idx):
                # ≤ 8 source tensors per launch (11 fine heads at 1024²: two launches)
                self.src_heads[src] = [
                    (idx[c:c + 8], torch.cat([self.heads[i]["convs"][0]["wdh"]
                                              for i in idx[c:c + 8]]).contiguous())
                    for c in range(0, len(idx), 8)]
        # the heads whose first conv reads the same FPN map, as ONE stride-2 conv with their weights
        # and biases concatenated along Cout; head j's 512 output channels land in its slot of the
        # stacked level buffer (mia_conv2d_planes; slots of one source are consecutive)
        self.src_fwd = {}
        if MERGE_HEADS:
            for src in ("c3", "p2", "p1"):
                idx = [i for i, hd in enumerate(self.heads) if hd["src"] == src]
                if len(idx) < 2:
                    continue
                r = self.heads[idx[0]]["res"][0]
                k0 = self.slot[r][idx[0]]
                if [self.slot[r][i] for i in idx] != list(range(k0, k0 + len(idx))):
                    continue
                self.src_fwd[src] = (idx, k0, r)
        # their concatenated weights / biases, built on the first forward that merges that source
        # (at the bench batch only c3 merges: no p1 / p2 copies are held)
        self._src_cat = {}
        # w = w0 + delta_i: the linear biases of rows i ≥ 1 include style 0's; the backward of
        # style 0 reads the sum of every row (mia_sum_slices)
        b0l = self.heads[0]["lb"]
        self.lin_bias = [b0l] + [(h["lb"] + b0l).contiguous() for h in self.heads[1:]]
        self.flops_fwd_per_image = self._count_flops()

    def _chan_part(self, ws, N, hw, c):
        """fp32 scratch of ops.chan_sum (one buffer, sized for the largest user)."""
        need = N * ops.chan_sum_parts(N, hw) * c
        buf = ws.cache.get("e.chan_part")
        if buf is None or buf.numel() < need:
            buf = torch.empty(need, dtype=torch.float32, device=self.device)
            ws.cache["e.chan_part"] = buf
        return buf

    def _level_buf(self, ws, kind, r, N):
        """Stacked head activations ('a') or their gradients ('g') at resolution r."""
        return self._buf(ws, f"h{kind}{r}", (len(self.slot[r]) * N, r, r, STYLE_DIM))

    def _head_view(self, ws, kind, i, j, N):
        r = self.heads[i]["res"][j]
        k = self.slot[r][i]
        return self._level_buf(ws, kind, r, N)[k * N:(k + 1) * N]

    def _feat_stack(self, ws, name, N):
        """(n_latent, N, 512) fp32: the heads' 512-vectors (f) or their gradients (gf)."""
        return self._buf(ws, name, (self.n_latent, N, STYLE_DIM), torch.float32)

    # ------------------------------------------------------------------------------------------
    def _count_flops(self):
        """Algorithmic conv/linear FLOPs of one forward at R² (the encoder's share of the
        SURVEY.md §8d per-image work; ≈118 GFLOP at R = 256)."""
        R = self.R
        mac = R * R * 9 * 3 * 64
        h = R
        res = {}
        for i, U in enumerate(self.units):
            ho = _s2_out(h) if U["stride"] == 2 else h
            mac += h * h * 9 * U["cin"] * U["depth"] + ho * ho * 9 * U["depth"] ** 2
            if U["cin"] != U["depth"]:
                mac += ho * ho * U["cin"] * U["depth"]
            h = ho
            res[i] = h
        h1, h2 = res[6], res[20]
        mac += h2 * h2 * 256 * STYLE_DIM + h1 * h1 * 128 * STYLE_DIM
        for hd in self.heads:
            h = {"c3": res[23], "p2": h2, "p1": h1}[hd["src"]]
            for _ in hd["convs"]:
                h = _s2_out(h)
                mac += h * h * 9 * STYLE_DIM * STYLE_DIM
            mac += STYLE_DIM * STYLE_DIM
        return 2 * mac

    def _buf(self, ws, name, shape, dtype=None):
        return ws.get("e." + name, shape, dtype or self.dtype)

    def _check_input(self, x):
        if x.dim() != 4 or x.shape[1] != x.shape[2] or x.shape[3] != CPAD or x.dtype != self.dtype:
            raise ValueError(f"e4e input must be (N, R, R, {CPAD}) {self.dtype} (the VGG input)")

    # ------------------------------------------------------------------------------------------
    def forward_nhwc(self, xin, ws, tag="e"):
        self._check_input(xin)
        N, R = xin.shape[0], xin.shape[1]
        f32 = torch.float32
        a0 = self._buf(ws, "a0", (N, R, R, 64))
        if self.in_neg:  # keep pre for the backward's mask, activation in a second pass
            m0 = self._buf(ws, "m0", (N, R, R, 64))
            ops.conv2d(xin, [_g3(self.in_w, R)], m0, (R, R), cout=64, bias=self.in_b)
            ops.prelu_fwd(m0, self.in_slope, a0)
        else:
            m0 = a0
            ops.conv2d(xin, [_g3(self.in_w, R)], a0, (R, R), cout=64, bias=self.in_b,
                       act_out=ACT_PRELU, act_slope=self.in_slope)
        self._m0 = m0  # the input PReLU's branch mask (m0 > 0 ⟺ pre > 0)
        U0 = self.units[0]
        xb = ops.se_apply(a0, None, None, 1, None, U0["bn1_g"], U0["bn1_b"],
                          self._buf(ws, "xb0", a0.shape))
        x, h = a0, R
        self._a0 = a0
        feats = {}
        for i, U in enumerate(self.units):
            d, s = U["depth"], U["stride"]
            ho = _s2_out(h) if s == 2 else h
            a1 = self._buf(ws, f"a1_{i}", (N, h, h, d))
            if U["neg"]:
                m1 = self._buf(ws, f"m1_{i}", (N, h, h, d))
                ops.conv2d(xb, [_g3(U["w1"], h)], m1, (h, h), cout=d)
                ops.prelu_fwd(m1, U["slope"], a1)
            else:
                m1 = a1
                ops.conv2d(xb, [_g3(U["w1"], h)], a1, (h, h), cout=d, act_out=ACT_PRELU,
                           act_slope=U["slope"])
            r = self._buf(ws, f"r_{i}", (N, ho, ho, d))
            ops.conv2d(a1, [_g3(U["w2"], ho)], r, (ho, ho), cout=d, stride=s, bias=U["b2"])
            # the SE average pool's sum: an ordered two-pass reduction with per-image pixel
            # chunks (mia_chan_sum's partials, finished in chunk order inside the SE kernel), so
            # the forward — and the PReLU / ReLU branches after it — reproduce bit for bit run to
            # run and batch to batch
            part = ops.chan_sum(r, None, self._chan_part(ws, N, ho * ho, d), None)
            u = self._buf(ws, f"u_{i}", (N, U["cr"]), f32)
            sv = self._buf(ws, f"s_{i}", (N, d), f32)
            ops.se_fwd_parts(part, ho * ho, U["se_w1"], U["se_w2"], u, sv)
            if U["cin"] != d:
                sc = self._buf(ws, f"sc_{i}", (N, ho, ho, d))
                ops.conv2d(x, [_g1(U["wsc"], ho)], sc, (ho, ho), cout=d, stride=s, bias=U["bsc"])
                ss = 1
            else:
                sc, ss = x, s
            out = self._buf(ws, f"out_{i}", (N, ho, ho, d))
            if i + 1 < len(self.units):
                Un = self.units[i + 1]
                xb = self._buf(ws, f"xb{i + 1}", out.shape)
                ops.se_apply(r, sv, sc, ss, out, Un["bn1_g"], Un["bn1_b"], xb)
            else:
                ops.se_apply(r, sv, sc, ss, out)
            U["_a1"], U["_m1"], U["_r"], U["_u"], U["_s"], U["_hw"] = a1, m1, r, u, sv, ho * ho
            x, h = out, ho
            if i in (6, 20, 23):
                feats[{6: "c1", 20: "c2", 23: "c3"}[i]] = out
        c1, c2, c3 = feats["c1"], feats["c2"], feats["c3"]
        h1, h2 = c1.shape[1], c2.shape[1]
        p2 = ops.bilinear_fwd(c3, self._buf(ws, "p2", (N, h2, h2, STYLE_DIM)))
        ops.conv2d(c2, [_g1(self.lat_w[0], h2)], p2, (h2, h2), cout=STYLE_DIM,
                   bias=self.lat_b[0], accumulate=True)
        p1 = ops.bilinear_fwd(p2, self._buf(ws, "p1", (N, h1, h1, STYLE_DIM)))
        ops.conv2d(c1, [_g1(self.lat_w[1], h1)], p1, (h1, h1), cout=STYLE_DIM,
                   bias=self.lat_b[1], accumulate=True)
        feats.update(p2=p2, p1=p1)
        self._feats = feats
        # style heads: the first conv of each head from its FPN map into the head's slot of the
        # stacked level buffer, then one batched launch per resolution level
        merged = set()
        for src, (idx, k0, r) in self.src_fwd.items():
            lim = MERGE_BELOW_TILES if self.dtype == torch.float32 else MERGE_BELOW_TILES_2B
            if -(-N * r * r // 128) * (STYLE_DIM // 128) >= lim:
                continue  # enough tiles per head: one launch per head
            merged.update(idx)
            if src not in self._src_cat:
                self._src_cat[src] = (
                    torch.cat([self.heads[i]["convs"][0]["w"] for i in idx]),
                    torch.cat([self.heads[i]["convs"][0]["b"] for i in idx]))
            wcat, bcat = self._src_cat[src]
            ops.conv2d_planes(feats[src], wcat, bcat,
                              self._level_buf(ws, "a", r, N)[k0 * N:(k0 + len(idx)) * N], (r, r),
                              planes=len(idx), act_out=ACT_PRELU, act_slope=self.slope_cat)
        for i, hd in enumerate(self.heads):
            if i in merged:
                continue
            x = feats[hd["src"]]
            cv = hd["convs"][0]
            r = hd["res"][0]
            ops.conv2d(x, [_g3(cv["w"], r)], self._head_view(ws, "a", i, 0, N), (r, r),
                       cout=STYLE_DIM, stride=2, bias=cv["b"], act_out=ACT_PRELU,
                       act_slope=self.slope001)
        for r_in, r_out, mem, bcat in self.levels:
            groups = [dict(_g3(self.heads[i]["convs"][j]["w"], r_out),
                           n_in=self.slot[r_in][i] * N, n_out=self.slot[r_out][i] * N,
                           c_off=k * STYLE_DIM) for k, (i, j) in enumerate(mem)]
            for c in range(0, len(groups), BATCH_MAX):  # ≤ 16 groups per launch (18 heads at 1024²)
                ops.conv2d_batched(self._level_buf(ws, "a", r_in, N), groups[c:c + BATCH_MAX],
                                   self._level_buf(ws, "a", r_out, N), (r_out, r_out), n=N,
                                   cout=STYLE_DIM, stride=2, bias=bcat, act_out=ACT_PRELU,
                                   act_slope=self.slope_cat)
        for i, hd in enumerate(self.heads):
            if hd["res"][-1] != 1:
                raise ValueError("GradualStyleBlock must end at 1×1 (encoder input R = 256)")
            hd["_acts"] = [self._head_view(ws, "a", i, j, N) for j in range(len(hd["convs"]))]
        # the 1×1 activations of all heads (stacked in head order) → the fp32 feature stack
        ops.cast(self._level_buf(ws, "a", 1, N), self._feat_stack(ws, "fst", N))
        lat = ws.get(f"{tag}.lat", (N, self.n_latent, STYLE_DIM), f32)
        self._plan(ws, N, "fwd", lat).run()
        return lat

    def _plan(self, ws, N, kind, lat):
        # cached in the workspace (a plan keeps its operand tensors alive): a fresh AttackEngine
        # per attack() call must not pin the previous calls' buffers through the encoder
        plans = ws.cache.setdefault("e4e.plans", {})
        key = (id(self), kind, N, lat.data_ptr())
        plan = plans.get(key)
        if plan is not None:
            return plan
        f32 = torch.float32
        S, D = self.n_latent, STYLE_DIM
        plan = ops.GemmPlan()
        f = list(self._feat_stack(ws, "fst", N).unbind(0))  # head i = slot i at 1×1
        if kind == "fwd":  # lat[:, i] = f_i·W_iᵀ (+ f_0·W_0ᵀ) + b
            for i, hd in enumerate(self.heads):
                segs = [(f[i], D, 1, hd["lw"], 1, D, D)]
                if i > 0:
                    segs.append((f[0], D, 1, self.heads[0]["lw"], 1, D, D))
                plan.add(lat[:, i, :], S * D, 1, N, D, segs, bias=self.lin_bias[i])
        else:  # ∂f_i = ∂lat[:, i]·W_i (i ≥ 1); ∂f_0 = Σ_i ∂lat[:, i]·W_0
            gf = list(self._feat_stack(ws, "gfst", N).unbind(0))
            gsum = self._buf(ws, "gsum", (N, D), f32)  # Σ_i ∂lat[:, i] (backward_nhwc)
            plan.add(gf[0], D, 1, N, D, [(gsum, D, 1, self.heads[0]["lw"], D, 1, D)])
            for i in range(1, S):
                plan.add(gf[i], D, 1, N, D, [(lat[:, i, :], S * D, 1, self.heads[i]["lw"], D, 1,
                                              D)])
        plans[key] = plan
        return plan

    @staticmethod
    def _s2_dgrad(g, phases, w_halo, y, mask, slope, accumulate):
        """Input gradient of a stride-2 3×3 conv into y: one halo-tiled launch where it applies
        (fp16/bf16, g side a multiple of 16, y exactly twice g), else the 4 phase GEMMs."""
        R, h = g.shape[1], y.shape[1]
        if w_halo is not None and h == 2 * R and ops.s2_dgrad_halo_ok(g.dtype, R, g.shape[-1],
                                                                      y.shape[-1]):
            ops.s2_dgrad_halo(g, w_halo, y, mask_a=mask, mask_slope=slope if mask is not None
                              else None, accumulate=accumulate)
        else:
            ops.conv2d(g, _phase_groups(phases, h), y, (h, h), cout=y.shape[-1], mask_a=mask,
                       mask_slope=slope if mask is not None else None, accumulate=accumulate)

    # ------------------------------------------------------------------------------------------
    def backward_nhwc(self, g_lat, ws, g_xin, accumulate=True):
        """Adds (or writes) ∂L/∂x' for ∂L/∂lat = g_lat (N, n_latent, 512) fp32 into g_xin."""
        N = g_lat.shape[0]
        self._check_input(g_xin)
        R = g_xin.shape[1]
        f32 = torch.float32
        D = STYLE_DIM
        feats = self._feats
        ops.sum_slices(g_lat, self._buf(ws, "gsum", (N, D), f32))
        self._plan(ws, N, "bwd", g_lat).run()
        gfeat = {k: self._buf(ws, "g" + k, feats[k].shape) for k in ("c3", "p2", "p1")}
        # style heads: the 1×1 gradients of all heads in one cast + LeakyReLU' pass, then the
        # batched levels top-down (one launch per sub-pixel phase; the 32² → 16² level of the fine
        # heads per head on the split-once halo kernel), then the first convs' input gradients
        # into the FPN maps (one multi-source launch per map where the halo kernel applies)
        g1 = self._level_buf(ws, "g", 1, N)
        ops.cast(self._feat_stack(ws, "gfst", N), g1)
        ops.prelu_bwd_scale(g1, self._level_buf(ws, "a", 1, N), self.slope001, g1)
        for r_in, r_out, mem, _ in reversed(self.levels):
            gin, gout = self._level_buf(ws, "g", r_out, N), self._level_buf(ws, "g", r_in, N)
            mask = self._level_buf(ws, "a", r_in, N)
            cv0 = self.heads[mem[0][0]]["convs"][mem[0][1]]
            if cv0["wdh"] is not None and all(self.heads[i]["convs"][j]["wdh"] is not None
                                              for i, j in mem):
                for i, j in mem:
                    ops.s2_dgrad_halo(self._head_view(ws, "g", i, j, N),
                                      self.heads[i]["convs"][j]["wdh"],
                                      self._head_view(ws, "g", i, j - 1, N),
                                      mask_a=self._head_view(ws, "a", i, j - 1, N),
                                      mask_slope=self.slope001)
                continue
            for ph in range(4):
                groups = []
                for k, (i, j) in enumerate(mem):
                    pg = _phase_groups([self.heads[i]["convs"][j]["wd"][ph]], r_in)
                    if pg:
                        groups.append(dict(pg[0], n_in=self.slot[r_out][i] * N,
                                           n_out=self.slot[r_in][i] * N, c_off=k * STYLE_DIM))
                for c in range(0, len(groups), BATCH_MAX):
                    ops.conv2d_batched(gin, groups[c:c + BATCH_MAX], gout, (r_in, r_in), n=N,
                                       cout=STYLE_DIM, mask_a=mask, mask_slope=self.slope_cat)
        seen = set()
        for src, chunks in self.src_heads.items():
            for c, (idx, wcat) in enumerate(chunks):
                ops.s2_dgrad_halo([self._head_view(ws, "g", i, 0, N) for i in idx], wcat,
                                  gfeat[src], accumulate=c > 0)
            seen.add(src)
        for i in reversed(range(self.n_latent)):
            hd = self.heads[i]
            if hd["src"] in self.src_heads:
                continue
            cv = hd["convs"][0]
            self._s2_dgrad(self._head_view(ws, "g", i, 0, N), cv["wd"], cv["wdh"],
                           gfeat[hd["src"]], None, self.slope001, hd["src"] in seen)
            seen.add(hd["src"])
        dbg = getattr(self, "debug", None)  # tests: dict to receive intermediate gradients
        if dbg is not None:
            dbg.update({"heads." + k: v.clone() for k, v in gfeat.items()})
        # FPN: p1 = up(p2) + lat2(c1), p2 = up(c3) + lat1(c2)
        U = self.units
        G = {i: self._buf(ws, f"G{i}", self.units[i]["_r"].shape) for i in (6, 20)}
        h1, h2 = feats["c1"].shape[1], feats["c2"].shape[1]
        ops.conv2d(gfeat["p1"], [_g1(self.lat_wd[1], h1)], G[6], (h1, h1), cout=128)
        ops.bilinear_bwd(gfeat["p1"], gfeat["p2"], accumulate=True)
        ops.conv2d(gfeat["p2"], [_g1(self.lat_wd[0], h2)], G[20], (h2, h2), cout=256)
        ops.bilinear_bwd(gfeat["p2"], gfeat["c3"], accumulate=True)
        if dbg is not None:
            dbg.update({"fpn.c3": gfeat["c3"].clone(), "fpn.c2": G[20].clone(),
                        "fpn.p2": gfeat["p2"].clone(),
                        "fpn.c1": G[6].clone()})
        # body, unit 23 → 0; Gc = ∂L/∂out_i
        Gc = gfeat["c3"]
        for i in reversed(range(len(U))):
            u = U[i]
            d, s, cin = u["depth"], u["stride"], u["cin"]
            h = u["_a1"].shape[1]
            part = ops.chan_sum(Gc, u["_r"], self._chan_part(ws, N, u["_hw"], d), None)
            gavg = ops.se_bwd_parts(part, u["_hw"], u["_s"], u["_u"], u["se_w1"], u["se_w2"],
                                    self._buf(ws, "gavg", (N, d), f32))
            g_r = ops.se_grad_scale(Gc, u["_s"], gavg, self._buf(ws, f"g_r{d}", Gc.shape))
            gp1 = self._buf(ws, f"gp1_{h}_{d}", (N, h, h, d))
            if s == 1:
                ops.conv2d(g_r, [_g3(u["w2d"], h)], gp1, (h, h), cout=d, mask_a=u["_m1"],
                           mask_slope=u["slope"])
            else:
                self._s2_dgrad(g_r, u["w2d"], u["w2dh"], gp1, u["_m1"], u["slope"], False)
            if cin == d and s == 1:  # identity shortcut: ∂x = γ1·dgrad + ∂out, in place
                tgt, acc = Gc, True
            elif i == 0:
                tgt, acc = self._buf(ws, "ga0", (N, h, h, cin)), False
            else:
                tgt = G.get(i - 1)
                acc = tgt is not None  # FPN lateral gradient already there (c1, c2)
                if tgt is None:
                    tgt = self._buf(ws, f"G{i - 1}", (N, h, h, cin))
            ops.conv2d(gp1, [_g3(u["w1d"], h)], tgt, (h, h), cout=cin, accumulate=acc)
            if cin != d:
                ho = Gc.shape[1]
                ops.conv2d(Gc, [dict(w=u["wscd"], kh=1, kw=1, ho=ho, wo=ho, a=(s, s))], tgt,
                           (h, h), cout=cin, accumulate=True)
            elif s == 2:
                ops.subsample_add(Gc, tgt)
            Gc = tgt
            if dbg is not None:
                dbg[f"in{i}"] = Gc.clone()
        gp0 = ops.prelu_bwd_scale(Gc, self._m0, self.in_slope, self._buf(ws, "gp0", Gc.shape))
        ops.conv2d(gp0, [_g3(self.in_wd, R)], g_xin, (R, R), cout=CPAD, accumulate=accumulate)
        return g_xin

    # ------------------------------------------------------------------------------------------
    def forward(self, x, ws, tag="e"):
        """x: (N,3,S,S) fp32 image → latents; pools to R² and packs NHWC like the VGG input."""
        N, S = x.shape[0], x.shape[-1]
        xin = ws.get(f"{tag}.xin", (N, self.R, self.R, CPAD), self.dtype)
        ops.image_to_nhwc(x, xin, S // self.R, CPAD)
        return self.forward_nhwc(xin, ws, tag)

    def __call__(self, x):
        from .workspace import Workspace
        ws = Workspace(x.device)
        return self.forward(x.float().contiguous(), ws).clone()
