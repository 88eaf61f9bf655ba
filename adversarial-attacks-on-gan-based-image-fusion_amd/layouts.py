"""Host-side (once per model) weight re-layout for the MFMA conv kernel.

The kernel computes y[n,p,co] = Σ_{tap,ci} x[n,p+tap,ci]·w[co][tap·Cin+ci] over a 3×3 / pad-1
window (tap = 3·ty + tx, offsets ty−1, tx−1). These helpers produce its weight matrices:

* ``fwd_matrix``      — [Cout][Kpad] from an OIHW 3×3 kernel (VGG conv, StyledConv).
* ``dgrad_matrix``    — [Cin][Kpad'] for the input gradient of that conv: flipped taps, swapped
                        channel roles (a stride-1 pad-1 conv's transpose is again such a conv).
* ``upconv_phases``   — folds ``conv_transpose2d(stride 2, pad 0)`` followed by rosinality's Blur
                        (upfirdn2d, k = [1,3,3,1]⊗[1,3,3,1]/64·4, pad (1,1)) into four 3×3 phase
                        kernels on the low-resolution grid: output pixel (2m+py, 2m'+px) =
                        Σ_t x[m+ty−1, m'+tx−1]·V[py,px][ty,tx] with
                        V[p][t] = Σ_j f[j]·W[1 − 2t + p + j] per axis, f = [1,3,3,1]/4.
                        Demodulation commutes with the (per-channel, linear) blur, so the phase
                        kernels carry the original weights' demod (ModulatedConv2d upsample branch).
"""
import weakref

import torch

BLUR_F = (0.25, 0.75, 0.75, 0.25)


def kpad_for(cin, dtype):
    bk = 32 if dtype == torch.float32 else 64
    return (9 * cin + bk - 1) // bk * bk


def fwd_matrix(w, dtype, cin_pad=None):
    """w: (Cout, Cin, 3, 3) → (Cout, Kpad) with K index = tap·Cin' + ci (Cin' = cin_pad or Cin)."""
    cout, cin = w.shape[:2]
    cp = cin_pad or cin
    wp = torch.zeros(cout, cp, 3, 3, dtype=torch.float64)
    wp[:, :cin] = w.double()
    m = wp.permute(0, 2, 3, 1).reshape(cout, 9 * cp)  # [co][ty][tx][ci]
    out = torch.zeros(cout, kpad_for(cp, dtype), dtype=torch.float64)
    out[:, :9 * cp] = m
    return out.to(dtype)


def dgrad_matrix(w, dtype, cin_pad=None):
    """Weights of the input-gradient conv: Wd[ci][tap'·Cout + co] = w[co][ci][2−ty][2−tx]."""
    cout, cin = w.shape[:2]
    cp = cin_pad or cin
    wt = torch.zeros(cp, cout, 3, 3, dtype=torch.float64)
    wt[:cin] = w.double().transpose(0, 1).flip(2, 3)
    return fwd_matrix(wt, dtype)


def upconv_subpixel_matrices(w, dtype):
    """conv_transpose2d(stride 2) as four sub-pixel phase GEMMs: T[2m+p] = Σ_j x[m−j]·W[p+2j].
    Phase (py,px) has kh = 2−py, kw = 2−px taps; as a window conv with input m + ty − (kh−1),
    tap (ty,tx) ↔ W[py + 2(kh−1−ty)][px + 2(kw−1−tx)]. Returns 4 [Cout][Kpad] matrices."""
    cout, cin = w.shape[:2]
    w = w.double()
    out = []
    for ph in range(4):
        py, px = ph >> 1, ph & 1
        kh, kw = 2 - py, 2 - px
        m = torch.zeros(cout, kh, kw, cin, dtype=torch.float64)
        for ty in range(kh):
            for tx in range(kw):
                m[:, ty, tx, :] = w[:, :, py + 2 * (kh - 1 - ty), px + 2 * (kw - 1 - tx)]
        bk = 32 if dtype == torch.float32 else 64
        kp = (kh * kw * cin + bk - 1) // bk * bk
        full = torch.zeros(cout, kp, dtype=torch.float64)
        full[:, :kh * kw * cin] = m.reshape(cout, -1)
        out.append(full.to(dtype))
    return out


# K-steps of the halo-tiled up-conv (mia_upconv_fwd_halo): input offset (jy, jx) → (−jy, −jx) and
# the phases p = 2·py + px of its two weight slots (None = zero slot)
UPCONV_HALO_STEPS = (((0, 0), (0, 1)), ((0, 0), (2, 3)), ((0, 1), (0, 2)), ((1, 0), (0, 1)),
                     ((1, 1), (0, None)))


def halo_bk(dtype):
    """Channels per 128-B operand row (one K-step of a channel block): 32 fp32, 64 otherwise."""
    return 32 if dtype == torch.float32 else 64


def upconv_halo_matrix(w, dtype):
    """Packed weights of mia_upconv_fwd_halo: (Cin/BK, 5, 2, Cout, BK) with BK = halo_bk(dtype),
    slot weight W[:, ci, py + 2·jy, px + 2·jx] (T[2m+p] = Σ_j x[m−j]·W[p+2j], as
    upconv_subpixel_matrices)."""
    cout, cin = w.shape[:2]
    if cin % 64:
        raise ValueError("Cin must be a multiple of 64")
    bk = halo_bk(dtype)
    w = w.double()
    out = torch.zeros(cin // bk, 5, 2, cout, bk, dtype=torch.float64)
    for st, ((jy, jx), phases) in enumerate(UPCONV_HALO_STEPS):
        for slot, ph in enumerate(phases):
            if ph is None:
                continue
            py, px = ph >> 1, ph & 1
            wk = w[:, :, py + 2 * jy, px + 2 * jx]  # (cout, cin)
            out[:, st, slot] = wk.reshape(cout, cin // bk, bk).permute(1, 0, 2)
    return out.to(dtype)


def upconv_dgrad_matrix(w, dtype):
    """Input gradient of conv_transpose2d(stride 2): gx[i] = Σ_k gT[2i+k]·W[k] — a stride-2 3×3
    conv with Wd[ci][(ky·3+kx)·Cout + co] = W[co][ci][ky][kx] (no flip)."""
    return fwd_matrix(w.double().transpose(0, 1), dtype)


def upconv_phases(w):
    """(Cout, Cin, 3, 3) → (4·Cout, Cin, 3, 3) phase kernels, row index = (2·py+px)·Cout + co."""
    cout, cin = w.shape[:2]
    w = w.double()
    v = torch.zeros(2, 2, cout, cin, 3, 3, dtype=torch.float64)
    for py in range(2):
        for px in range(2):
            for ty in range(3):
                for tx in range(3):
                    acc = torch.zeros(cout, cin, dtype=torch.float64)
                    for jy in range(4):
                        ky = 1 - 2 * ty + py + jy
                        if not 0 <= ky <= 2:
                            continue
                        for jx in range(4):
                            kx = 1 - 2 * tx + px + jx
                            if not 0 <= kx <= 2:
                                continue
                            acc += BLUR_F[jy] * BLUR_F[jx] * w[:, :, ky, kx]
                    v[py, px, :, :, ty, tx] = acc
    return v.reshape(4 * cout, cin, 3, 3)


# ---- e4e encoder: strided convolutions ------------------------------------------------------------
# Input gradient of a stride-2, pad-1 3×3 conv (out[o] = Σ_k in[2o + k − 1]·W[k] per axis) as four
# sub-pixel phase GEMMs over the output gradient g: gin[2i] = g[i]·W[1];
# gin[2i+1] = g[i]·W[2] + g[i+1]·W[0]. Phase p of an axis is a window conv with kh = 1 + p taps,
# pad 0, tap t ↔ kernel index S2_KMAP[p][t], placed at output row 2i + p.
S2_KMAP = ((1,), (2, 0))


def s2_dgrad_phases(w, dtype):
    """w: (Cout, Cin, 3, 3) of the forward stride-2 conv → [(matrix [Cin][Kpad], py, px)] for
    phases p = 2·py + px, K index = (ty·kw + tx)·Cout + co (mia_conv2d groups)."""
    cout, cin = w.shape[:2]
    w = w.double()
    bk = 32 if dtype == torch.float32 else 64
    out = []
    for ph in range(4):
        py, px = ph >> 1, ph & 1
        ky, kx = S2_KMAP[py], S2_KMAP[px]
        m = torch.zeros(cin, len(ky), len(kx), cout, dtype=torch.float64)
        for ty, a in enumerate(ky):
            for tx, b in enumerate(kx):
                m[:, ty, tx, :] = w[:, :, a, b].t()
        k = len(ky) * len(kx) * cout
        full = torch.zeros(cin, (k + bk - 1) // bk * bk, dtype=torch.float64)
        full[:, :k] = m.reshape(cin, -1)
        out.append((full.to(dtype), py, px))
    return out


def conv1x1_matrix(w, dtype):
    """(Cout, Cin[, 1, 1]) → [Cout][Kpad] (K = Cin, zero-padded to the K-step)."""
    w = w.reshape(w.shape[0], -1).double()
    cout, cin = w.shape
    bk = 32 if dtype == torch.float32 else 64
    full = torch.zeros(cout, (cin + bk - 1) // bk * bk, dtype=torch.float64)
    full[:, :cin] = w
    return full.to(dtype)


def s2_dgrad_halo_matrix(w, dtype):
    """Packed weights of mia_conv_s2_dgrad_halo for the forward stride-2 conv w (Cout, Cin, 3, 3):
    the halo up-conv layout of the channel-transposed, spatially flipped kernel (the input
    gradient is the transposed conv mirrored: offsets +j, output phase 1 − p, kernel index
    2 − (p + 2j)). (Cout/BK, 5, 2, Cin, BK)."""
    return upconv_halo_matrix(w.double().transpose(0, 1).flip(2, 3), dtype)


def _hi16(t):
    """Top 16 bits of fp32 words as int64 in [0, 65535]."""
    return (t.view(torch.int32).to(torch.int64) >> 16) & 0xFFFF


def _pack_words(lo16, hi16):
    """Two 16-bit fields → int32 words (bit patterns)."""
    v = lo16 | (hi16 << 16)
    return (v - ((v >> 31) << 32)).to(torch.int32)


def split_f32(w):
    """Pre-split fp32 weights for the split-once kernels (mia_conv_args.w_split,
    csrc/conv_halo_x6.hip; the packed up-conv / stride-2-adjoint weights viewed as rows of their
    last dimension): w [Cout][Kpad] fp32 (Kpad % 4 == 0) → int32 words
    [Cout][Kpad] of per-4-k-quad records [hi0 hi1 hi2 hi3 | mid0 mid1 mid2 mid3] (bf16), then
    [Cout][Kpad/2] words of [lo0 lo1 lo2 lo3] (bf16) — w = hi + mid + lo exactly, hi = w with the
    low 16 bits cleared, mid = (w − hi) likewise, lo = w − hi − mid (conv_common.h split3)."""
    if w.dtype != torch.float32 or w.dim() < 2 or w.shape[-1] % 4:
        raise ValueError("split_f32: [...][Kpad] fp32 with Kpad % 4 == 0 (rows = all but the last "
                         "dimension)")
    dev = w.device
    a = w.detach().to("cpu").contiguous().reshape(-1, w.shape[-1])
    mask = torch.tensor(-65536, dtype=torch.int32)  # 0xffff0000
    hi = (a.view(torch.int32) & mask).view(torch.float32)
    r = a - hi
    mid = (r.view(torch.int32) & mask).view(torch.float32)
    lo = r - mid
    cout, kpad = a.shape
    H, M, L = (_hi16(t).reshape(cout, kpad // 4, 4) for t in (hi, mid, lo))
    hm = torch.stack([_pack_words(H[..., 0], H[..., 1]), _pack_words(H[..., 2], H[..., 3]),
                      _pack_words(M[..., 0], M[..., 1]), _pack_words(M[..., 2], M[..., 3])], -1)
    lw = torch.stack([_pack_words(L[..., 0], L[..., 1]), _pack_words(L[..., 2], L[..., 3])], -1)
    return torch.cat([hm.reshape(-1), lw.reshape(-1)]).to(dev)


# split copies of device fp32 weight matrices, made on first use: data_ptr → (weakref to the
# weight tensor, its version counter, split tensor). An entry is used only while the weakref still
# names the same live tensor and its in-place version is unchanged.
_SPLITS = {}


def split_for(w):
    """The split_f32 copy of a device fp32 weight matrix (cached), or None when the library's fp32
    arithmetic is the native A/B build or w is not fp32."""
    from . import _lib
    if w.dtype != torch.float32 or not w.is_cuda or _lib.F32_ARITH != "bf16x6":
        return None
    key = w.data_ptr()
    e = _SPLITS.get(key)
    if e is not None and e[0]() is w and e[1] == w._version:
        return e[2]
    sp = split_f32(w)

    def _drop(_ref, key=key):
        cur = _SPLITS.get(key)
        if cur is not None and cur[0] is _ref:
            del _SPLITS[key]

    _SPLITS[key] = (weakref.ref(w, _drop), w._version, sp)
    return sp
