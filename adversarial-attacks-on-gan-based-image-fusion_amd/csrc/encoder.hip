// e4e encoder (Encoder4Editing(50, 'ir_se'), behind net.encoder: code/utils/model_utils.py:24,
// code/attack/attack_main2.py:597,622) — the non-conv pieces of its forward and input gradient.
// The convolutions run on the shared MFMA kernels (mia_conv2d / mia_conv3x3); what is left is
// HBM-bound elementwise work on NHWC feature maps and per-(image, channel) vectors:
//   * SEModule(C, 16) of bottleneck_IR_SE: the average pool comes from the conv epilogue (csum),
//     the two 1×1 FCs run per image in one block (C ≤ 512, C/16 ≤ 32), the channel scale and the
//     residual add run fused with the NEXT unit's BatchNorm (two outputs from one read);
//   * their adjoints (channel dot, FC backward, the BN2-scaled gradient), the PReLU backward of
//     the input layer, the MaxPool2d(1, 2) shortcut adjoint;
//   * FPN bilinear up-sampling (align_corners=True) and its adjoint in gather form (no atomics).
// Every elementwise kernel works on 16-byte vectors of 8 channels (fp16/bf16; 2×16 B for fp32).
#include "conv_common.h"

namespace mia {

static int ew_grid(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (int)std::min<int64_t>(b, 65536);
}

// the per-(image, channel) sum of mia_chan_sum: its nch ordered pixel-chunk partials added in
// chunk order from 0 (the additions of chan_fin_kernel), or the finished sum when nch == 0
__device__ __forceinline__ float chan_total(const float* __restrict__ v, int nch, int n, int C,
                                            int c) {
  if (nch == 0) return v[(size_t)n * C + c];
  const float* p = v + (size_t)n * nch * C + c;
  float s = 0.f;
  int q = 0;
  for (; q + 8 <= nch; q += 8) {  // loads batched ahead of the in-order adds (bit-identical)
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = p[(size_t)(q + u) * C];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += t[u];
  }
  for (; q < nch; ++q) s += p[(size_t)q * C];
  return s;
}

// Σ_{j<Cr} w[j]·x[j] in j order with the (strided) weight loads batched by 8 — the SE FCs' inner
// loops, one L2 round trip per batch instead of per term (bit-identical to the plain loop)
__device__ __forceinline__ float dot_strided(const float* __restrict__ w, size_t stride,
                                             const float* x, int Cr) {
  float a = 0.f;
  int j = 0;
  for (; j + 8 <= Cr; j += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = w[(size_t)(j + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) a = __builtin_fmaf(t[u], x[j + u], a);  // (fused, as the loop's)
  }
  for (; j < Cr; ++j) a += w[(size_t)j * stride] * x[j];
  return a;
}

// Σ over this lane's channels c = lane + 64·u < C (C ≤ 512) of w[c·stride]·x[c], in u order with
// the weight loads issued first (bit-identical to the c += 64 loop)
__device__ __forceinline__ float lane_dot8(const float* __restrict__ w, size_t stride,
                                           const float* x, int lane, int C) {
  float t[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = lane + 64 * u;
    t[u] = c < C ? w[(size_t)c * stride] : 0.f;
  }
  float a = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (lane + 64 * u < C) a = __builtin_fmaf(t[u], x[lane + 64 * u], a);
  return a;
}

// ---- SE forward: u = relu(W1·avg), s = sigmoid(W2·u), one block per image ----------------------
__global__ __launch_bounds__(256) void se_fwd_kernel(const float* __restrict__ csum, int nch,
                                                     const float* __restrict__ w1,
                                                     const float* __restrict__ w2, float* u_out,
                                                     float* s_out, int C, int Cr, float inv_hw) {
  __shared__ float avg[512];
  __shared__ float uu[64];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int c = tid; c < C; c += 256) avg[c] = chan_total(csum, nch, n, C, c) * inv_hw;
  __syncthreads();
  for (int j = wid; j < Cr; j += 4) {
    const float a = wave_sum(lane_dot8(w1 + (size_t)j * C, 1, avg, lane, C));
    if (lane == 0) {
      const float r = a > 0.f ? a : 0.f;
      uu[j] = r;
      u_out[(size_t)n * Cr + j] = r;
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const float z = dot_strided(w2 + (size_t)c * Cr, 1, uu, Cr);
    s_out[(size_t)n * C + c] = 1.f / (1.f + __expf(-z));
  }
}

// ---- SE backward: gz = gs·s(1−s); gu = (W2ᵀ gz)·[u>0]; gavg = inv_hw·W1ᵀ gu -------------------
__global__ __launch_bounds__(256) void se_bwd_kernel(const float* __restrict__ gs, int nch,
                                                     const float* __restrict__ s,
                                                     const float* __restrict__ u,
                                                     const float* __restrict__ w1,
                                                     const float* __restrict__ w2, float* gavg,
                                                     int C, int Cr, float inv_hw) {
  __shared__ float gz[512];
  __shared__ float gu[64];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int c = tid; c < C; c += 256) {
    const float sv = s[(size_t)n * C + c];
    gz[c] = chan_total(gs, nch, n, C, c) * sv * (1.f - sv);
  }
  __syncthreads();
  for (int j = wid; j < Cr; j += 4) {
    const float a = wave_sum(lane_dot8(w2 + j, Cr, gz, lane, C));
    if (lane == 0) gu[j] = u[(size_t)n * Cr + j] > 0.f ? a : 0.f;
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const float a = dot_strided(w1 + c, C, gu, Cr);
    gavg[(size_t)n * C + c] = a * inv_hw;
  }
}

// ---- out = r·s + shortcut; xb = out·g + b (the next unit's BatchNorm) ---------------------------
template <typename T>
__global__ __launch_bounds__(256) void se_apply_kernel(const T* __restrict__ r,
                                                       const float* __restrict__ s,
                                                       const T* __restrict__ sc, int ss,
                                                       T* out, const float* __restrict__ g,
                                                       const float* __restrict__ b, T* xb, int N,
                                                       int H, int W, int C) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t pix = i / cv;  // (n, y, x)
    const int x = (int)(pix % W);
    const int64_t ny = pix / W;
    const int y = (int)(ny % H), n = (int)(ny / H);
    float v[8];
    load8<T>(r + pix * C + c, v);
    if (s) {
      float sv[8];
      load8f(s + (size_t)n * C + c, sv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= sv[e];
    }
    if (sc) {
      float sh[8];
      const int64_t sp = ((int64_t)n * H * ss + (int64_t)y * ss) * (W * ss) + (int64_t)x * ss;
      load8<T>(sc + sp * C + c, sh);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += sh[e];
    }
    if (out) store8<T>(out + pix * C + c, v);
    if (xb) {
      float gg[8], bb[8];
      load8f(g + c, gg);
      load8f(b + c, bb);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] * gg[e] + bb[e];
      store8<T>(xb + pix * C + c, v);
    }
  }
}

// ---- gs[n][c] += Σ_p a·b: block (chunk, n); lanes own 8-channel vectors, LDS reduction; the
// block's partial goes to its slot (chunk) of the library's reduction scratch (red_finish) -------
template <typename T>
__global__ __launch_bounds__(256) void chan_dot_kernel(const T* __restrict__ a,
                                                       const T* __restrict__ b, float* part, int HW,
                                                       int C, int pix_per_chunk) {
  __shared__ float red[256 * 8];
  const int n = blockIdx.y, tid = threadIdx.x;
  const int cv = C / 8;
  const int lanes_per_pix = cv < 256 ? cv : 256;  // C ≤ 2048
  const int pr = 256 / lanes_per_pix;             // pixels in flight per block
  const int vc = tid % lanes_per_pix, pl = tid / lanes_per_pix;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int p0 = blockIdx.x * pix_per_chunk, p1 = min(HW, p0 + pix_per_chunk);
  if (pl < pr) {
    for (int pix = p0 + pl; pix < p1; pix += pr) {
      for (int c8 = vc; c8 < cv; c8 += lanes_per_pix) {
        float va[8], vb[8];
        const size_t off = ((size_t)n * HW + pix) * C + c8 * 8;
        load8<T>(a + off, va);
        load8<T>(b + off, vb);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += va[e] * vb[e];
      }
    }
  }
  // LDS image red[e][thread]: consecutive lanes on consecutive banks for the stores and for the
  // reads below (the [thread][e] image put 8 lanes on one bank: 0.645 bank-conflict ratio, r04)
#pragma unroll
  for (int e = 0; e < 8; ++e) red[e * 256 + tid] = acc[e];
  __syncthreads();
  if (tid < lanes_per_pix) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = 0.f;
      for (int q = 0; q < pr; ++q) s += red[e * 256 + q * lanes_per_pix + tid];
      red_store(part, gridDim.x, gridDim.y * C, 0, blockIdx.x, n * C + tid * 8 + e, s);
    }
  }
}

// ---- deterministic per-(image, channel) sums: Σ_p a·b (DOT) or Σ_p a over the pixels ------------
// chunk q of image n writes its partial to part[(n·nch + q)·C + c] (a fixed-order reduction inside
// the block), then chan_fin adds the nch partials in order: bit-reproducible run to run, unlike
// atomics across blocks (the SE average pool feeds PReLU / ReLU branches downstream).
template <typename T, bool DOT>
__global__ __launch_bounds__(256) void chan_part_kernel(const T* __restrict__ a,
                                                        const T* __restrict__ b,
                                                        float* __restrict__ part, int HW, int C,
                                                        int pix_per_chunk) {
  __shared__ float red[256 * 8];
  const int n = blockIdx.y, tid = threadIdx.x;
  const int cv = C / 8;
  const int lanes_per_pix = cv < 256 ? cv : 256;
  const int pr = 256 / lanes_per_pix;
  const int vc = tid % lanes_per_pix, pl = tid / lanes_per_pix;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const int p0 = blockIdx.x * pix_per_chunk, p1 = min(HW, p0 + pix_per_chunk);
  if (pl < pr) {
    for (int pix = p0 + pl; pix < p1; pix += pr) {
      for (int c8 = vc; c8 < cv; c8 += lanes_per_pix) {
        float va[8], vb[8];
        const size_t off = ((size_t)n * HW + pix) * C + c8 * 8;
        load8<T>(a + off, va);
        if constexpr (DOT) {
          load8<T>(b + off, vb);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += va[e] * vb[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += va[e];
        }
      }
    }
  }
  // (C > 2048 is rejected: every channel chunk c8 < cv maps to one lane, lanes_per_pix = cv)
#pragma unroll
  for (int e = 0; e < 8; ++e) red[e * 256 + tid] = acc[e];  // conflict-free image (chan_dot)
  __syncthreads();
  if (tid < lanes_per_pix) {
    float* dst = part + ((size_t)n * gridDim.x + blockIdx.x) * C + tid * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = 0.f;
      for (int q = 0; q < pr; ++q) s += red[e * 256 + q * lanes_per_pix + tid];
      dst[e] = s;
    }
  }
}

__global__ __launch_bounds__(256) void chan_fin_kernel(const float* __restrict__ part,
                                                       float* out, int N, int C, int nch,
                                                       int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - (i / C) * C;
  float s = accumulate ? out[i] : 0.f;
  for (int q = 0; q < nch; ++q) s += part[((size_t)n * nch + q) * C + c];
  out[i] = s;
}

// ---- g_r = gamma·(g_out·s + gavg) ----------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void se_grad_scale_kernel(const T* __restrict__ go,
                                                            const float* __restrict__ s,
                                                            const float* __restrict__ gavg,
                                                            const float* __restrict__ gamma,
                                                            T* gr, int HW, int C, int64_t total) {
  const int cv = C / 8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t pix = i / cv;
    const int n = (int)(pix / HW);
    float v[8], sv[8], ga[8], gm[8];
    load8<T>(go + pix * C + c, v);
    load8f(s + (size_t)n * C + c, sv);
    load8f(gavg + (size_t)n * C + c, ga);
    if (gamma) {
      load8f(gamma + c, gm);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) gm[e] = 1.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = gm[e] * (v[e] * sv[e] + ga[e]);
    store8<T>(gr + pix * C + c, v);
  }
}

// ---- g = g_a·(a > 0 ? 1 : slope)·gamma -----------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void prelu_bwd_scale_kernel(const T* __restrict__ ga,
                                                              const T* __restrict__ act,
                                                              const float* __restrict__ slope,
                                                              const float* __restrict__ gamma,
                                                              T* g, int C, int64_t total) {
  const int cv = C / 8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t pix = i / cv;
    float v[8], av[8], sl[8], gm[8];
    load8<T>(ga + pix * C + c, v);
    load8<T>(act + pix * C + c, av);
    load8f(slope + c, sl);
    if (gamma) {
      load8f(gamma + c, gm);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) gm[e] = 1.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (av[e] > 0.f ? v[e] : sl[e] * v[e]) * gm[e];
    store8<T>(g + pix * C + c, v);
  }
}

// ---- a = pre > 0 ? pre : slope·pre (PReLU forward from a stored pre-activation) -------------------
// Round 6: the e4e units whose PReLU has a negative slope keep the conv output (pre) for the
// backward's branch mask — the stored activation's sign no longer tells the branch — and take
// their activation from this pass (same single rounding of slope·pre as the conv epilogue's
// MIA_ACT_PRELU at fp32).
template <typename T>
__global__ __launch_bounds__(256) void prelu_fwd_kernel(const T* __restrict__ pre,
                                                        const float* __restrict__ slope,
                                                        T* __restrict__ a, int C, int64_t total) {
  const int cv = C / 8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t pix = i / cv;
    float v[8], sl[8];
    load8<T>(pre + pix * C + c, v);
    load8f(slope + c, sl);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : sl[e] * v[e];
    store8<T>(a + pix * C + c, v);
  }
}

// ---- gx[n][2y][2x] += g[n][y][x] -----------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void subsample_add_kernel(const T* __restrict__ g, T* gx, int N,
                                                            int H, int W, int C) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t pix = i / cv;
    const int x = (int)(pix % W);
    const int64_t ny = pix / W;
    const int y = (int)(ny % H), n = (int)(ny / H);
    const int64_t dp = ((int64_t)n * 2 * H + 2 * y) * (2 * W) + 2 * x;
    float v[8], o[8];
    load8<T>(g + pix * C + c, v);
    load8<T>(gx + dp * C + c, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += v[e];
    store8<T>(gx + dp * C + c, o);
  }
}

// ---- bilinear, align_corners=True (ATen upsample_bilinear2d: scale = (in−1)/(out−1) in fp32,
// src = scale·dst, i0 = (int)src, i1 = i0 + (i0 < in−1), λ1 = src − i0) ---------------------------
__device__ __forceinline__ void bl_coord(int o, float scale, int in, int& i0, int& i1, float& l1) {
  const float src = scale * (float)o;
  i0 = (int)src;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

template <typename T>
__global__ __launch_bounds__(256) void bilinear_fwd_kernel(const T* __restrict__ x, T* y, int N,
                                                           int Hi, int Wi, int Ho, int Wo, int C,
                                                           float sh, float sw, int accumulate) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * Ho * Wo * cv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t pix = i / cv;
    const int xo = (int)(pix % Wo);
    const int64_t ny = pix / Wo;
    const int yo = (int)(ny % Ho), n = (int)(ny / Ho);
    int y0, y1, x0, x1;
    float ly, lx;
    bl_coord(yo, sh, Hi, y0, y1, ly);
    bl_coord(xo, sw, Wi, x0, x1, lx);
    const T* base = x + (size_t)n * Hi * Wi * C + c;
    float a[8], b[8], d[8], e4[8], v[8];
    load8<T>(base + ((size_t)y0 * Wi + x0) * C, a);
    load8<T>(base + ((size_t)y0 * Wi + x1) * C, b);
    load8<T>(base + ((size_t)y1 * Wi + x0) * C, d);
    load8<T>(base + ((size_t)y1 * Wi + x1) * C, e4);
    const float hy = 1.f - ly, hx = 1.f - lx;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = hy * (hx * a[e] + lx * b[e]) + ly * (hx * d[e] + lx * e4[e]);
    if (accumulate) {
      float o[8];
      load8<T>(y + pix * C + c, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += o[e];
    }
    store8<T>(y + pix * C + c, v);
  }
}

// adjoint: input pixel (yi, xi) gathers every output whose i0 or i1 is yi (resp. xi); the output
// rows that can touch yi lie within ±(1/scale + 2) of yi/scale
template <typename T>
__global__ __launch_bounds__(256) void bilinear_bwd_kernel(const T* __restrict__ gy, T* gx, int N,
                                                           int Hi, int Wi, int Ho, int Wo, int C,
                                                           float sh, float sw, int accumulate) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * Hi * Wi * cv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % cv) * 8;
    const int64_t pix = i / cv;
    const int xi = (int)(pix % Wi);
    const int64_t ny = pix / Wi;
    const int yi = (int)(ny % Hi), n = (int)(ny / Hi);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const int ry = sh > 0.f ? (int)(1.f / sh) + 2 : Ho, rx = sw > 0.f ? (int)(1.f / sw) + 2 : Wo;
    const int cy = sh > 0.f ? (int)((float)yi / sh) : 0, cx = sw > 0.f ? (int)((float)xi / sw) : 0;
    const int ya = max(0, cy - ry), yb = min(Ho - 1, cy + ry);
    const int xa = max(0, cx - rx), xb = min(Wo - 1, cx + rx);
    for (int yo = ya; yo <= yb; ++yo) {
      int y0, y1;
      float ly;
      bl_coord(yo, sh, Hi, y0, y1, ly);
      float wy = 0.f;
      if (y0 == yi) wy += 1.f - ly;
      if (y1 == yi) wy += ly;
      if (wy == 0.f) continue;
      for (int xo = xa; xo <= xb; ++xo) {
        int x0, x1;
        float lx;
        bl_coord(xo, sw, Wi, x0, x1, lx);
        float wx = 0.f;
        if (x0 == xi) wx += 1.f - lx;
        if (x1 == xi) wx += lx;
        if (wx == 0.f) continue;
        float g[8];
        load8<T>(gy + (((size_t)n * Ho + yo) * Wo + xo) * C + c, g);
        const float w = wy * wx;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += w * g[e];
      }
    }
    if (accumulate) {
      float o[8];
      load8<T>(gx + pix * C + c, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += o[e];
    }
    store8<T>(gx + pix * C + c, acc);
  }
}

// ---- y = scale·x with a dtype conversion (latent features fp32 ↔ feature-map dtype) --------------
template <typename S, typename D>
__global__ __launch_bounds__(256) void cast_kernel(const S* __restrict__ x, D* y, int64_t n,
                                                   float scale) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[i] = from_f<D>(to_f(x[i]) * scale);
}

static float bl_scale(int in, int out) {
  return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
}

}  // namespace mia

using namespace mia;

#define ENC_CHECK_C(C) MIA_CHECK_ARG((C) > 0 && (C) % 8 == 0, "C must be a positive multiple of 8")

extern "C" int mia_se_fwd(const float* csum, const float* w1, const float* w2, float* u, float* s,
                          int N, int C, int Cr, float inv_hw, void* stream) {
  return mia_se_fwd_parts(csum, 0, w1, w2, u, s, N, C, Cr, inv_hw, stream);
}

extern "C" int mia_se_fwd_parts(const float* part, int nch, const float* w1, const float* w2,
                                float* u, float* s, int N, int C, int Cr, float inv_hw,
                                void* stream) {
  MIA_CHECK_ARG(part && w1 && w2 && u && s && N > 0 && nch >= 0, "bad args");
  MIA_CHECK_ARG(C > 0 && C <= 512 && Cr > 0 && Cr <= 64, "C ≤ 512, C/r ≤ 64");
  hipLaunchKernelGGL(se_fwd_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, part, nch, w1, w2,
                     u, s, C, Cr, inv_hw);
  return check_launch("se_fwd");
}

extern "C" int mia_se_bwd(const float* gs, const float* s, const float* u, const float* w1,
                          const float* w2, float* gavg, int N, int C, int Cr, float inv_hw,
                          void* stream) {
  return mia_se_bwd_parts(gs, 0, s, u, w1, w2, gavg, N, C, Cr, inv_hw, stream);
}

extern "C" int mia_se_bwd_parts(const float* part, int nch, const float* s, const float* u,
                                const float* w1, const float* w2, float* gavg, int N, int C,
                                int Cr, float inv_hw, void* stream) {
  MIA_CHECK_ARG(part && s && u && w1 && w2 && gavg && N > 0 && nch >= 0, "bad args");
  MIA_CHECK_ARG(C > 0 && C <= 512 && Cr > 0 && Cr <= 64, "C ≤ 512, C/r ≤ 64");
  hipLaunchKernelGGL(se_bwd_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, part, nch, s, u, w1,
                     w2, gavg, C, Cr, inv_hw);
  return check_launch("se_bwd");
}

extern "C" int mia_se_apply(const void* r, const float* s, const void* sc, int ss, void* out,
                            const float* g, const float* b, void* xb, int N, int H, int W, int C,
                            int dtype, void* stream) {
  MIA_CHECK_ARG(r && (out || xb) && N > 0 && H > 0 && W > 0, "bad args");
  MIA_CHECK_ARG(ss == 1 || ss == 2, "shortcut stride 1 or 2");
  MIA_CHECK_ARG(!xb || (g && b), "xb needs g and b");
  ENC_CHECK_C(C);
  const int grid = ew_grid((int64_t)N * H * W * (C / 8));
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(se_apply_kernel<T>, dim3(grid), dim3(256), 0,
                                                  (hipStream_t)stream, (const T*)r, s,
                                                  (const T*)sc, ss, (T*)out, g, b, (T*)xb, N, H,
                                                  W, C));
  return check_launch("se_apply");
}

// pixel chunks per image: a function of HW only, so an image's sums are the same fp32 additions
// whatever the batch (batch-1 and batch-N runs agree bit for bit)
static int chan_chunks(int N, int HW) {
  (void)N;
  return std::max(1, std::min(HW / 16, 32));
}

extern "C" int mia_chan_dot(const void* a, const void* b, float* gs, int N, int HW, int C,
                            int accumulate, int dtype, void* stream) {
  MIA_CHECK_ARG(a && b && gs && N > 0 && HW > 0, "bad args");
  ENC_CHECK_C(C);
  MIA_CHECK_ARG(C <= 2048, "C ≤ 2048");
  hipStream_t st = (hipStream_t)stream;
  if (!accumulate && hipMemsetAsync(gs, 0, (size_t)N * C * sizeof(float), st) != hipSuccess)
    return set_error("chan_dot: memset failed");
  const int chunks = chan_chunks(N, HW);
  const int ppc = (HW + chunks - 1) / chunks;
  const int nch = (HW + ppc - 1) / ppc;
  RedQ r;
  int rc = red_begin(r, gs, nullptr, nullptr, nch, N * C, st);
  if (rc != MIA_OK) return rc;
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(chan_dot_kernel<T>, dim3(nch, N), dim3(256), 0,
                                                  st, (const T*)a, (const T*)b, r.part, HW, C,
                                                  ppc));
  rc = check_launch("chan_dot");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

extern "C" int mia_chan_sum_parts(int N, int HW) {
  const int chunks = chan_chunks(N, HW);
  const int ppc = (HW + chunks - 1) / chunks;
  return (HW + ppc - 1) / ppc;
}

extern "C" int mia_chan_sum(const void* a, const void* b, float* part, float* out, int N, int HW,
                            int C, int accumulate, int dtype, void* stream) {
  MIA_CHECK_ARG(a && part && N > 0 && HW > 0, "bad args");
  MIA_CHECK_ARG(out || !accumulate, "accumulate needs out");
  ENC_CHECK_C(C);
  MIA_CHECK_ARG(C <= 2048, "C ≤ 2048");
  hipStream_t st = (hipStream_t)stream;
  const int chunks = chan_chunks(N, HW);
  const int ppc = (HW + chunks - 1) / chunks;
  const int nch = (HW + ppc - 1) / ppc;
  MIA_DISPATCH_DTYPE(dtype, T, {
    if (b)
      hipLaunchKernelGGL((chan_part_kernel<T, true>), dim3(nch, N), dim3(256), 0, st,
                         (const T*)a, (const T*)b, part, HW, C, ppc);
    else
      hipLaunchKernelGGL((chan_part_kernel<T, false>), dim3(nch, N), dim3(256), 0, st,
                         (const T*)a, (const T*)nullptr, part, HW, C, ppc);
  });
  const int rc = check_launch("chan_part");
  if (rc || !out) return rc;  // out NULL: the partials only (mia_se_fwd_parts / mia_se_bwd_parts)
  hipLaunchKernelGGL(chan_fin_kernel, dim3((N * C + 255) / 256), dim3(256), 0, st, part, out, N, C,
                     nch, accumulate);
  return check_launch("chan_fin");
}

extern "C" int mia_se_grad_scale(const void* g_out, const float* s, const float* gavg,
                                 const float* gamma, void* g_r, int N, int HW, int C, int dtype,
                                 void* stream) {
  MIA_CHECK_ARG(g_out && s && gavg && g_r && N > 0 && HW > 0, "bad args");
  ENC_CHECK_C(C);
  const int64_t total = (int64_t)N * HW * (C / 8);
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(se_grad_scale_kernel<T>, dim3(ew_grid(total)),
                                                  dim3(256), 0, (hipStream_t)stream,
                                                  (const T*)g_out, s, gavg, gamma, (T*)g_r, HW, C,
                                                  total));
  return check_launch("se_grad_scale");
}

extern "C" int mia_prelu_bwd_scale(const void* g_a, const void* a, const float* slope,
                                   const float* gamma, void* g, int64_t pixels, int C, int dtype,
                                   void* stream) {
  MIA_CHECK_ARG(g_a && a && slope && g && pixels > 0, "bad args");
  ENC_CHECK_C(C);
  const int64_t total = pixels * (C / 8);
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(prelu_bwd_scale_kernel<T>,
                                                  dim3(ew_grid(total)), dim3(256), 0,
                                                  (hipStream_t)stream, (const T*)g_a, (const T*)a,
                                                  slope, gamma, (T*)g, C, total));
  return check_launch("prelu_bwd_scale");
}

extern "C" int mia_prelu_fwd(const void* pre, const float* slope, void* a, int64_t pixels, int C,
                             int dtype, void* stream) {
  MIA_CHECK_ARG(pre && slope && a && pixels > 0, "bad args");
  ENC_CHECK_C(C);
  const int64_t total = pixels * (C / 8);
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(prelu_fwd_kernel<T>, dim3(ew_grid(total)),
                                                  dim3(256), 0, (hipStream_t)stream,
                                                  (const T*)pre, slope, (T*)a, C, total));
  return check_launch("prelu_fwd");
}

extern "C" int mia_subsample_add(const void* g, void* gx, int N, int H, int W, int C, int dtype,
                                 void* stream) {
  MIA_CHECK_ARG(g && gx && N > 0 && H > 0 && W > 0, "bad args");
  ENC_CHECK_C(C);
  const int grid = ew_grid((int64_t)N * H * W * (C / 8));
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(subsample_add_kernel<T>, dim3(grid), dim3(256),
                                                  0, (hipStream_t)stream, (const T*)g, (T*)gx, N,
                                                  H, W, C));
  return check_launch("subsample_add");
}

extern "C" int mia_bilinear_fwd(const void* x, void* y, int N, int Hi, int Wi, int Ho, int Wo,
                                int C, int accumulate, int dtype, void* stream) {
  MIA_CHECK_ARG(x && y && N > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "bad args");
  ENC_CHECK_C(C);
  const int grid = ew_grid((int64_t)N * Ho * Wo * (C / 8));
  const float sh = bl_scale(Hi, Ho), sw = bl_scale(Wi, Wo);
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(bilinear_fwd_kernel<T>, dim3(grid), dim3(256),
                                                  0, (hipStream_t)stream, (const T*)x, (T*)y, N,
                                                  Hi, Wi, Ho, Wo, C, sh, sw, accumulate));
  return check_launch("bilinear_fwd");
}

extern "C" int mia_bilinear_bwd(const void* gy, void* gx, int N, int Hi, int Wi, int Ho, int Wo,
                                int C, int accumulate, int dtype, void* stream) {
  MIA_CHECK_ARG(gy && gx && N > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "bad args");
  MIA_CHECK_ARG(Ho >= Hi && Wo >= Wi, "up-sampling only (the FPN case)");
  ENC_CHECK_C(C);
  const int grid = ew_grid((int64_t)N * Hi * Wi * (C / 8));
  const float sh = bl_scale(Hi, Ho), sw = bl_scale(Wi, Wo);
  MIA_DISPATCH_DTYPE(dtype, T, hipLaunchKernelGGL(bilinear_bwd_kernel<T>, dim3(grid), dim3(256),
                                                  0, (hipStream_t)stream, (const T*)gy, (T*)gx, N,
                                                  Hi, Wi, Ho, Wo, C, sh, sw, accumulate));
  return check_launch("bilinear_bwd");
}

extern "C" int mia_cast(const void* x, int xdtype, void* y, int ydtype, int64_t n, float scale,
                        void* stream) {
  MIA_CHECK_ARG(x && y && n > 0, "bad args");
  const int grid = ew_grid(n);
  hipStream_t st = (hipStream_t)stream;
  MIA_DISPATCH_DTYPE(xdtype, S, {
    MIA_DISPATCH_DTYPE(ydtype, D, hipLaunchKernelGGL((cast_kernel<S, D>), dim3(grid), dim3(256),
                                                     0, st, (const S*)x, (D*)y, n, scale));
  });
  return check_launch("cast");
}
