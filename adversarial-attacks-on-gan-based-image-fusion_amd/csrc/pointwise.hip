// HBM-bound kernels of the attack step (gfx950): bias/act, StyledConv backward front, ToRGB,
// upfirdn2d, max/avg pooling, MSE pieces, image layout changes and the PGD sign-project step.
// Feature maps are NHWC and moved in 16-byte vectors (4 fp32 / 8 fp16|bf16 per lane).
#include "mia_common.h"

namespace mia {

constexpr int TPB = 256;

static inline int blocks_for(int64_t n, int per_block = TPB, int cap = 1 << 20) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return (int)(b > cap ? cap : b);
}

// ---------------------------------------------------------------------------------------------
// K4 forward, standalone: y = lrelu(x + nw·noise[p] + b[c])·√2 (rosinality FusedLeakyReLU after
// NoiseInjection). The fused path writes `pre` from the conv epilogue instead.
template <typename T>
__global__ void bias_act_fwd_kernel(const T* __restrict__ x, const float* __restrict__ noise,
                                    float nw, const float* __restrict__ bias, T* __restrict__ y,
                                    int64_t nvec, int C, int HW) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * TPB) {
    const int64_t e0 = i * V;
    const int c0 = (int)(e0 % C);
    const int p = (int)((e0 / C) % HW);
    VT v = ((const VT*)x)[i];
    const float nz = noise ? nw * noise[p] : 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = from_f<T>(lrelu_s2(to_f(v[e]) + nz + (bias ? bias[c0 + e] : 0.f)));
    ((VT*)y)[i] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// StyledConv backward front. One block = a run of pixels of one image, all channels.
template <typename T>
__global__ void bias_act_bwd_kernel(const T* __restrict__ g_a, const T* __restrict__ pre,
                                    const float* __restrict__ noise, float nw,
                                    const float* __restrict__ bias, const float* __restrict__ demod,
                                    T* __restrict__ gy, float* __restrict__ qpart, int H, int W,
                                    int C, int unshuffle, int from_act, int pix_per_block) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  __shared__ float red[TPB * 8];
  const int n = blockIdx.y;
  const int HW = H * W;
  const int tpp = C / V;             // threads per pixel (≤ 256)
  const int ppp = TPB / tpp;         // pixels per pass
  const int t = threadIdx.x;
  const int chunk = t % tpp, sub = t / tpp;
  const int c0 = chunk * V;
  float qa[V];
#pragma unroll
  for (int e = 0; e < V; ++e) qa[e] = 0.f;
  float dm[V], bs[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    dm[e] = demod[(size_t)n * C + c0 + e];
    bs[e] = bias ? bias[c0 + e] : 0.f;
  }
  const int p_begin = blockIdx.x * pix_per_block;
  const int p_end = min(p_begin + pix_per_block, HW);
  if (sub < ppp) {
    for (int p = p_begin + sub; p < p_end; p += ppp) {
      const size_t off = ((size_t)n * HW + p) * C + c0;
      const VT ga = *(const VT*)(g_a + off);
      const VT pr = *(const VT*)(pre + off);
      const float nz = noise ? nw * noise[p] : 0.f;
      VT o;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float pin = to_f(pr[e]);
        const float gr = lrelu_s2_grad(pin);  // same sign for pre and act = lrelu(pre)·√2
        const float pv = from_act ? pin / gr : pin;
        const float gp = to_f(ga[e]) * gr;
        qa[e] += gp * (pv - nz - bs[e]);
        o[e] = from_f<T>(gp * dm[e]);
      }
      size_t ooff = off;
      if (unshuffle) {
        const int y = p / W, x = p - (p / W) * W;
        const int R = H / 2, Rw = W / 2;
        const int ph = ((y & 1) << 1) | (x & 1);
        ooff = (((size_t)n * R + (y >> 1)) * Rw + (x >> 1)) * (4 * C) + ph * C + c0;
      }
      *(VT*)(gy + ooff) = o;
    }
  }
  // reduce q over the `ppp` pixel lanes sharing a channel chunk
#pragma unroll
  for (int e = 0; e < V; ++e) red[t * V + e] = qa[e];
  __syncthreads();
  if (sub == 0) {
    for (int s = 1; s < ppp; ++s)
#pragma unroll
      for (int e = 0; e < V; ++e) qa[e] += red[(s * tpp + chunk) * V + e];
    // the block's partial into its slot (blockIdx.x); red_finish adds the slots in order
#pragma unroll
    for (int e = 0; e < V; ++e)
      red_store(qpart, gridDim.x, gridDim.y * C, 0, blockIdx.x, n * C + c0 + e, qa[e]);
  }
}

// ---------------------------------------------------------------------------------------------
// Blur of the up-sampling StyledConv (rosinality Blur: upfirdn2d, k = [1,3,3,1]⊗[1,3,3,1]/64·4,
// pad (1,1)) applied to the transposed-conv output T (N, 2R+1, 2R+1, C), fused with the
// demodulation scale, noise injection and bias: pre = demod·blur(T) + nw·noise + b.
__constant__ float kBlur4[4] = {0.25f, 0.75f, 0.75f, 0.25f};

// Both directions are the same separable 4-tap FIR (factor-2 up-sampling phases). A thread owns a
// 2-wide × 2·KQ-tall output strip of one 8-channel (16-byte) vector and streams down the 2·KQ+3
// input rows it needs: each row is loaded once (5 vectors), filtered horizontally into the strip's
// 2 columns, and accumulated into the ≤ 4 output rows it feeds; an output row is stored as soon as
// its 4th input row has been added (≈ 3.4 loads per output instead of 16 for a direct 4×4 FIR).
//   forward : out = pre (N,2R,2R,C),    in = T  (N,2R+1,2R+1,C), input row of output row 0 is −1
//   backward: out = gT (N,2R+1,2R+1,C), in = gy (N,2R,2R,C),     input row of output row 0 is −2
// (the adjoint flips the taps; the kernel is symmetric so the weights are the same).
// input rows in flight per thread: 4 (round 6; 2 before: fp32 forward / adjoint −1.5 / −3.9 %,
// fp16 −2.9 / −2.5 % per generator pass, still 2 waves per SIMD; profiles/r06_blur_pf_ab.txt)
#ifndef MIA_BLUR_PF
#define MIA_BLUR_PF 4
#endif
#ifndef MIA_BLUR_KQ  // output rows per strip / 2 (swept 2 … 6: profiles/r06_blur_kq_sweep.txt)
#define MIA_BLUR_KQ 4
#endif
constexpr int kBlurKQ = MIA_BLUR_KQ;
static __device__ __attribute__((aligned(16))) uint4 g_blur_zero[1];  // zero page (out-of-range taps)


// V consecutive fp32 values (V = 8 or 4) with 16-byte loads
template <int V>
__device__ __forceinline__ void load8f_or_4(const float* p, float (&v)[V]) {
#pragma unroll
  for (int q = 0; q < V / 4; ++q) {
    const f32x4 t = *(const f32x4*)(p + 4 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * q + e] = t[e];
  }
}

template <typename T, bool FWD, bool NOISE>
__global__ __launch_bounds__(256) void blur4_strip_kernel(
    const T* __restrict__ in, T* __restrict__ out, const float* __restrict__ demod,
    const float* __restrict__ noise, float nw, const float* __restrict__ bias, int N, int R, int C,
    int act_out) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  constexpr int KQ = kBlurKQ, OR = 2 * KQ, IR = 2 * KQ + 3;
  const int Hin = FWD ? 2 * R + 1 : 2 * R;
  const int Hout = FWD ? 2 * R : 2 * R + 1;
  const int Q = (Hout + 1) / 2;     // 2-wide columns per row
  const int SY = (Hout + OR - 1) / OR;  // strips per column
  const int off0 = FWD ? -1 : -2;
  const int nc = C / V;
  const int64_t total = (int64_t)N * SY * Q * nc;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    int cv, qx, sy, n;
    if (total < (1LL << 31)) {  // 32-bit divisions: a third of the 64-bit ones' VALU
      unsigned u = (unsigned)i;
      cv = (int)(u % (unsigned)nc);
      u /= (unsigned)nc;
      qx = (int)(u % (unsigned)Q);
      u /= (unsigned)Q;
      sy = (int)(u % (unsigned)SY);
      n = (int)(u / (unsigned)SY);
    } else {
      cv = (int)(i % nc);
      const int64_t r1 = i / nc;
      qx = (int)(r1 % Q);
      const int64_t r2 = r1 / Q;
      sy = (int)(r2 % SY);
      n = (int)(r2 / SY);
    }
    const int x0 = 2 * qx + off0, y0 = sy * OR + off0;
    const int oy0 = sy * OR, ox0 = 2 * qx;
    float dm[V], bs[V];
    if (FWD) {
      load8f_or_4(demod + (size_t)n * C + cv * V, dm);
      if (bias) {
        load8f_or_4(bias + cv * V, bs);
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) bs[e] = 0.f;
      }
    }
    const T* base = in + (size_t)n * Hin * Hin * C + cv * V;
    T* obase = out + (size_t)n * Hout * Hout * C + cv * V;
    // noise of the whole strip up front: a global load issued between the pipelined row loads
    // would force a vmcnt(0) drain (the counter retires in order)
    // (NOISE is a template flag so that no branch separates these loads from the row loads)
    float nzs[OR][2];
#pragma unroll
    for (int a = 0; a < OR; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        nzs[a][b] = NOISE ? noise[min(oy0 + a, Hout - 1) * Hout + min(ox0 + b, Hout - 1)] : 0.f;
    float acc[OR][2][V];
    // software pipeline: rows rl+1 … rl+PF are in flight while row rl is filtered. Loads are
    // unconditional: an out-of-range tap reads the zero page (round 6: the address is selected,
    // not the loaded values zeroed; with 32-bit index math −1 … −4 %, profiles/r06_blur_v2_ab.txt).
    int xc[5];
    bool xv[5];
#pragma unroll
    for (int lc = 0; lc < 5; ++lc) {
      const int xx = x0 + lc;
      xv[lc] = xx >= 0 && xx < Hin;
      xc[lc] = min(max(xx, 0), Hin - 1);
    }
    constexpr int PF = MIA_BLUR_PF;  // input rows in flight ahead of the one being filtered
    VT nx[PF][5];
    // out-of-range taps load the zero page (the address is selected, not the 8 loaded values)
    auto src = [&](int yy, int lc) {
      const bool ok = yy >= 0 && yy < Hin && xv[lc];
      return ok ? base + ((size_t)yy * Hin + xc[lc]) * C : (const T*)g_blur_zero;
    };
#pragma unroll
    for (int q = 0; q < PF; ++q)
#pragma unroll
      for (int lc = 0; lc < 5; ++lc) nx[q][lc] = *(const VT*)src(y0 + q, lc);
#pragma unroll
    for (int rl = 0; rl < IR; ++rl) {
      const int yy = y0 + rl;
      VT v[5];
#pragma unroll
      for (int lc = 0; lc < 5; ++lc) {
        v[lc] = nx[0][lc];
#pragma unroll
        for (int q = 0; q + 1 < PF; ++q) nx[q][lc] = nx[q + 1][lc];
      }
      if (rl + PF < IR) {
#pragma unroll
        for (int lc = 0; lc < 5; ++lc) nx[PF - 1][lc] = *(const VT*)src(yy + PF, lc);
      }
      float h[2][V];
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < V; ++e)
          h[b][e] = kBlur4[0] * to_f(v[b][e]) + kBlur4[1] * to_f(v[b + 1][e]) +
                    kBlur4[2] * to_f(v[b + 2][e]) + kBlur4[3] * to_f(v[b + 3][e]);
#pragma unroll
      for (int a = 0; a < OR; ++a) {
        const int j = rl - a;
        if (j < 0 || j > 3) continue;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < V; ++e)
            acc[a][b][e] = (j == 0 ? 0.f : acc[a][b][e]) + kBlur4[j] * h[b][e];
        if (j != 3) continue;
        // output row a is complete
        const int oy = oy0 + a;
        if (oy >= Hout) continue;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int ox = ox0 + b;
          if (ox >= Hout) continue;
          VT o;
          const float nz = nw * nzs[a][b];
#pragma unroll
          for (int e = 0; e < V; ++e) {
            float r = acc[a][b][e];
            if (FWD) {
              r = r * dm[e] + nz + bs[e];
              if (act_out) r = lrelu_s2(r);
            }
            o[e] = from_f<T>(r);
          }
          *(VT*)(obase + ((size_t)oy * Hout + ox) * C) = o;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// upfirdn2d on fp32 NCHW planes with a separable kernel (rosinality op/upfirdn2d semantics).
__device__ __forceinline__ float upfir_at(const float* __restrict__ x, int H, int W, int oy, int ox,
                                          const float* kf, int kt, int up, int down, int pad0) {
  float acc = 0.f;
  for (int jy = 0; jy < kt; ++jy) {
    const int ty = oy * down + jy - pad0;
    if (ty < 0 || ty % up) continue;
    const int iy = ty / up;
    if (iy >= H) continue;
    for (int jx = 0; jx < kt; ++jx) {
      const int tx = ox * down + jx - pad0;
      if (tx < 0 || tx % up) continue;
      const int ix = tx / up;
      if (ix >= W) continue;
      acc += x[iy * W + ix] * kf[jy] * kf[jx];
    }
  }
  return acc;
}

struct Taps8 { float k[8]; };

__global__ void upfirdn2d_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int planes,
                                     int H, int W, int Ho, int Wo, Taps8 kf, int kt, int up,
                                     int down, int pad0) {
  const int64_t total = (int64_t)planes * Ho * Wo;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int ox = (int)(i % Wo);
    const int oy = (int)((i / Wo) % Ho);
    const int64_t pl = i / ((int64_t)Wo * Ho);
    y[i] = upfir_at(x + pl * H * W, H, W, oy, ox, kf.k, kt, up, down, pad0);
  }
}

__global__ void upfirdn2d_bwd_kernel(const float* __restrict__ gy, float* __restrict__ gx,
                                     int planes, int H, int W, int Ho, int Wo, Taps8 kf, int kt,
                                     int up, int down, int pad0) {
  const int64_t total = (int64_t)planes * H * W;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int ix = (int)(i % W);
    const int iy = (int)((i / W) % H);
    const int64_t pl = i / ((int64_t)W * H);
    const float* g = gy + pl * Ho * Wo;
    float acc = 0.f;
    for (int jy = 0; jy < kt; ++jy) {
      const int sy = iy * up + pad0 - jy;  // = oy*down
      if (sy < 0 || sy % down) continue;
      const int oy = sy / down;
      if (oy >= Ho) continue;
      for (int jx = 0; jx < kt; ++jx) {
        const int sx = ix * up + pad0 - jx;
        if (sx < 0 || sx % down) continue;
        const int ox = sx / down;
        if (ox >= Wo) continue;
        acc += g[oy * Wo + ox] * kf.k[jy] * kf.k[jx];
      }
    }
    gx[i] = acc;
  }
}

// ---------------------------------------------------------------------------------------------
// ToRGB (1x1 modulated conv without demod) + bias + up-sampled skip. A group of `tpp` lanes owns a
// pixel (each lane a slice of channels); the 3 partial dot products are reduced by shuffles.
__constant__ float kUp4[4] = {0.25f, 0.75f, 0.75f, 0.25f};  // [1,3,3,1]/sum · 2 (per axis)

// The ToRGB skip term upfirdn2d(skip, [1,3,3,1]⊗[1,3,3,1]/16·4, up = 2, pad = (2, 1)) at output
// (y, x): the two taps per axis that land on input samples, added in upfir_at's order with its
// expression (bit-identical), loaded unconditionally from clamped addresses (out-of-range taps
// zeroed) so that the four loads issue back-to-back.
__device__ __forceinline__ float skip_up2(const float* __restrict__ sk, int Hs, int Ws, int y,
                                          int x) {
  const int py = y & 1, px = x & 1;
  const int iy0 = (y - 2 + py) >> 1, ix0 = (x - 2 + px) >> 1;
  float v[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int iy = iy0 + a, ix = ix0 + b;
      const bool ok = iy >= 0 && iy < Hs && ix >= 0 && ix < Ws;
      const float t = sk[min(max(iy, 0), Hs - 1) * Ws + min(max(ix, 0), Ws - 1)];
      v[a][b] = ok ? t : 0.f;
    }
  float acc = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc += v[a][b] * kUp4[py + 2 * a] * kUp4[px + 2 * b];
  return acc;
}

template <typename T, int LV>
__global__ __launch_bounds__(TPB) void torgb_fwd_kernel(const T* __restrict__ pre, const float* __restrict__ s,
                                 const float* __restrict__ wr, const float* __restrict__ bias,
                                 const float* __restrict__ skip, float* __restrict__ rgb, int H,
                                 int W, int Cin, int tpp, int cpt, int pix_per_block, int act_in) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  constexpr int U = 4;  // pixels in flight per lane group (U independent 16-B loads per lane)
  extern __shared__ float wm[];  // [3][Cin]
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < 3 * Cin; i += TPB) wm[i] = wr[i] * s[(size_t)n * Cin + (i % Cin)];
  __syncthreads();
  const int HW = H * W, Hs = H / 2, Ws = W / 2;
  const int t = threadIdx.x;
  const int g = t % tpp, sub = t / tpp, ppp = TPB / tpp;
  const int p_begin = blockIdx.x * pix_per_block;
  const int p_end = min(p_begin + pix_per_block, HW);
  const T* img = pre + (size_t)n * HW * Cin;
  // The 12 sums (pixel u, channel c) of a lane group sit in 16 slots k = 4u + c (c = 3 empty) and
  // are reduce-scattered over the group's lanes: at level o (o = 1, 2, 4, 8 while o < tpp) a lane
  // keeps the half of its slots picked by lane bit o and adds the partner's copy of that half —
  // 8 + 4 + 2 + 1 shuffles instead of a butterfly's 12 per level; levels o ≥ 16 add the one slot
  // left. Each addition pairs the same lanes in the same level order as a butterfly (own +
  // partner), so every sum is bit-identical to it. LV = min(4, log2 tpp) scatter levels (a
  // template parameter: levels skipped at run time would keep both versions of the slots live).
  // This lane ends with slots base … base + nsl − 1.
  constexpr int nsl = 16 >> LV;
  int base = 0;
#pragma unroll
  for (int lv = 0; lv < LV; ++lv)
    if (g & (1 << lv)) base += 8 >> lv;
  const bool owner = g < 16;  // lanes g ≥ 16 hold copies of lanes g − 16's slots
  auto skip_at = [&](int k, int pb) {  // the up-sampled skip term of slot k (0 if none)
    const int u = k >> 2, c = k & 3, p = pb + u * ppp + sub;
    if (!skip || !owner || c == 3 || p >= p_end) return 0.f;
    const int y = p / W, x = p - (p / W) * W;
    return skip_up2(skip + ((size_t)n * 3 + c) * Hs * Ws, Hs, Ws, y, x);
  };
  for (int pb = p_begin; pb < p_end; pb += ppp * U) {
    // the skip terms first: their loads overlap the channel loads instead of following the
    // reduction (the first 4 of the lane's slots: all of them from tpp = 4 on)
    float skv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) skv[i] = i < nsl ? skip_at(base + i, pb) : 0.f;
    float a[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u][0] = a[u][1] = a[u][2] = 0.f;
    for (int cc = 0; cc < cpt; ++cc) {
      const int c0 = (g + cc * tpp) * V;
      VT v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped, unconditional: the U loads issue back-to-back
        const int p = min(pb + u * ppp + sub, p_end - 1);
        v[u] = *(const VT*)(img + (size_t)p * Cin + c0);
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float w0 = wm[c0 + e], w1 = wm[Cin + c0 + e], w2 = wm[2 * Cin + c0 + e];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float x = act_in ? lrelu_s2(to_f(v[u][e])) : to_f(v[u][e]);
          // fused explicitly: a contractible a += x·w may be left unfused when the vectorizer
          // pairs the products, which made the 2-byte outputs depend on code generation
          a[u][0] = __builtin_fmaf(x, w0, a[u][0]);
          a[u][1] = __builtin_fmaf(x, w1, a[u][1]);
          a[u][2] = __builtin_fmaf(x, w2, a[u][2]);
        }
      }
    }
    float sl[16];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      sl[4 * u] = a[u][0];
      sl[4 * u + 1] = a[u][1];
      sl[4 * u + 2] = a[u][2];
      sl[4 * u + 3] = 0.f;
    }
#pragma unroll
    for (int lv = 0; lv < LV; ++lv) {
      const int o = 1 << lv, h = 8 >> lv;
      const bool hi = (g & o) != 0;
#pragma unroll
      for (int i = 0; i < h; ++i) {
        // (the asm hides that both operands are loads of sl: folding the selects into one
        // select-indexed load would keep sl in memory as a 16-way compare chain)
        float x = sl[i], y = sl[h + i];
        asm volatile("" : "+v"(x), "+v"(y));
        const float keep = hi ? y : x, send = hi ? x : y;
        sl[i] = keep + __shfl_xor(send, o, 64);
      }
    }
    for (int o = 16; o < tpp; o <<= 1) sl[0] += __shfl_xor(sl[0], o, 64);
#pragma unroll
    for (int i = 0; i < nsl; ++i) {
      const int k = base + i, u = k >> 2, c = k & 3;
      const int p = pb + u * ppp + sub;
      if (!owner || c == 3 || p >= p_end) continue;
      float r = bias[c];
      r += sl[i];
      if (skip) r += i < 4 ? skv[i] : skip_at(k, pb);
      rgb[((size_t)n * 3 + c) * HW + p] = r;
    }
  }
}

// FRONT: the ToRGB feeds the topmost StyledConv, whose activation gradient is this ToRGB's alone;
// then also run that conv's backward front (as mia_bias_act_bwd(from_act) would): g_a is written
// as gy = g·lrelu'(a)·demod and q[n][c] += g·lrelu'(a)·(pre − nw·noise − b).
struct TorgbFront {
  const float* demod;
  const float* noise;
  float nw;
  const float* bias;
  float* q;
};

template <typename T, bool FRONT>
__global__ void torgb_bwd_kernel(const float* __restrict__ grgb, const T* __restrict__ pre,
                                 const float* __restrict__ s, const float* __restrict__ wr,
                                 T* __restrict__ g_a, float* __restrict__ part_out, int H, int W,
                                 int Cin, int accumulate, int pix_per_block, int act_in,
                                 TorgbFront fr) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  extern __shared__ float sh[];  // wr [3][Cin], s [Cin], partials [TPB/tpp][Cin] (× 2 if FRONT)
  const int n = blockIdx.y;
  float* w3 = sh;
  float* sn = sh + 3 * Cin;
  float* part = sh + 4 * Cin;
  for (int i = threadIdx.x; i < 3 * Cin; i += TPB) w3[i] = wr[i];
  for (int i = threadIdx.x; i < Cin; i += TPB) sn[i] = s[(size_t)n * Cin + i];
  __syncthreads();
  const int HW = H * W;
  const int nch = Cin / V;                // chunks per pixel
  const int tpp = nch < TPB ? nch : TPB;  // one chunk per thread
  const int ppp = TPB / tpp;
  const int t = threadIdx.x;
  const int chunk = t % tpp, sub = t / tpp;
  const int c0 = chunk * V;
  float acc[V], qa[V], dm[V], bs[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = qa[e] = 0.f;
  if (FRONT) {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      dm[e] = fr.demod[(size_t)n * Cin + c0 + e];
      bs[e] = fr.bias ? fr.bias[c0 + e] : 0.f;
    }
  }
  const int p_begin = blockIdx.x * pix_per_block;
  const int p_end = min(p_begin + pix_per_block, HW);
  if (sub < ppp) {
    for (int p = p_begin + sub; p < p_end; p += ppp) {
      const float g0 = grgb[((size_t)n * 3 + 0) * HW + p];
      const float g1 = grgb[((size_t)n * 3 + 1) * HW + p];
      const float g2 = grgb[((size_t)n * 3 + 2) * HW + p];
      const size_t off = ((size_t)n * HW + p) * Cin + c0;
      const VT pr = *(const VT*)(pre + off);
      VT ga;
      if (accumulate) ga = *(const VT*)(g_a + off);
      const float nz = (FRONT && fr.noise) ? fr.nw * fr.noise[p] : 0.f;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int c = c0 + e;
        const float u = g0 * w3[c] + g1 * w3[Cin + c] + g2 * w3[2 * Cin + c];
        acc[e] += (act_in ? lrelu_s2(to_f(pr[e])) : to_f(pr[e])) * u;
        float gv = sn[c] * u + (accumulate ? to_f(ga[e]) : 0.f);
        if (FRONT) {  // stored activation a = pr (act_in NONE)
          const float a = to_f(pr[e]);
          const float gr = lrelu_s2_grad(a);
          const float gp = gv * gr;
          qa[e] += gp * (a * lrelu_s2_inv_grad(a) - nz - bs[e]);
          gv = gp * dm[e];
        }
        ga[e] = from_f<T>(gv);
      }
      *(VT*)(g_a + off) = ga;
    }
  }
  float* partq = part + ppp * Cin;
  if (sub < ppp) {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      part[sub * Cin + c0 + e] = acc[e];
      if (FRONT) partq[sub * Cin + c0 + e] = qa[e];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < Cin; c += TPB) {
    float sum = 0.f, sq = 0.f;
    for (int sb = 0; sb < ppp; ++sb) {
      sum += part[sb * Cin + c];
      if (FRONT) sq += partq[sb * Cin + c];
    }
    // the block's partials into its slot (blockIdx.x): gs (quantity 0) and q (1)
    red_store(part_out, gridDim.x, gridDim.y * Cin, 0, blockIdx.x, n * Cin + c, sum);
    if (FRONT) red_store(part_out, gridDim.x, gridDim.y * Cin, 1, blockIdx.x, n * Cin + c, sq);
  }
}

// ---------------------------------------------------------------------------------------------
// MaxPool 2x2 stride 2 (NHWC), PyTorch semantics incl. ceil_mode and first-max tie rule.
// One thread per 2×2 window and 16-byte channel vector. All loads are unconditional (coordinates
// clamped into the image; a clamped duplicate is excluded by its validity flag), so they issue
// back-to-back instead of each behind its own branch and vmcnt(0).
template <typename T>
__global__ void maxpool2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H,
                                    int W, int C, int Ho, int Wo) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  const int nc = C / V;
  const int64_t total = (int64_t)N * Ho * Wo * nc;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int cv = (int)(i % nc);
    const int64_t pix = i / nc;
    const int ox = (int)(pix % Wo);
    const int oy = (int)((pix / Wo) % Ho);
    const int n = (int)(pix / ((int64_t)Wo * Ho));
    const int y0 = 2 * oy, x0 = 2 * ox;
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const T* b = x + (size_t)n * H * W * C + cv * V;
    const VT v[4] = {*(const VT*)(b + ((size_t)y0 * W + x0) * C),
                     *(const VT*)(b + ((size_t)y0 * W + x1) * C),
                     *(const VT*)(b + ((size_t)y1 * W + x0) * C),
                     *(const VT*)(b + ((size_t)y1 * W + x1) * C)};
    const bool ok[4] = {true, x0 + 1 < W, y0 + 1 < H, x0 + 1 < W && y0 + 1 < H};
    VT best = v[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      if (!ok[k]) continue;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float fv = to_f(v[k][e]), fb = to_f(best[e]);
        if (fv > fb || fv != fv) best[e] = v[k][e];  // first max wins; NaN propagates
      }
    }
    *(VT*)(y + pix * C + cv * V) = best;
  }
}

// Backward per window: the window's gradient goes to its first-max position; the tap-MSE term
// tap_coef·(x − t) and the ReLU mask (x > 0) of the layer below are fused. Windows beyond
// (Ho, Wo) (floor mode, odd size) only carry the tap/mask terms.
template <typename T, bool TAP>
__global__ void maxpool2_bwd_kernel(const T* __restrict__ x, const T* __restrict__ gout,
                                    T* __restrict__ gin, int N, int H, int W, int C, int Ho, int Wo,
                                    const T* __restrict__ tap_t, float tap_coef, int mask) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  const int nc = C / V;
  const int WY = (H + 1) / 2, WX = (W + 1) / 2;
  const int64_t total = (int64_t)N * WY * WX * nc;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int cv = (int)(i % nc);
    const int64_t w = i / nc;
    const int wx = (int)(w % WX);
    const int wy = (int)((w / WX) % WY);
    const int n = (int)(w / ((int64_t)WX * WY));
    const int y0 = 2 * wy, x0 = 2 * wx;
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const size_t off[4] = {((size_t)y0 * W + x0) * C, ((size_t)y0 * W + x1) * C,
                           ((size_t)y1 * W + x0) * C, ((size_t)y1 * W + x1) * C};
    const bool ok[4] = {true, x0 + 1 < W, y0 + 1 < H, x0 + 1 < W && y0 + 1 < H};
    const size_t img = (size_t)n * H * W * C + cv * V;
    const bool pooled = wy < Ho && wx < Wo;
    const VT go = *(const VT*)(gout + (((size_t)n * Ho + min(wy, Ho - 1)) * Wo + min(wx, Wo - 1)) * C +
                               cv * V);
    VT xv[4], tv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) xv[k] = *(const VT*)(x + img + off[k]);
    if (TAP) {
#pragma unroll
      for (int k = 0; k < 4; ++k) tv[k] = *(const VT*)(tap_t + img + off[k]);
    }
    int bpos[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      float bv = to_f(xv[0][e]);
      bpos[e] = 0;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float fv = to_f(xv[k][e]);
        if (ok[k] && (fv > bv || fv != fv)) { bv = fv; bpos[e] = k; }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!ok[k]) continue;
      VT o;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float xf = to_f(xv[k][e]);
        float r = (pooled && bpos[e] == k) ? to_f(go[e]) : 0.f;
        if (TAP) r += tap_coef * (xf - to_f(tv[k][e]));
        if (mask && !(xf > 0.f)) r = 0.f;
        o[e] = from_f<T>(r);
      }
      *(VT*)(gin + img + off[k]) = o;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// avg_pool2d(k, stride k) on fp32 NCHW planes and its backward.
__global__ void avgpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int planes,
                                   int H, int W, int k) {
  const int Ho = H / k, Wo = W / k;
  const int64_t total = (int64_t)planes * Ho * Wo;
  const float inv = 1.f / (float)(k * k);
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int ox = (int)(i % Wo);
    const int oy = (int)((i / Wo) % Ho);
    const int64_t pl = i / ((int64_t)Wo * Ho);
    const float* xp = x + pl * H * W + (size_t)oy * k * W + ox * k;
    float acc = 0.f;
    for (int dy = 0; dy < k; ++dy)
      for (int dx = 0; dx < k; ++dx) acc += xp[dy * W + dx];
    y[i] = acc * inv;
  }
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ gy, float* __restrict__ gx,
                                   int planes, int H, int W, int k, int accumulate) {
  const int Ho = H / k, Wo = W / k;
  const int64_t total = (int64_t)planes * H * W;
  const float inv = 1.f / (float)(k * k);
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int ix = (int)(i % W);
    const int iy = (int)((i / W) % H);
    const int64_t pl = i / ((int64_t)W * H);
    const int oy = iy / k, ox = ix / k;
    float v = (oy < Ho && ox < Wo) ? gy[pl * Ho * Wo + oy * Wo + ox] * inv : 0.f;
    if (accumulate) v += gx[i];
    gx[i] = v;
  }
}

// NCHW fp32 (N,3,S,S) → avg_pool(pf) → NHWC (N,S/pf,S/pf,cpad) in T, channels ≥ 3 zero.
template <typename T>
__global__ void image_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int S,
                                     int pf, int cpad) {
  const int R = S / pf;
  const int64_t total = (int64_t)N * R * R * cpad;
  const float inv = 1.f / (float)(pf * pf);
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int c = (int)(i % cpad);
    const int64_t pix = i / cpad;
    const int xo = (int)(pix % R);
    const int yo = (int)((pix / R) % R);
    const int n = (int)(pix / ((int64_t)R * R));
    float v = 0.f;
    if (c < 3) {
      const float* xp = x + (((size_t)n * 3 + c) * S + (size_t)yo * pf) * S + xo * pf;
      for (int dy = 0; dy < pf; ++dy)
        for (int dx = 0; dx < pf; ++dx) v += xp[dy * S + dx];
      v *= inv;
    }
    y[i] = from_f<T>(v);
  }
}

// The same with cpad a multiple of the 16-byte vector (the product's CPAD = 8): one thread per
// output pixel, its 3 planes' loads coalesced across the wave and its cpad channels written as
// whole 16-byte vectors (the element-per-thread form wrote 2- / 4-byte scalars at 1.8 TB/s).
// Same sums in the same order: bit-identical.
template <typename T>
__global__ __launch_bounds__(TPB) void image_to_nhwc_vec_kernel(const float* __restrict__ x,
                                                                T* __restrict__ y, int N, int S,
                                                                int pf, int cpad) {
  typedef typename Vec<T>::type VT;
  constexpr int V = Vec<T>::N;
  const int R = S / pf;
  const int64_t total = (int64_t)N * R * R;
  const float inv = 1.f / (float)(pf * pf);
  for (int64_t pix = blockIdx.x * (int64_t)TPB + threadIdx.x; pix < total;
       pix += (int64_t)gridDim.x * TPB) {
    const int xo = (int)(pix % R);
    const int yo = (int)((pix / R) % R);
    const int n = (int)(pix / ((int64_t)R * R));
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* xp = x + (((size_t)n * 3 + c) * S + (size_t)yo * pf) * S + xo * pf;
      float a = 0.f;
      for (int dy = 0; dy < pf; ++dy)
        for (int dx = 0; dx < pf; ++dx) a += xp[dy * S + dx];
      v[c] = a * inv;
    }
    T* out = y + pix * cpad;
    for (int q = 0; q < cpad / V; ++q) {
      VT o;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int ch = q * V + e;
        o[e] = from_f<T>(ch < 3 ? v[ch < 3 ? ch : 0] : 0.f);
      }
      *(VT*)(out + q * V) = o;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// MSE pieces (K10).
template <typename T>
__global__ void mse_sum_kernel(const T* __restrict__ a, const T* __restrict__ b,
                               float* __restrict__ part, int64_t len, float coef) {
  const int n = blockIdx.y;
  const T* pa = a + (size_t)n * len;
  const T* pb = b + (size_t)n * len;
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    const float d = to_f(pa[i]) - to_f(pb[i]);
    acc += d * d;
  }
  __shared__ float red[TPB / 64];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < TPB / 64; ++w) s += red[w];
    red_store(part, gridDim.x, gridDim.y, 0, blockIdx.x, n, coef * s);  // the block's slot
  }
}

__global__ void mse_grad_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                    float* __restrict__ g, int64_t len, float coef, int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    float v = coef * (a[i] - b[i]);
    if (accumulate) v += g[i];
    g[i] = v;
  }
}

template <typename T>
__global__ void tap_grad_kernel(const T* __restrict__ a, const T* __restrict__ t, T* __restrict__ g,
                                int64_t len, float coef, int mask) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    const float av = to_f(a[i]);
    float v = coef * (av - to_f(t[i]));
    if (mask && !(av > 0.f)) v = 0.f;
    g[i] = from_f<T>(v);
  }
}

template <typename T>
__global__ void image_grad_kernel(const float* __restrict__ rec, const float* __restrict__ t,
                                  const T* __restrict__ gv, float* __restrict__ gimg, int N, int S,
                                  int pf, int cpad, float coef) {
  const int R = S / pf;
  const int64_t total = (int64_t)N * 3 * S * S;
  const float inv = 1.f / (float)(pf * pf);
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const int x = (int)(i % S);
    const int y = (int)((i / S) % S);
    const int c = (int)((i / ((int64_t)S * S)) % 3);
    const int n = (int)(i / ((int64_t)S * S * 3));
    float g = coef * (rec[i] - t[i]);
    if (gv) g += to_f(gv[(((size_t)n * R + y / pf) * R + x / pf) * cpad + c]) * inv;
    gimg[i] = g;
  }
}

// ---------------------------------------------------------------------------------------------
// K11: PGD step with cost = −L (interpolation.py:92-94; torchattacks targeted form :83-86).
// Every operation is a single fp32 op with no contraction opportunity (a·sign is exact), so for an
// identical gradient the result is bit-identical to torch's fp32 CPU ops.
__device__ __forceinline__ float project1(float xa, float x0, float g, float a, float e, float lo,
                                          float hi) {
#pragma clang fp contract(off)
  const float sg = g < 0.f ? 1.f : (g > 0.f ? -1.f : 0.f);  // sign(−g)
  float adv = xa + a * sg;
  float d = adv - x0;
  d = fminf(fmaxf(d, -e), e);
  float r = x0 + d;
  return fminf(fmaxf(r, lo), hi);
}

__global__ void random_start_kernel(float* __restrict__ x, const float* __restrict__ x0,
                                    const float* __restrict__ u, int64_t len, float e, float lo,
                                    float hi) {
#pragma clang fp contract(off)
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    const float ue = e * u[i];  // rounded separately (no contraction), as torch mul then add
    x[i] = fminf(fmaxf(x0[i] + ue, lo), hi);
  }
}

__global__ void sign_project_kernel(float* __restrict__ x, const float* __restrict__ x0,
                                    const float* __restrict__ g, int64_t len, float a, float e,
                                    float lo, float hi) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB)
    x[i] = project1(x[i], x0[i], g[i], a, e, lo, hi);
}

// ∇_x L at image element i (NCHW fp32, S² planes): the image-MSE term coef_img·(x − x0) plus the
// adjoints of the two avg_pool2d's (attack_main2.py:590-591): the VGG input-path gradient at S/pf
// (NHWC, cpad channels) and the encoder gradient at enc_res, each spread over its pooling window.
template <typename T>
__device__ __forceinline__ float assemble_grad(int64_t i, float xv, float x0v, const T* gv,
                                               const float* genc, int S, int pf, int cpad,
                                               int enc_res, float coef_img) {
  const int R = S / pf;
  const int ek = S / enc_res;
  const int xx = (int)(i % S);
  const int yy = (int)((i / S) % S);
  const int c = (int)((i / ((int64_t)S * S)) % 3);
  const int n = (int)(i / ((int64_t)S * S * 3));
  float g = coef_img * (xv - x0v);
  if (gv) g += to_f(gv[(((size_t)n * R + yy / pf) * R + xx / pf) * cpad + c]) / (float)(pf * pf);
  if (genc) g += genc[(((size_t)n * 3 + c) * enc_res + yy / ek) * enc_res + xx / ek] / (float)(ek * ek);
  return g;
}

// A non-finite gradient element (an fp16 loss-scale overflow upstream, or a NaN in the
// weights) marks its image in nonfinite[n]; the host reads the flags once per attack
// (pgd.AttackEngine) instead of letting sign(NaN) = 0 freeze the pixel silently. Racing writers
// store the same value.
__device__ __forceinline__ void flag_nonfinite(int* nonfinite, int64_t i, int S, float g) {
  if (nonfinite && !__builtin_isfinite(g)) nonfinite[i / ((int64_t)3 * S * S)] = 1;
}

template <typename T>
__global__ void pgd_update_kernel(float* __restrict__ x, const float* __restrict__ x0,
                                  const T* __restrict__ gv, const float* __restrict__ genc, int N,
                                  int S, int pf, int cpad, int enc_res, float coef_img, float a,
                                  float e, float lo, float hi, int* __restrict__ nonfinite) {
  const int64_t total = (int64_t)N * 3 * S * S;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const float xv = x[i], x0v = x0[i];
    const float g = assemble_grad(i, xv, x0v, gv, genc, S, pf, cpad, enc_res, coef_img);
    flag_nonfinite(nonfinite, i, S, g);
    x[i] = project1(xv, x0v, g, a, e, lo, hi);
  }
}

template <typename T>
__global__ void grad_assemble_kernel(const float* __restrict__ x, const float* __restrict__ x0,
                                     const T* __restrict__ gv, const float* __restrict__ genc,
                                     float* __restrict__ g, int N, int S, int pf, int cpad,
                                     int enc_res, float coef_img, float scale,
                                     int* __restrict__ nonfinite) {
  const int64_t total = (int64_t)N * 3 * S * S;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB) {
    const float v = scale * assemble_grad(i, x[i], x0[i], gv, genc, S, pf, cpad, enc_res, coef_img);
    flag_nonfinite(nonfinite, i, S, v);
    g[i] = v;
  }
}

// ---- C&W L2 in tanh space (torchattacks CW, interpolation.py:98-193), images in [-1, 1]:
// adv = tanh(w) (= 2·½(tanh w + 1) − 1), w0 = atanh(x) with x clamped to ±(1 − 2⁻²⁰) so that
// saturated pixels stay finite.
__global__ void cw_init_kernel(const float* __restrict__ x, float* __restrict__ w, int64_t len) {
  constexpr float lim = 1.f - 9.5367431640625e-07f;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB)
    w[i] = atanhf(fminf(fmaxf(x[i], -lim), lim));
}

__global__ void cw_tanh_kernel(const float* __restrict__ w, float* __restrict__ adv, int64_t len) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB)
    adv[i] = tanhf(w[i]);
}

// ∂cost/∂w with cost = Σ_n ‖(adv − x)/2‖² + c·Σ_n f_n(adv) and adv = tanh w:
//   gw = (½(adv − x) + c·scale·g_f)·(1 − adv²)        (g_f = ∇f, loss-scaled; scale undoes it)
__global__ void cw_grad_kernel(const float* __restrict__ adv, const float* __restrict__ x,
                               const float* __restrict__ gf, float* __restrict__ gw, int64_t len,
                               float c, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    const float a = adv[i];
    gw[i] = (0.5f * (a - x[i]) + c * scale * gf[i]) * (1.f - a * a);
  }
}

// Best-L2 bookkeeping (torchattacks CW :154-163), one block per image: an image is a success when
// its objective is below the clean image's (f_n < f0_n, the GAN objective has no labels) and its
// L2 = l2_scale·Σ(adv − x)² beats the best so far; then best_adv[n] ← adv[n].
__global__ void cw_select_kernel(const float* __restrict__ adv, float* __restrict__ best_adv,
                                 const float* __restrict__ sq, float* __restrict__ best_l2,
                                 const float* __restrict__ f, const float* __restrict__ f0,
                                 int64_t plane, float l2_scale) {
  const int n = blockIdx.x;
  const float l2 = l2_scale * sq[n];
  const bool take = f[n] < f0[n] && best_l2[n] > l2;
  __syncthreads();
  if (!take) return;
  for (int64_t i = threadIdx.x; i < plane; i += TPB) best_adv[(size_t)n * plane + i] = adv[(size_t)n * plane + i];
  if (threadIdx.x == 0) best_l2[n] = l2;
}

// K12: Adam on pixels (torch.optim.Adam single-tensor semantics, no weight decay).
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t len, float lr, float b1, float b2,
                            float eps, float bc1, float bc2sqrt) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    const float gi = g[i];
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2sqrt + eps;
    p[i] = p[i] - (lr / bc1) * (mi / denom);
  }
}

// Adversarial patch (code/attack/patch/adversarial_patch.py:131-134, attack_main2.py:413-420):
//   patch −= g (the full-image gradient, step 1);  adv = (1 − m)·img + m·patch;
//   adv = clamp(adv, lo, hi) with lo / hi = min / max of the clean images.
// Each torch op is one fp32 rounding (no contraction), so the result is bit-identical to torch's
// fp32 ops for the same gradient. `g` may be null (composite only, patch_white_box). `shared` =
// numel of mask / patch when they are one image broadcast over the batch (0: same shape as img).
__global__ void patch_update_kernel(float* __restrict__ patch, const float* __restrict__ g,
                                    const float* __restrict__ img, const float* __restrict__ mask,
                                    float* __restrict__ adv, int64_t len, int64_t shared, float lo,
                                    float hi) {
#pragma clang fp contract(off)
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    const int64_t j = shared ? i % shared : i;
    float pv = patch[j];
    if (g) {
      pv = pv - g[i];
      patch[j] = pv;
    }
    const float m = mask[j];
    const float a = (1.f - m) * img[i];
    const float b = m * pv;
    adv[i] = fminf(fmaxf(a + b, lo), hi);
  }
}

// PixelNorm of the mapping network input (rosinality PixelNorm): y = x / sqrt(mean(x²) + eps)
// over each row of `cols` values; one block per row.
__global__ void pixel_norm_kernel(const float* __restrict__ x, float* __restrict__ y, int cols,
                                  float eps) {
  const float* xr = x + (size_t)blockIdx.x * cols;
  float* yr = y + (size_t)blockIdx.x * cols;
  float acc = 0.f;
  for (int i = threadIdx.x; i < cols; i += TPB) acc += xr[i] * xr[i];
  __shared__ float red[TPB / 64];
  __shared__ float inv;
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < TPB / 64; ++w) s += red[w];
    inv = rsqrtf(s / (float)cols + eps);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cols; i += TPB) yr[i] = xr[i] * inv;
}

// Truncation trick (rosinality Generator.forward): out = mean + psi·(w − mean), mean broadcast
// over rows.
__global__ void truncate_kernel(const float* __restrict__ w, const float* __restrict__ mean,
                                float psi, float* __restrict__ out, int64_t len, int cols) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < len; i += (int64_t)gridDim.x * TPB) {
    const float m = mean[i % cols];
    out[i] = m + psi * (w[i] - m);
  }
}

__global__ void repeat_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                              int64_t bytes, int count) {
  const int64_t total = bytes * count;
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < total; i += (int64_t)gridDim.x * TPB)
    dst[i] = src[i % bytes];
}

}  // namespace mia

using namespace mia;

#define MIA_LAUNCH(kern, grid, block, shmem, ...)                                  \
  do {                                                                             \
    hipLaunchKernelGGL(kern, grid, block, shmem, (hipStream_t)stream, __VA_ARGS__); \
    return check_launch(#kern);                                                    \
  } while (0)

extern "C" int mia_bias_act_fwd(const void* x, const float* noise, float noise_w,
                                const float* bias, void* y, int N, int H, int W, int C, int dtype,
                                void* stream) {
  MIA_CHECK_ARG(x && y && N > 0 && H > 0 && W > 0 && C > 0, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(C % V == 0, "C must be a multiple of the vector width");
  const int64_t nvec = (int64_t)N * H * W * C / V;
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH(bias_act_fwd_kernel<T>, dim3(blocks_for(nvec, TPB, 65536)), dim3(TPB), 0,
                 (const T*)x, noise, noise_w, bias, (T*)y, nvec, C, H * W));
  return MIA_OK;
}

extern "C" int mia_bias_act_bwd(const void* g_a, const void* pre, const float* noise,
                                float noise_w, const float* bias, const float* demod, void* gy,
                                float* q, int N, int H, int W, int C, int unshuffle, int from_act,
                                int dtype, void* stream) {
  MIA_CHECK_ARG(g_a && pre && demod && gy && q, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(C % V == 0 && C / V <= TPB && (TPB % (C / V)) == 0, "C/V must divide 256");
  MIA_CHECK_ARG(!unshuffle || (H % 2 == 0 && W % 2 == 0), "unshuffle needs even H, W");
  const int HW = H * W;
  const int ppp = TPB / (C / V);
  const int ppb = ppp * 16;
  dim3 grid((HW + ppb - 1) / ppb, N);
  RedQ r;
  int rc = red_begin(r, q, nullptr, nullptr, grid.x, N * C, (hipStream_t)stream);
  if (rc != MIA_OK) return rc;
  MIA_DISPATCH_DTYPE(dtype, T,
      hipLaunchKernelGGL(bias_act_bwd_kernel<T>, grid, dim3(TPB), 0, (hipStream_t)stream,
                         (const T*)g_a, (const T*)pre, noise, noise_w, bias, demod, (T*)gy, r.part,
                         H, W, C, unshuffle, from_act, ppb));
  rc = check_launch("bias_act_bwd_kernel");
  return rc != MIA_OK ? rc : red_finish(r, (hipStream_t)stream);
}

extern "C" int mia_upconv_blur_fwd(const void* t, void* pre, const float* demod,
                                   const float* noise, float noise_w, const float* bias, int N,
                                   int R, int C, int act_out, int dtype, void* stream) {
  MIA_CHECK_ARG(t && pre && demod && N > 0 && R > 0, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(C % V == 0, "C must be a multiple of the vector width");
  const int SY = (2 * R + 2 * kBlurKQ - 1) / (2 * kBlurKQ);
  const int64_t total = (int64_t)N * SY * R * (C / V);
  MIA_DISPATCH_DTYPE(dtype, T,
      if (noise) {
        MIA_LAUNCH((blur4_strip_kernel<T, true, true>), dim3(blocks_for(total, TPB, 65536)),
                   dim3(TPB), 0, (const T*)t, (T*)pre, demod, noise, noise_w, bias, N, R, C,
                   act_out);
      } else {
        MIA_LAUNCH((blur4_strip_kernel<T, true, false>), dim3(blocks_for(total, TPB, 65536)),
                   dim3(TPB), 0, (const T*)t, (T*)pre, demod, noise, noise_w, bias, N, R, C,
                   act_out);
      });
  return MIA_OK;
}

extern "C" int mia_upconv_blur_bwd(const void* gy, void* gt, int N, int R, int C, int dtype,
                                   void* stream) {
  MIA_CHECK_ARG(gy && gt && N > 0 && R > 0, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(C % V == 0, "C must be a multiple of the vector width");
  const int SY = (2 * R + 1 + 2 * kBlurKQ - 1) / (2 * kBlurKQ);
  const int64_t total = (int64_t)N * SY * (R + 1) * (C / V);
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH((blur4_strip_kernel<T, false, false>), dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0,
                 (const T*)gy, (T*)gt, nullptr, nullptr, 0.f, nullptr, N, R, C, 0));
  return MIA_OK;
}

static int make_taps(const float* k1d, int ktaps, Taps8* kf) {
  if (ktaps < 1 || ktaps > 8) return mia::set_error("upfirdn2d: 1..8 taps");
  for (int j = 0; j < 8; ++j) kf->k[j] = 0.f;
  for (int j = 0; j < ktaps; ++j) kf->k[j] = k1d[ktaps - 1 - j];  // flipped (correlation form)
  return MIA_OK;
}

extern "C" int mia_upfirdn2d_fwd(const float* x, float* y, int planes, int H, int W,
                                 const float* k1d, int ktaps, int up, int down, int pad0, int pad1,
                                 void* stream) {
  MIA_CHECK_ARG(x && y && k1d && up >= 1 && down >= 1, "bad args");
  Taps8 kf;
  if (make_taps(k1d, ktaps, &kf)) return MIA_EINVAL;
  const int Ho = (H * up + pad0 + pad1 - ktaps) / down + 1;
  const int Wo = (W * up + pad0 + pad1 - ktaps) / down + 1;
  MIA_CHECK_ARG(Ho > 0 && Wo > 0, "empty output");
  const int64_t total = (int64_t)planes * Ho * Wo;
  MIA_LAUNCH(upfirdn2d_fwd_kernel, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, x, y, planes,
             H, W, Ho, Wo, kf, ktaps, up, down, pad0);
}

extern "C" int mia_upfirdn2d_bwd(const float* gy, float* gx, int planes, int H, int W,
                                 const float* k1d, int ktaps, int up, int down, int pad0, int pad1,
                                 void* stream) {
  MIA_CHECK_ARG(gy && gx && k1d && up >= 1 && down >= 1, "bad args");
  Taps8 kf;
  if (make_taps(k1d, ktaps, &kf)) return MIA_EINVAL;
  const int Ho = (H * up + pad0 + pad1 - ktaps) / down + 1;
  const int Wo = (W * up + pad0 + pad1 - ktaps) / down + 1;
  MIA_CHECK_ARG(Ho > 0 && Wo > 0, "empty output");
  const int64_t total = (int64_t)planes * H * W;
  MIA_LAUNCH(upfirdn2d_bwd_kernel, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, gy, gx,
             planes, H, W, Ho, Wo, kf, ktaps, up, down, pad0);
}

// the ToRGB forward with lv = min(4, log2 tpp) reduce-scatter levels (each lane keeps 16 >> lv
// of the lane group's 16 sum slots)
template <typename T>
static int launch_torgb_fwd(dim3 grid, size_t sh, const T* pre, const float* style,
                            const float* wr, const float* bias, const float* skip, float* rgb,
                            int H, int W, int Cin, int tpp, int cpt, int ppb, int act_in,
                            hipStream_t st) {
  const int lv = tpp >= 16 ? 4 : tpp == 8 ? 3 : tpp == 4 ? 2 : tpp == 2 ? 1 : 0;
  auto fn = lv == 4 ? torgb_fwd_kernel<T, 4> : lv == 3 ? torgb_fwd_kernel<T, 3>
          : lv == 2 ? torgb_fwd_kernel<T, 2> : lv == 1 ? torgb_fwd_kernel<T, 1>
                    : torgb_fwd_kernel<T, 0>;
  hipLaunchKernelGGL(fn, grid, dim3(TPB), sh, st, pre, style, wr, bias, skip, rgb, H, W, Cin, tpp,
                     cpt, ppb, act_in);
  return check_launch("torgb_fwd_kernel");
}

extern "C" int mia_torgb_fwd(const void* pre, const float* style, const float* wr,
                             const float* bias, const float* skip, float* rgb, int N, int H, int W,
                             int Cin, int act_in, int dtype, void* stream) {
  MIA_CHECK_ARG(pre && style && wr && bias && rgb, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(Cin % V == 0, "Cin must be a multiple of the vector width");
  int nch = Cin / V;
  int tpp = 1;
  while (tpp * 2 <= nch && tpp * 2 <= 64) tpp *= 2;
  MIA_CHECK_ARG(nch % tpp == 0, "Cin/V must be a power of two times tpp");
  const int cpt = nch / tpp;
  const int ppb = (TPB / tpp) * 16;  // 4 passes of U = 4 pixels per lane group
  dim3 grid((H * W + ppb - 1) / ppb, N);
  const size_t sh = 3 * Cin * sizeof(float);
  MIA_DISPATCH_DTYPE(dtype, T,
      return launch_torgb_fwd<T>(grid, sh, (const T*)pre, style, wr, bias, skip, rgb, H, W, Cin,
                                 tpp, cpt, ppb, act_in, (hipStream_t)stream));
  return MIA_OK;
}

extern "C" int mia_torgb_bwd(const float* g_rgb, const void* pre, const float* style,
                             const float* wr, void* g_a, float* gs, int N, int H, int W, int Cin,
                             int accumulate, int act_in, int dtype, void* stream) {
  MIA_CHECK_ARG(g_rgb && pre && style && wr && g_a && gs, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(Cin % V == 0 && Cin / V <= TPB && TPB % (Cin / V) == 0, "Cin/V must divide 256");
  const int ppp = TPB / (Cin / V);
  const int ppb = ppp * 16;
  dim3 grid((H * W + ppb - 1) / ppb, N);
  const size_t sh = (4 * Cin + (size_t)ppp * Cin) * sizeof(float);
  MIA_CHECK_ARG(sh <= 64 * 1024, "LDS budget");
  const TorgbFront fr{};
  RedQ r;
  int rc = red_begin(r, gs, nullptr, nullptr, grid.x, N * Cin, (hipStream_t)stream);
  if (rc != MIA_OK) return rc;
  MIA_DISPATCH_DTYPE(dtype, T,
      hipLaunchKernelGGL((torgb_bwd_kernel<T, false>), grid, dim3(TPB), sh, (hipStream_t)stream,
                         g_rgb, (const T*)pre, style, wr, (T*)g_a, r.part, H, W, Cin, accumulate,
                         ppb, act_in, fr));
  rc = check_launch("torgb_bwd_kernel");
  return rc != MIA_OK ? rc : red_finish(r, (hipStream_t)stream);
}

extern "C" int mia_torgb_bwd_front(const float* g_rgb, const void* act, const float* style,
                                   const float* wr, void* gy, float* gs, int N, int H, int W,
                                   int Cin, const float* demod, const float* noise, float noise_w,
                                   const float* bias, float* q, int dtype, void* stream) {
  MIA_CHECK_ARG(g_rgb && act && style && wr && gy && gs && demod && q, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(Cin % V == 0 && Cin / V <= TPB && TPB % (Cin / V) == 0, "Cin/V must divide 256");
  const int ppp = TPB / (Cin / V);
  const int ppb = ppp * 16;
  dim3 grid((H * W + ppb - 1) / ppb, N);
  const size_t sh = (4 * Cin + 2 * (size_t)ppp * Cin) * sizeof(float);
  MIA_CHECK_ARG(sh <= 64 * 1024, "LDS budget");
  const TorgbFront fr{demod, noise, noise_w, bias, q};
  RedQ r;
  int rc = red_begin(r, gs, q, nullptr, grid.x, N * Cin, (hipStream_t)stream);
  if (rc != MIA_OK) return rc;
  MIA_DISPATCH_DTYPE(dtype, T,
      hipLaunchKernelGGL((torgb_bwd_kernel<T, true>), grid, dim3(TPB), sh, (hipStream_t)stream,
                         g_rgb, (const T*)act, style, wr, (T*)gy, r.part, H, W, Cin, 0, ppb,
                         MIA_ACT_NONE, fr));
  rc = check_launch("torgb_bwd_kernel");
  return rc != MIA_OK ? rc : red_finish(r, (hipStream_t)stream);
}

static inline int pool_out(int H, int ceil_mode) { return ceil_mode ? (H + 1) / 2 : H / 2; }

extern "C" int mia_maxpool2_fwd(const void* x, void* y, int N, int H, int W, int C, int ceil_mode,
                                int dtype, void* stream) {
  MIA_CHECK_ARG(x && y && H >= 2 && W >= 2, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(C % V == 0, "C must be a multiple of the vector width");
  const int Ho = pool_out(H, ceil_mode), Wo = pool_out(W, ceil_mode);
  const int64_t total = (int64_t)N * Ho * Wo * (C / V);
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH(maxpool2_fwd_kernel<T>, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0,
                 (const T*)x, (T*)y, N, H, W, C, Ho, Wo));
  return MIA_OK;
}

extern "C" int mia_maxpool2_bwd(const void* x, const void* g_out, void* g_in, int N, int H, int W,
                                int C, int ceil_mode, const void* tap_t, float tap_coef, int mask,
                                int dtype, void* stream) {
  MIA_CHECK_ARG(x && g_out && g_in && H >= 2 && W >= 2, "bad args");
  const int V = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(C % V == 0, "C must be a multiple of the vector width");
  const int Ho = pool_out(H, ceil_mode), Wo = pool_out(W, ceil_mode);
  const int64_t total = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / V);
  MIA_DISPATCH_DTYPE(dtype, T,
      if (tap_t) {
        MIA_LAUNCH((maxpool2_bwd_kernel<T, true>), dim3(blocks_for(total, TPB, 65536)), dim3(TPB),
                   0, (const T*)x, (const T*)g_out, (T*)g_in, N, H, W, C, Ho, Wo, (const T*)tap_t,
                   tap_coef, mask);
      } else {
        MIA_LAUNCH((maxpool2_bwd_kernel<T, false>), dim3(blocks_for(total, TPB, 65536)), dim3(TPB),
                   0, (const T*)x, (const T*)g_out, (T*)g_in, N, H, W, C, Ho, Wo, (const T*)tap_t,
                   tap_coef, mask);
      });
  return MIA_OK;
}

extern "C" int mia_avgpool_fwd(const float* x, float* y, int planes, int H, int W, int k,
                               void* stream) {
  MIA_CHECK_ARG(x && y && k >= 1 && H >= k && W >= k, "bad args");
  const int64_t total = (int64_t)planes * (H / k) * (W / k);
  MIA_LAUNCH(avgpool_fwd_kernel, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, x, y, planes,
             H, W, k);
}

extern "C" int mia_avgpool_bwd(const float* gy, float* gx, int planes, int H, int W, int k,
                               int accumulate, void* stream) {
  MIA_CHECK_ARG(gy && gx && k >= 1 && H >= k && W >= k, "bad args");
  const int64_t total = (int64_t)planes * H * W;
  MIA_LAUNCH(avgpool_bwd_kernel, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, gy, gx, planes,
             H, W, k, accumulate);
}

extern "C" int mia_image_to_nhwc(const float* x, void* y, int N, int S, int pf, int cpad,
                                 int dtype, void* stream) {
  MIA_CHECK_ARG(x && y && pf >= 1 && S % pf == 0 && cpad >= 3, "bad args");
  const int R = S / pf;
  const int64_t total = (int64_t)N * R * R * cpad;
  const int V = dtype == MIA_F32 ? 4 : 8;
  if (cpad % V == 0) {
    const int64_t pixels = (int64_t)N * R * R;
    MIA_DISPATCH_DTYPE(dtype, T,
        MIA_LAUNCH(image_to_nhwc_vec_kernel<T>, dim3(blocks_for(pixels, TPB, 65536)), dim3(TPB),
                   0, x, (T*)y, N, S, pf, cpad));
  }
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH(image_to_nhwc_kernel<T>, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, x,
                 (T*)y, N, S, pf, cpad));
  return MIA_OK;
}

extern "C" int mia_mse_sum(const void* a, const void* b, float* loss, int n, int64_t len,
                           float coef, int dtype, void* stream) {
  MIA_CHECK_ARG(a && b && loss && n > 0 && len > 0, "bad args");
  dim3 grid(blocks_for(len, TPB, 1024), n);
  RedQ r;
  int rc = red_begin(r, loss, nullptr, nullptr, grid.x, n, (hipStream_t)stream);
  if (rc != MIA_OK) return rc;
  MIA_DISPATCH_DTYPE(dtype, T,
      hipLaunchKernelGGL(mse_sum_kernel<T>, grid, dim3(TPB), 0, (hipStream_t)stream, (const T*)a,
                         (const T*)b, r.part, len, coef));
  rc = check_launch("mse_sum_kernel");
  return rc != MIA_OK ? rc : red_finish(r, (hipStream_t)stream);
}

extern "C" int mia_mse_grad_f32(const float* a, const float* b, float* g, int64_t len, float coef,
                                int accumulate, void* stream) {
  MIA_CHECK_ARG(a && b && g && len > 0, "bad args");
  MIA_LAUNCH(mse_grad_f32_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, a, b, g, len,
             coef, accumulate);
}

extern "C" int mia_tap_grad(const void* a, const void* t, void* g, int64_t len, float coef,
                            int mask, int dtype, void* stream) {
  MIA_CHECK_ARG(a && t && g && len > 0, "bad args");
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH(tap_grad_kernel<T>, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, (const T*)a,
                 (const T*)t, (T*)g, len, coef, mask));
  return MIA_OK;
}

extern "C" int mia_mse_fwd_bwd(const void* a, const void* b, float* loss, void* g, int n,
                               int64_t len, float coef_loss, float coef_grad, int accumulate,
                               int dtype, void* stream) {
  MIA_CHECK_ARG(a && b && (loss || g) && n > 0 && len > 0, "bad args");
  MIA_CHECK_ARG(!g || dtype == MIA_F32 || !accumulate,
                "accumulating gradient is fp32 only (mia_mse_grad_f32)");
  if (loss) {
    const int rc = mia_mse_sum(a, b, loss, n, len, coef_loss, dtype, stream);
    if (rc != MIA_OK) return rc;
  }
  if (!g) return MIA_OK;
  if (dtype == MIA_F32)
    return mia_mse_grad_f32((const float*)a, (const float*)b, (float*)g, (int64_t)n * len,
                            coef_grad, accumulate, stream);
  return mia_tap_grad(a, b, g, (int64_t)n * len, coef_grad, 0, dtype, stream);
}

extern "C" int mia_image_grad(const float* rec, const float* t, const void* g_vgg, float* g_img,
                              int N, int S, int pf, int cpad, float coef, int dtype, void* stream) {
  MIA_CHECK_ARG(rec && t && g_img && pf >= 1 && S % pf == 0, "bad args");
  const int64_t total = (int64_t)N * 3 * S * S;
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH(image_grad_kernel<T>, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, rec, t,
                 (const T*)g_vgg, g_img, N, S, pf, cpad, coef));
  return MIA_OK;
}

extern "C" int mia_pgd_update(float* x, const float* x0, const void* g_vgg, const float* g_enc,
                              int N, int S, int pf, int cpad, int enc_res, float coef_img, float a,
                              float e, float lo, float hi, int* nonfinite, int dtype,
                              void* stream) {
  MIA_CHECK_ARG(x && x0 && pf >= 1 && S % pf == 0 && enc_res >= 1 && S % enc_res == 0, "bad args");
  const int64_t total = (int64_t)N * 3 * S * S;
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH(pgd_update_kernel<T>, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, x, x0,
                 (const T*)g_vgg, g_enc, N, S, pf, cpad, enc_res, coef_img, a, e, lo, hi,
                 nonfinite));
  return MIA_OK;
}

extern "C" int mia_grad_assemble(const float* x, const float* x0, const void* g_vgg,
                                 const float* g_enc, float* g, int N, int S, int pf, int cpad,
                                 int enc_res, float coef_img, float scale, int* nonfinite,
                                 int dtype, void* stream) {
  MIA_CHECK_ARG(x && x0 && g && pf >= 1 && S % pf == 0 && (!g_enc || S % enc_res == 0), "bad args");
  const int64_t total = (int64_t)N * 3 * S * S;
  MIA_DISPATCH_DTYPE(dtype, T,
      MIA_LAUNCH(grad_assemble_kernel<T>, dim3(blocks_for(total, TPB, 65536)), dim3(TPB), 0, x,
                 x0, (const T*)g_vgg, g_enc, g, N, S, pf, cpad, enc_res, coef_img, scale,
                 nonfinite));
  return MIA_OK;
}

extern "C" int mia_cw_init(const float* x, float* w, int64_t len, void* stream) {
  MIA_CHECK_ARG(x && w && len > 0, "bad args");
  MIA_LAUNCH(cw_init_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, x, w, len);
}

extern "C" int mia_cw_tanh(const float* w, float* adv, int64_t len, void* stream) {
  MIA_CHECK_ARG(w && adv && len > 0, "bad args");
  MIA_LAUNCH(cw_tanh_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, w, adv, len);
}

extern "C" int mia_cw_grad(const float* adv, const float* x, const float* g_f, float* g_w,
                           int64_t len, float c, float scale, void* stream) {
  MIA_CHECK_ARG(adv && x && g_f && g_w && len > 0, "bad args");
  MIA_LAUNCH(cw_grad_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, adv, x, g_f, g_w,
             len, c, scale);
}

extern "C" int mia_cw_select(const float* adv, float* best_adv, const float* sq, float* best_l2,
                             const float* f, const float* f0, int N, int64_t plane, float l2_scale,
                             void* stream) {
  MIA_CHECK_ARG(adv && best_adv && sq && best_l2 && f && f0 && N > 0 && plane > 0, "bad args");
  MIA_LAUNCH(cw_select_kernel, dim3(N), dim3(TPB), 0, adv, best_adv, sq, best_l2, f, f0, plane,
             l2_scale);
}

extern "C" int mia_random_start(float* x, const float* x0, const float* u, int64_t len, float e,
                                float lo, float hi, void* stream) {
  MIA_CHECK_ARG(x && x0 && u && len > 0, "bad args");
  MIA_LAUNCH(random_start_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, x, x0, u, len,
             e, lo, hi);
}

extern "C" int mia_sign_project(float* x, const float* x0, const float* g, int64_t len, float a,
                                float e, float lo, float hi, void* stream) {
  MIA_CHECK_ARG(x && x0 && g && len > 0, "bad args");
  MIA_LAUNCH(sign_project_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, x, x0, g, len,
             a, e, lo, hi);
}

extern "C" int mia_adam_step(float* p, const float* g, float* m, float* v, int64_t len, float lr,
                             float beta1, float beta2, float eps, int t, void* stream) {
  MIA_CHECK_ARG(p && g && m && v && len > 0 && t >= 1, "bad args");
  const float bc1 = 1.f - powf(beta1, (float)t);
  const float bc2sqrt = sqrtf(1.f - powf(beta2, (float)t));
  MIA_LAUNCH(adam_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, p, g, m, v, len, lr,
             beta1, beta2, eps, bc1, bc2sqrt);
}

extern "C" int mia_patch_update(float* patch, const float* g, const float* img, const float* mask,
                                float* adv, int64_t len, int64_t shared, float lo, float hi,
                                void* stream) {
  MIA_CHECK_ARG(patch && img && mask && adv && len > 0 && shared >= 0 && lo <= hi, "bad args");
  MIA_CHECK_ARG(!g || !shared, "a gradient step needs a per-image patch (shared = 0)");
  MIA_CHECK_ARG(!shared || len % shared == 0, "len must be a multiple of shared");
  MIA_LAUNCH(patch_update_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, patch, g, img,
             mask, adv, len, shared, lo, hi);
}

extern "C" int mia_pixel_norm(const float* x, float* y, int rows, int cols, float eps,
                              void* stream) {
  MIA_CHECK_ARG(x && y && rows > 0 && cols > 0, "bad args");
  MIA_LAUNCH(pixel_norm_kernel, dim3(rows), dim3(TPB), 0, x, y, cols, eps);
}

extern "C" int mia_truncate(const float* w, const float* mean, float psi, float* out, int rows,
                            int cols, void* stream) {
  MIA_CHECK_ARG(w && mean && out && rows > 0 && cols > 0, "bad args");
  const int64_t len = (int64_t)rows * cols;
  MIA_LAUNCH(truncate_kernel, dim3(blocks_for(len, TPB, 65536)), dim3(TPB), 0, w, mean, psi, out,
             len, cols);
}

extern "C" int mia_repeat(const void* src, void* dst, int64_t bytes, int count, void* stream) {
  MIA_CHECK_ARG(src && dst && bytes > 0 && count > 0, "bad args");
  MIA_LAUNCH(repeat_kernel, dim3(blocks_for(bytes * count, TPB, 65536)), dim3(TPB), 0,
             (const uint8_t*)src, (uint8_t*)dst, bytes, count);
}

// Byte fill on the caller's stream as a kernel of our own (no hipMemsetAsync: the runtime's fill
// path crashed inside rocprofv3 --pmc collection, and a plain kernel is capturable like the rest):
// 16-byte stores when the buffer and length allow, else 4-byte, else bytes.
template <typename V>
__global__ void fill_kernel(V* __restrict__ dst, V v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)mia::TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * mia::TPB)
    dst[i] = v;
}

extern "C" int mia_memset(void* dst, int value, int64_t bytes, void* stream) {
  MIA_CHECK_ARG(dst && bytes >= 0, "bad args");
  if (bytes == 0) return MIA_OK;
  const unsigned b = (unsigned)value & 0xffu, w = b * 0x01010101u;
  const uintptr_t a = (uintptr_t)dst;
  if (a % 16 == 0 && bytes % 16 == 0) {
    const int64_t n = bytes / 16;
    MIA_LAUNCH(fill_kernel<uint4>, dim3(blocks_for(n, mia::TPB, 65536)), dim3(mia::TPB), 0,
               (uint4*)dst, make_uint4(w, w, w, w), n);
  } else if (a % 4 == 0 && bytes % 4 == 0) {
    const int64_t n = bytes / 4;
    MIA_LAUNCH(fill_kernel<unsigned>, dim3(blocks_for(n, mia::TPB, 65536)), dim3(mia::TPB), 0,
               (unsigned*)dst, w, n);
  } else {
    MIA_LAUNCH(fill_kernel<unsigned char>, dim3(blocks_for(bytes, mia::TPB, 65536)),
               dim3(mia::TPB), 0, (unsigned char*)dst, (unsigned char)b, bytes);
  }
  return MIA_OK;
}
