// Implicit-GEMM 3x3 convolution on CDNA4 MFMA (gfx950), NHWC.
//
// One kernel serves every dense contraction of the attack step:
//   * VGG conv + bias + ReLU forward        (code/vgg.py:45-62)
//   * VGG conv input-gradient                (flipped/transposed weights; tap-MSE + ReLU mask fused)
//   * ModulatedConv2d forward [ext]          (modulation = per-(n,ci) A-operand scale applied to the
//                                             MFMA fragments, demodulation = per-(n,co) epilogue
//                                             scale: one shared-weight GEMM, never N per-sample
//                                             weight tensors)
//   * up-sampling ModulatedConv2d [ext]      (conv_transpose2d(stride 2) ∘ Blur folded into four
//                                             3x3 phase kernels on the low-res grid, pixel-shuffled
//                                             in the epilogue)
//   * ModulatedConv2d input/style gradient   (dgrad GEMM + Σ_p gx̃·x style reduction in the epilogue)
//
// GEMM view: M = N·H·W output pixels, N-dim = Cout, K = 9·Cin (tap-major, channel-minor).
// Block tile BM×BN×BK, 256 threads = 4 waves (2×2), each wave FM×FN MFMA 16×16 fragments.
//   f16/bf16: v_mfma_f32_16x16x32_{f16,bf16}, BK = 64;  f32: v_mfma_f32_16x16x4_f32, BK = 32.
// Every tile row (one pixel's or one output channel's K-slice) is 128 B = 8 chunks of 16 B.
//
// Staging: both operands go global → LDS by LDS-DMA (global_load_lds_dwordx4), a 2-stage ring:
// the loads of K-step k+1 are issued before the MFMAs of step k and retired by the barrier at its
// end. The im2col gather is done by the per-lane SOURCE address (one pixel row + tap offset);
// lanes whose tap falls outside the image (or whose row is beyond M / Cout) read a 16-byte zero
// vector instead, so the loop has no branches. LDS-DMA writes lane-linearly, so the bank
// swizzle (chunk' = chunk ^ ((row>>1)&7), conflict-free for the ds_read_b128 fragment lane groups
// on 128-B rows) is applied by permuting which chunk each lane fetches (guide rule 21).
// The modulation prologue x̃ = act(x)·s[n][ci] is applied to A fragments after ds_read, with s
// held in an LDS table for the (≤ 9) images a tile spans.
#include <algorithm>
#include <type_traits>

#include "mia_common.h"

namespace mia {

struct ConvK {
  mia_conv_args a;
  int M, HW, cout_mod, ystride, log2cin, n_first_max;
};

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

__device__ __attribute__((aligned(16))) uint4 g_zero16[4];  // zero source for masked DMA lanes

__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  // Blocks are dealt round-robin over the 8 XCDs; give each XCD a contiguous run of logical tiles
  // so tiles sharing A rows / B columns hit the same L2 (bijective for any nblk).
  if (nblk < 16) return b;
  const int xcd = b & 7, q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

__device__ __forceinline__ int fsw(int row) { return (row >> 1) & 7; }

template <typename T>
__device__ __forceinline__ f32x4 mfma_chunk(const typename Vec<T>::type& a,
                                            const typename Vec<T>::type& b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mfma_chunk<_Float16>(const f16x8& a, const f16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma_chunk<__bf16>(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma_chunk<float>(const f32x4& a, const f32x4& b, f32x4 c) {
  // fp32: lane group q holds k = 4q..4q+3 of the chunk; step s uses k = 4q+s for both operands
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == MIA_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == MIA_ACT_LRELU_S2) return lrelu_s2(v);
  return v;
}

// x̃ = act(x)·s on a 16-byte fragment; for LRELU the table already holds s·√2, and
// leaky_relu(x, 0.2) = max(x, 0.2·x).
template <typename T>
__device__ __forceinline__ void modulate(typename Vec<T>::type& v, const typename Vec<T>::type& s,
                                         bool lrelu) {
  if constexpr (std::is_same<T, _Float16>::value) {
    if (lrelu) v = __builtin_elementwise_max(v, v * (_Float16)0.2f);
    v = v * s;
  } else {
#pragma unroll
    for (int e = 0; e < Vec<T>::N; ++e) {
      float f = (float)v[e];
      if (lrelu) f = fmaxf(f, 0.2f * f);
      v[e] = (T)(f * (float)s[e]);
    }
  }
}

constexpr int ROWB = 128;  // bytes per tile row (one K-step slice)

template <typename T, int BM, int BN, bool PRO>
__global__ __launch_bounds__(256, 2) void conv3x3_kernel(const ConvK k) {
  typedef typename Vec<T>::type VT;
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = ROWB / (int)sizeof(T);
  constexpr int FM = BM / 32, FN = BN / 32;         // 2×2 waves
  constexpr int A_INS = BM / 32, B_INS = BN / 32;   // 1-KB DMA pieces per wave per K-step
  constexpr int STAGE = (BM + BN) * ROWB;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nbn = (p.Cout + BN - 1) / BN;
  const int nbm = (k.M + BM - 1) / BM;
  const int b = xcd_remap(blockIdx.x, nbm * nbn);
  const int m0 = (b / nbn) * BM, n0 = (b % nbn) * BN;
  const int H = p.H, W = p.W, Cin = p.Cin;
  const int lc = k.log2cin;

  const T* __restrict__ X = (const T*)p.x;
  const T* __restrict__ Wt = (const T*)p.w;
  const T* zero = (const T*)g_zero16;

  // ---- per-lane DMA source state -----------------------------------------------------------
  int a_base[A_INS], a_koff[A_INS], a_mask[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wid * A_INS + j) * 8 + (lane >> 3);
    a_koff[j] = ((lane & 7) ^ fsw(row)) * VEC;
    const int m = m0 + row;
    int msk = 0, base = 0;
    if (m < k.M) {
      const int n = m / k.HW;
      const int rem = m - n * k.HW;
      const int y = rem / W, x = rem - (rem / W) * W;
      base = ((n * H + y) * W + x) * Cin;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) msk |= 1 << t;
      }
    }
    a_base[j] = base;
    a_mask[j] = msk;
  }
  const T* b_src[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wid * B_INS + j) * 8 + (lane >> 3);
    const int c = n0 + row;
    b_src[j] = c < p.Cout ? Wt + (size_t)c * p.Kpad + ((lane & 7) ^ fsw(row)) * VEC : nullptr;
  }

  auto issue = [&](int kb, int st) {
    char* sa = smem + st * STAGE;
    char* sb = sa + BM * ROWB;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int kk = kb * BK + a_koff[j];
      const int tap = kk >> lc;
      const int ci = kk & (Cin - 1);
      const int dy = (tap * 11) >> 5;  // tap / 3 for tap < 9
      const int dx = tap - 3 * dy;
      const T* src = ((a_mask[j] >> tap) & 1)
                         ? X + (a_base[j] + ((dy - 1) * W + (dx - 1)) * Cin + ci)
                         : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(sa + (wid * A_INS + j) * 1024), 16,
                                       0, 0);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const T* src = b_src[j] ? b_src[j] + (size_t)kb * BK : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(sb + (wid * B_INS + j) * 1024), 16,
                                       0, 0);
    }
  };

  // ---- modulation table (PRO): s[n][ci] (·√2 for lrelu inputs) for the images of this tile ----
  const int n_first = m0 / k.HW;
  T* stab = (T*)(smem + 2 * STAGE);
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;
  int a_nl[FM];
  if constexpr (PRO) {
    const int n_last = (min(m0 + BM, k.M) - 1) / k.HW;
    const int cnt = (n_last - n_first + 1) * Cin;
    const float mul = lrelu_in ? SQRT2 : 1.f;
    for (int i = tid; i < cnt; i += 256) {
      const float sv = p.in_scale ? p.in_scale[(size_t)n_first * Cin + i] : 1.f;
      stab[i] = from_f<T>(sv * mul);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = min(m0 + wm * FM * 16 + 16 * i + (lane & 15), k.M - 1);
      a_nl[i] = (m / k.HW - n_first) * Cin;
    }
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.Kpad / BK;
  issue(0, 0);
  __syncthreads();
  const int frow = lane & 15, fq = lane >> 4;
  for (int kb = 0; kb < nk; ++kb) {
    const int st = kb & 1;
    if (kb + 1 < nk) issue(kb + 1, st ^ 1);
    const char* sa = smem + st * STAGE;
    const char* sb = sa + BM * ROWB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + fq;
      VT af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * FM * 16 + 16 * i + frow;
        af[i] = *(const VT*)(sa + row * ROWB + ((ch ^ fsw(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * FN * 16 + 16 * j + frow;
        bf[j] = *(const VT*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
      }
      if constexpr (PRO) {
        const int ci = (kb * BK + ch * VEC) & (Cin - 1);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const VT sv = *(const VT*)(stab + a_nl[i] + ci);
          modulate<T>(af[i], sv, lrelu_in);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma_chunk<T>(af[i], bf[j], acc[i][j]);
    }
    __syncthreads();  // retires the DMA of step kb+1 (vmcnt(0)) and frees stage st for kb+2
  }

  // ---- epilogue ---------------------------------------------------------------------------
  const int Cout = p.Cout;
  const int row_base = m0 + wm * FM * 16 + fq * 4;
  const int col_base = n0 + wn * FN * 16 + frow;

  if (p.sdot) {
    const T* AX = (const T*)p.aux_x;
    const int last = min(m0 + BM, k.M) - 1;
    const bool single = (m0 / k.HW) == (last / k.HW);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = col_base + 16 * j;
      float part = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = row_base + 16 * i + r;
          if (row < k.M && col < Cout) {
            const float xv = apply_act(to_f(AX[(size_t)row * Cout + col]), p.act_aux);
            const float c = acc[i][j][r] * xv;
            if (single) part += c;
            else atomicAdd(&p.sdot[(size_t)(row / k.HW) * Cout + col], c);
          }
        }
      if (single) {
        part += __shfl_xor(part, 16, 64);
        part += __shfl_xor(part, 32, 64);
        if (fq == 0 && col < Cout) atomicAdd(&p.sdot[(size_t)(m0 / k.HW) * Cout + col], part);
      }
    }
  }
  if (!p.y) return;

  T* __restrict__ Y = (T*)p.y;
  const T* TA = (const T*)p.tap_a;
  const T* TT = (const T*)p.tap_t;
  const T* MA = (const T*)p.mask_a;
  const int Ho = p.shuffle_out ? 2 * H : H, Wo = p.shuffle_out ? 2 * W : W;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row_base + 16 * i + r;
      if (row >= k.M) continue;
      const int n = row / k.HW;
      const int pix = row - n * k.HW;
      const int y = pix / W, x = pix - (pix / W) * W;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = col_base + 16 * j;
        if (col >= Cout) continue;
        int cm = col, yo = y, xo = x;
        if (p.shuffle_out) {
          const int ph = col / k.cout_mod;
          cm = col - ph * k.cout_mod;
          yo = 2 * y + (ph >> 1);
          xo = 2 * x + (ph & 1);
        }
        const size_t off = ((size_t)(n * Ho + yo) * Wo + xo) * k.ystride + cm;
        const size_t aoff = (size_t)row * Cout + col;
        float v = acc[i][j][r];
        if (p.out_scale) v *= p.out_scale[(size_t)n * k.cout_mod + cm];
        if (p.noise) v += p.noise_w * p.noise[yo * Wo + xo];
        if (p.bias) v += p.bias[cm];
        if (TA) v += p.tap_coef * (to_f(TA[aoff]) - to_f(TT[aoff]));
        if (MA && !(to_f(MA[aoff]) > 0.f)) v = 0.f;
        v = apply_act(v, p.act_out);
        if (p.accumulate) v += to_f(Y[off]);
        Y[off] = from_f<T>(v);
      }
    }
}

template <typename T, int BM, int BN, bool PRO>
static int launch_tile(const ConvK& k, hipStream_t st) {
  const int nbm = (k.M + BM - 1) / BM, nbn = (k.a.Cout + BN - 1) / BN;
  const int nblk = nbm * nbn;
  size_t lds = 2 * (BM + BN) * ROWB;
  if (PRO) lds += (size_t)k.n_first_max * k.a.Cin * sizeof(T);
  auto fn = conv3x3_kernel<T, BM, BN, PRO>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    attr_set = true;
  }
  hipLaunchKernelGGL(fn, dim3(nblk), dim3(256), lds, st, k);
  return check_launch("conv3x3");
}

template <typename T, bool PRO>
static int launch_bn(const ConvK& k, hipStream_t st) {
  if (k.a.Cout <= 64) return launch_tile<T, 128, 64, PRO>(k, st);
  return launch_tile<T, 128, 128, PRO>(k, st);
}

template <typename T>
static int launch_conv(const ConvK& k, hipStream_t st) {
  const bool pro = k.a.in_scale != nullptr || k.a.act_in != MIA_ACT_NONE;
  return pro ? launch_bn<T, true>(k, st) : launch_bn<T, false>(k, st);
}

static int bk_for(int dtype) { return dtype == MIA_F32 ? 32 : 64; }

}  // namespace mia

using namespace mia;

extern "C" int mia_conv_kpad(int cin, int dtype) {
  const int bk = bk_for(dtype);
  return (9 * cin + bk - 1) / bk * bk;
}

extern "C" int mia_conv3x3(const mia_conv_args* args, int dtype, void* stream) {
  MIA_CHECK_ARG(args != nullptr, "null args");
  const mia_conv_args& a = *args;
  MIA_CHECK_ARG(a.x && a.w, "x and w are required");
  MIA_CHECK_ARG(a.N > 0 && a.H > 0 && a.W > 0 && a.Cin > 0 && a.Cout > 0, "bad shape");
  MIA_CHECK_ARG(dtype == MIA_F32 || dtype == MIA_F16 || dtype == MIA_BF16, "bad dtype");
  const int vec = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(a.Cin >= vec && (a.Cin & (a.Cin - 1)) == 0,
                "Cin must be a power of two ≥ the 16-byte vector");
  MIA_CHECK_ARG(a.Kpad == mia_conv_kpad(a.Cin, dtype), "Kpad must be mia_conv_kpad()");
  MIA_CHECK_ARG(!a.shuffle_out || a.Cout % 4 == 0, "shuffle_out needs Cout % 4 == 0");
  MIA_CHECK_ARG(!a.sdot || a.aux_x, "sdot needs aux_x");
  MIA_CHECK_ARG(!a.tap_a || a.tap_t, "tap_a needs tap_t");
  MIA_CHECK_ARG(!a.shuffle_out || !(a.tap_a || a.mask_a || a.sdot),
                "aux inputs need un-shuffled output");
  MIA_CHECK_ARG((int64_t)a.N * a.H * a.W * a.Cin < (1LL << 31), "input too large for 32-bit offsets");
  MIA_CHECK_ARG(a.in_scale == nullptr || a.Cin <= 2048, "modulated Cin ≤ 2048");
  ConvK k;
  k.a = a;
  k.M = a.N * a.H * a.W;
  k.HW = a.H * a.W;
  k.cout_mod = a.shuffle_out ? a.Cout / 4 : a.Cout;
  k.ystride = a.y_cstride > 0 ? a.y_cstride : k.cout_mod;
  int lc = 0;
  while ((1 << lc) < a.Cin) ++lc;
  k.log2cin = lc;
  k.n_first_max = std::min(a.N, (128 + k.HW - 1) / k.HW + 1);
  MIA_CHECK_ARG(k.ystride >= k.cout_mod, "y_cstride < Cout");
  hipStream_t st = (hipStream_t)stream;
  MIA_DISPATCH_DTYPE(dtype, T, return launch_conv<T>(k, st));
  return MIA_OK;
}

extern "C" int mia_modconv_fwd(const void* x, const void* w, void* pre, int N, int H, int W,
                               int Cin, int Cout, int Kpad, int act_in, const float* style,
                               const float* demod, const float* noise, float noise_w,
                               const float* bias, int upsample, int dtype, void* stream) {
  mia_conv_args a = {};
  a.x = x; a.w = w; a.y = pre;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = upsample ? 4 * Cout : Cout; a.Kpad = Kpad;
  a.act_in = act_in; a.in_scale = style; a.out_scale = demod; a.noise = noise; a.noise_w = noise_w;
  a.bias = bias; a.shuffle_out = upsample;
  return mia_conv3x3(&a, dtype, stream);
}

extern "C" int mia_modconv_bwd(const void* gy, const void* w_t, void* gx, int N, int H, int W,
                               int Cin_g, int Cout_g, int Kpad, const void* x_fwd, int act_x,
                               const float* style, float* sdot, int dtype, void* stream) {
  mia_conv_args a = {};
  a.x = gy; a.w = w_t; a.y = gx;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin_g; a.Cout = Cout_g; a.Kpad = Kpad;
  a.out_scale = style; a.aux_x = x_fwd; a.act_aux = act_x; a.sdot = sdot;
  return mia_conv3x3(&a, dtype, stream);
}

extern "C" int mia_vgg_conv_relu_fwd(const void* x, const void* w, const float* bias, void* y,
                                     int N, int H, int W, int Cin, int Cout, int Kpad, int dtype,
                                     void* stream) {
  mia_conv_args a = {};
  a.x = x; a.w = w; a.y = y; a.bias = bias; a.act_out = MIA_ACT_RELU;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.Kpad = Kpad;
  return mia_conv3x3(&a, dtype, stream);
}

extern "C" int mia_vgg_conv_dgrad(const void* g, const void* w_t, void* gx, int N, int H, int W,
                                  int Cin_g, int Cout_g, int Kpad, const void* tap_a,
                                  const void* tap_t, float tap_coef, const void* mask_a,
                                  int dtype, void* stream) {
  mia_conv_args a = {};
  a.x = g; a.w = w_t; a.y = gx;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin_g; a.Cout = Cout_g; a.Kpad = Kpad;
  a.tap_a = tap_a; a.tap_t = tap_t; a.tap_coef = tap_coef; a.mask_a = mask_a;
  return mia_conv3x3(&a, dtype, stream);
}
