// Implicit-GEMM 3x3 convolution on CDNA4 MFMA (gfx950), NHWC.
//
// One kernel serves every dense contraction of the attack step:
//   * VGG conv + bias + ReLU forward        (code/vgg.py:45-62)
//   * VGG conv input-gradient                (flipped/transposed weights; tap-MSE + ReLU mask fused)
//   * ModulatedConv2d forward [ext]          (modulation = per-(n,ci) A-operand scale, demodulation =
//                                             per-(n,co) epilogue scale: one shared-weight GEMM,
//                                             never N per-sample weight tensors)
//   * up-sampling ModulatedConv2d [ext]      (conv_transpose2d(stride 2) ∘ Blur folded into four
//                                             3x3 phase kernels on the low-res grid, pixel-shuffled
//                                             in the epilogue)
//   * ModulatedConv2d input/style gradient   (dgrad GEMM + Σ_p gx̃·x style reduction in the epilogue)
//
// GEMM view: M = N·H·W output pixels, N-dim = Cout, K = 9·Cin (tap-major, channel-minor).
// Tile BM×BN×BK with 256 threads = 4 waves (WM×WN), wave tile of FM×FN MFMA 16×16 fragments.
//   f16/bf16: v_mfma_f32_16x16x32_{f16,bf16}, BK = 32;  f32: v_mfma_f32_16x16x4_f32 ×4, BK = 16.
// A and B tiles are staged global → registers → LDS (double buffered, one barrier per K-step) in
// 16-byte chunks; each tile row is 64 B (4 chunks), XOR-swizzled so the ds_read_b128 fragment reads
// are bank-conflict-free (chunk' = chunk ^ ((4 − (row>>2)) & 3), derived for the gfx950 b128 lane
// groups {0–3,12–15,20–27},{4–11,16–19,28–31},…).
// The fp32 path permutes K inside a chunk (lane group q holds k = 4q..4q+3 and step s uses k=4q+s
// for both operands), so one ds_read_b128 feeds four 16x16x4 MFMAs.
#include "mia_common.h"

namespace mia {

struct ConvK {
  mia_conv_args a;
  int M, HW, cout_mod, ystride;
};

__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  // Blocks are dealt round-robin over the 8 XCDs; give each XCD a contiguous run of logical tiles
  // so tiles sharing A rows / B columns hit the same L2 (bijective for any nblk).
  if (nblk < 16) return b;
  const int xcd = b & 7, q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

__device__ __forceinline__ int swz(int row) { return (4 - ((row >> 2) & 3)) & 3; }

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

template <typename T, int BM, int BN, int WM, int WN, bool PRO>
__global__ __launch_bounds__(256) void conv3x3_kernel(const ConvK k) {
  typedef typename Vec<T>::type VT;
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = 4 * VEC;
  constexpr int FM = BM / (WM * 16), FN = BN / (WN * 16);
  constexpr int A_CH = BM * 4 / 256, B_CH = BN * 4 / 256;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small");

  __shared__ VT lds[2][(BM + BN) * 4];

  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nbn = (p.Cout + BN - 1) / BN;
  const int nbm = (k.M + BM - 1) / BM;
  const int b = xcd_remap(blockIdx.x, nbm * nbn);
  const int m0 = (b / nbn) * BM, n0 = (b % nbn) * BN;
  const int H = p.H, W = p.W, Cin = p.Cin;

  // ---- staging state -----------------------------------------------------------------------
  const T* __restrict__ X = (const T*)p.x;
  const T* __restrict__ Wt = (const T*)p.w;
  const int kq = tid & 3;
  int a_n[A_CH], a_y[A_CH], a_x[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int j = 0; j < A_CH; ++j) {
    const int m = m0 + (tid >> 2) + 64 * j;
    a_ok[j] = m < k.M;
    const int mm = a_ok[j] ? m : 0;
    a_n[j] = mm / k.HW;
    const int rem = mm - a_n[j] * k.HW;
    a_y[j] = rem / W;
    a_x[j] = rem - a_y[j] * W;
  }
  const T* b_ptr[B_CH];
  bool b_ok[B_CH];
#pragma unroll
  for (int j = 0; j < B_CH; ++j) {
    const int c = n0 + (tid >> 2) + 64 * j;
    b_ok[j] = c < p.Cout;
    b_ptr[j] = Wt + (size_t)(b_ok[j] ? c : 0) * p.Kpad + kq * VEC;
  }
  int tap = (kq * VEC) / Cin, ci = (kq * VEC) - tap * Cin;
  VT ra[A_CH], rb[B_CH];

  auto load_tile = [&](int kb) {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      VT v = {};
      if (a_ok[j] && tap < 9) {
        const int ty = tap / 3;
        const int yy = a_y[j] + ty - 1, xx = a_x[j] + (tap - 3 * ty) - 1;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
          v = *(const VT*)(X + ((size_t)(a_n[j] * H + yy) * W + xx) * Cin + ci);
          if constexpr (PRO) {
            const float* sc = p.in_scale ? p.in_scale + (size_t)a_n[j] * Cin + ci : nullptr;
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
              float f = apply_act(to_f(v[e]), p.act_in);
              if (sc) f *= sc[e];
              v[e] = from_f<T>(f);
            }
          }
        }
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      VT v = {};
      if (b_ok[j]) v = *(const VT*)(b_ptr[j] + (size_t)kb * BK);
      rb[j] = v;
    }
  };
  auto advance = [&]() {
    ci += BK;
    while (ci >= Cin) { ci -= Cin; ++tap; }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A_CH; ++j) {
      const int r = (tid >> 2) + 64 * j;
      lds[buf][r * 4 + (kq ^ swz(r))] = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_CH; ++j) {
      const int r = (tid >> 2) + 64 * j;
      lds[buf][(BM + r) * 4 + (kq ^ swz(r))] = rb[j];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.Kpad / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int frow = lane & 15, fq = lane >> 4;
  const int fsw = fq ^ swz(frow);
  for (int kb = 0; kb < nk; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nk) {
      advance();
      load_tile(kb + 1);
    }
    VT af[FM], bf[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = lds[cur][(wm * FM * 16 + 16 * i + frow) * 4 + fsw];
#pragma unroll
    for (int j = 0; j < FN; ++j) bf[j] = lds[cur][(BM + wn * FN * 16 + 16 * j + frow) * 4 + fsw];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma_chunk<T>(af[i], bf[j], acc[i][j]);
    if (kb + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
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

template <typename T, int BM, int BN, int WM, int WN>
static int launch_tile(const ConvK& k, hipStream_t st) {
  const int nbm = (k.M + BM - 1) / BM, nbn = (k.a.Cout + BN - 1) / BN;
  const int nblk = nbm * nbn;
  const bool pro = k.a.in_scale != nullptr || k.a.act_in != MIA_ACT_NONE;
  if (pro)
    hipLaunchKernelGGL((conv3x3_kernel<T, BM, BN, WM, WN, true>), dim3(nblk), dim3(256), 0, st, k);
  else
    hipLaunchKernelGGL((conv3x3_kernel<T, BM, BN, WM, WN, false>), dim3(nblk), dim3(256), 0, st, k);
  return check_launch("conv3x3");
}

template <typename T>
static int launch_conv(const ConvK& k, hipStream_t st) {
  if (k.a.Cout <= 64) return launch_tile<T, 128, 64, 2, 2>(k, st);
  return launch_tile<T, 128, 128, 2, 2>(k, st);
}

static int bk_for(int dtype) { return dtype == MIA_F32 ? 16 : 32; }
static int vec_for(int dtype) { return dtype == MIA_F32 ? 4 : 8; }

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
  MIA_CHECK_ARG(a.Cin % vec_for(dtype) == 0, "Cin must be a multiple of the 16-byte vector");
  MIA_CHECK_ARG(a.Kpad % bk_for(dtype) == 0 && a.Kpad >= 9 * a.Cin, "Kpad must be mia_conv_kpad()");
  MIA_CHECK_ARG(!a.shuffle_out || a.Cout % 4 == 0, "shuffle_out needs Cout % 4 == 0");
  MIA_CHECK_ARG(!a.sdot || a.aux_x, "sdot needs aux_x");
  MIA_CHECK_ARG(!a.tap_a || a.tap_t, "tap_a needs tap_t");
  MIA_CHECK_ARG(!a.shuffle_out || !(a.tap_a || a.mask_a || a.sdot), "aux inputs need un-shuffled output");
  MIA_CHECK_ARG((int64_t)a.N * a.H * a.W < (1LL << 31), "too many pixels");
  ConvK k;
  k.a = a;
  k.M = a.N * a.H * a.W;
  k.HW = a.H * a.W;
  k.cout_mod = a.shuffle_out ? a.Cout / 4 : a.Cout;
  k.ystride = a.y_cstride > 0 ? a.y_cstride : k.cout_mod;
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
