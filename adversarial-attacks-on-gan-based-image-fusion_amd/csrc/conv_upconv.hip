// Up-sampling StyledConv forward as ONE halo-tiled MFMA kernel (fp32 / fp16 / bf16): the modulated
// conv_transpose2d(stride 2) of rosinality ModulatedConv2d(upsample=True) [ext], reached through
// net.decoder (code/attack/attack_main2.py:619-621). Blur, demod, noise, bias and the activation
// follow in mia_upconv_blur_fwd.
//
// Sub-pixel form (layouts.upconv_subpixel_matrices): T[2m+p] = Σ_j x[m−j]·W[p+2j], so output phase
// (py, px) at input position (y, x) reads the input at offsets (−jy, −jx), jy ∈ {0,1} if py = 0
// else {0} (same for x): 4 + 2 + 2 + 1 = 9 (offset, phase) products per input pixel — the MACs of
// the transposed conv, no zero taps. The generic kernel runs the 4 phases as im2col GEMMs that
// gather every input pixel once per tap; here a block owns an 8×16 INPUT patch × 64 output
// channels × all 4 phases:
//   * per 64-channel block the (8+1)×(16+1) input halo is DMA'd into LDS once and read by all
//     9 products;
//   * a K-step is (offset, two phases sharing it): (0,0)·{p0,p1}, (0,0)·{p2,p3}, (0,−1)·{p0,p2},
//     (−1,0)·{p0,p1}, (−1,−1)·{p0}; each step reads the offset's A fragments once for both
//     phases, so the LDS reads per MFMA equal the stride-1 halo kernel's (0.5);
//   * weights: the packed [Cin/BK][5][2][Cout][BK] tensor (layouts.upconv_halo_matrix; BK = the
//     channels of one 128-B row: 64 for 2-byte types, 32 for fp32), one 16-KB stage (2 slots × 64
//     channels × 128 B) per K-step through a 2-stage LDS-DMA ring;
//   * waves split DMA roles as in conv_halo.hip (2 weight waves, 2 halo waves, vmcnt retires in
//     issue order); the next channel block's halo streams during steps 0–3;
//   * accumulators: 4 phases × 4 patch rows × 2 channel fragments per wave (128 VGPRs); the
//     2-byte epilogue exchanges fragment pairs (v_permlane16_swap) for 16-byte stores into T, the
//     fp32 one stores each lane's 4 consecutive channels as one 16-byte vector.
// The phase positions on the last row / column of T's phase grids (y = R or x = R; they exist for
// the even phases only) go to the generic kernel as four one-row / one-column groups.
//
// DG (input-gradient mode): the same kernel computes the input gradient of a stride-2, pad-1 3×3
// conv (the e4e encoder's strided convs): gin[2i] = g[i]·W[1], gin[2i+1] = g[i]·W[2] + g[i+1]·W[0]
// per axis — the transposed conv mirrored: offsets (0, +1) instead of (0, −1), output phase
// 1 − p, weights flipped (layouts.s2_dgrad_halo_matrix). Every output row 2i + q of an input
// patch lies inside the output, so no edge launch; the epilogue applies the slope mask of the
// layer below (PReLU / LeakyReLU backward) and optionally accumulates.
#include "conv_common.h"

namespace mia {

struct HaloUp {
  static constexpr int PH = 8, PW = 16, WM = 2, WN = 2, FM = 4, FN = 2, NW = 4, NT = 256;
  static constexpr int BN = WN * FN * 16;                       // output channels per block
  static constexpr int HSIDE = PW + 1, HROWS = (PH + 1) * HSIDE;  // 153 halo pixels
  static constexpr int HPIECES = (HROWS + 7) / 8;               // 20 pieces of 8 rows
  static constexpr int HBUF = HPIECES * 8 * ROWB;
  static constexpr int BROWS = 2 * BN, BSTAGE = BROWS * ROWB;   // two phase slots per K-step
  static constexpr int BWAVES = 2, HWAVES = 2;
  static constexpr int B_INS = BROWS / (8 * BWAVES);            // 8 weight pieces per B-wave
  static constexpr int H_INS = (HPIECES + HWAVES - 1) / HWAVES; // 10 halo pieces per H-wave
  static constexpr int HPS = (H_INS + 3) / 4;                   // issued during steps 0–3
  static constexpr int NSTEP = 5, STAGES = 2;
  static_assert(B_INS * 8 * BWAVES == BROWS && H_INS * HWAVES == HPIECES, "");
};

// K-step st: offset (jy, jx) and the phases of its two weight slots (−1: none)
__device__ __forceinline__ constexpr int up_jy(int st) { return st == 3 || st == 4 ? 1 : 0; }
__device__ __forceinline__ constexpr int up_jx(int st) { return st == 2 || st == 4 ? 1 : 0; }
__device__ __forceinline__ constexpr int up_phase(int st, int slot) {
  return st == 0 ? slot : st == 1 ? 2 + slot : st == 2 ? 2 * slot : st == 3 ? slot : (slot ? -1 : 0);
}

struct UpK {
  const void* x;
  const void* w;  // packed [Cin/BK][5][2][Cout][BK]
  void* t;        // (N, 2R+1, 2R+1, Cout); DG: (N, 2R, 2R, Cout)
  const float* style;
  const void* mask_a;       // DG: (N, 2R, 2R, Cout) or NULL
  const float* mask_slope;  // DG: [Cout] or NULL (→ 0)
  int N, R, Cin, Cout, act_in, nbn, nblk, accumulate;
};

template <typename T, bool PRO, bool DG>
__global__ __launch_bounds__(256, 2) void upconv_halo_kernel(const UpK k) {
  typedef HaloUp TL;
  typedef typename Vec<T>::type VT;
  constexpr int VEC = Vec<T>::N, BK = ROWB / (int)sizeof(T);  // elements per chunk / per row
  constexpr int FM = TL::FM, FN = TL::FN, WN = TL::WN, BN = TL::BN, PH = TL::PH, PW = TL::PW;
  constexpr int HSIDE = TL::HSIDE, HROWS = TL::HROWS, HBUF = TL::HBUF, BSTAGE = TL::BSTAGE;
  constexpr int B_INS = TL::B_INS, H_INS = TL::H_INS, HPS = TL::HPS, BWAVES = TL::BWAVES;
  constexpr int HWAVES = TL::HWAVES;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                    // 2 halo buffers
  char* const bring = smem + 2 * HBUF;        // weight ring
  T* const stab = (T*)(bring + TL::STAGES * BSTAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int R = k.R, Cin = k.Cin, Cout = k.Cout;
  const int bl = xcd_remap(blockIdx.x, k.nblk);
  const int mt = bl / k.nbn, n0 = (bl % k.nbn) * BN;
  const int ptx = R / PW, pty = R / PH;
  const int x0 = (mt % ptx) * PW;
  const int y0 = ((mt / ptx) % pty) * PH;
  const int n = mt / (ptx * pty);
  const T* __restrict__ X = (const T*)k.x;
  const T* __restrict__ Wt = (const T*)k.w;
  const T* zero = (const T*)g_zero16;
  const bool bwave = wid < BWAVES;
  const int hw = wid - BWAVES;

  // per-lane DMA sources: B-wave w owns weight rows (w·B_INS + j)·8 + lane/8 = slot·64 + channel;
  // H-wave hw owns halo pieces hw + 2·j
  const T* src[H_INS];
#pragma unroll
  for (int j = 0; j < H_INS; ++j) {
    src[j] = nullptr;
    if (bwave) {
      if (j < B_INS) {
        const int row = (wid * B_INS + j) * 8 + (lane >> 3);
        const int slot = row / BN, c = n0 + row % BN;
        src[j] = Wt + ((size_t)slot * Cout + c) * BK + ((lane & 7) ^ fsw(row)) * VEC;
      }
    } else {
      const int hr = (hw + HWAVES * j) * 8 + (lane >> 3);
      const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
      const int y = y0 + hy - (DG ? 0 : 1), x = x0 + hx - (DG ? 0 : 1);
      if (hr < HROWS && y >= 0 && y < R && x >= 0 && x < R)
        src[j] = X + ((size_t)(n * R + y) * R + x) * Cin + ((lane & 7) ^ fsw(hr)) * VEC;
    }
  }
  const int ncb = Cin / BK, nk = TL::NSTEP * ncb;
  const size_t wstep = (size_t)2 * Cout * BK;  // elements per K-step of the packed weights

  auto issue_b = [&](int s, int stg) {
    char* dst = bring + stg * BSTAGE;
#pragma unroll
    for (int j = 0; j < B_INS; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(src[j] + s * wstep),
                                       (lptr_t)(dst + (wid * B_INS + j) * 1024), 16, 0, 0);
  };
  auto issue_h = [&](int cb, int j, int buf) {
    const T* a = src[j] ? src[j] + cb * BK : zero;
    __builtin_amdgcn_global_load_lds((gptr_t)a,
                                     (lptr_t)(hbuf + buf * HBUF + (hw + HWAVES * j) * 1024), 16,
                                     0, 0);
  };

  const bool lrelu_in = k.act_in == MIA_ACT_LRELU_S2;
  if constexpr (PRO) {
    const float mul = lrelu_in ? SQRT2 : 1.f;
    for (int i = tid; i < Cin; i += TL::NT) {
      const float sv = k.style ? k.style[(size_t)n * Cin + i] : 1.f;
      stab[i] = from_f<T>(sv * mul);
    }
  }
  if (bwave) {
    issue_b(0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < H_INS; ++j) issue_h(0, j, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[4][FM][FN];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fq = lane >> 4;
  for (int cb = 0; cb < ncb; ++cb) {
    const char* ha = hbuf + (cb & 1) * HBUF;
#pragma unroll
    for (int st = 0; st < TL::NSTEP; ++st) {
      const int s = cb * TL::NSTEP + st;
      const int stg = s & 1;
      const char* sb = bring + stg * BSTAGE;
      if (bwave && s + 1 < nk) issue_b(s + 1, stg ^ 1);
      const int jy = up_jy(st), jx = up_jx(st);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = h * 4 + fq;
        VT af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int hr = DG ? (wm * FM + i + jy) * HSIDE + frow + jx
                            : (wm * FM + i + 1 - jy) * HSIDE + frow + 1 - jx;
          af[i] = *(const VT*)(ha + hr * ROWB + ((ch ^ fsw(hr)) << 4));
        }
        if constexpr (PRO) {
          const VT sv = *(const VT*)(stab + cb * BK + ch * VEC);
#pragma unroll
          for (int i = 0; i < FM; ++i) modulate<T>(af[i], sv, lrelu_in);
        }
#pragma unroll
        for (int slot = 0; slot < 2; ++slot) {
          const int ph = up_phase(st, slot);
          if (ph < 0) continue;
          VT bf[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int row = slot * BN + wn * FN * 16 + 16 * j + frow;
            bf[j] = *(const VT*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[ph][i][j] = mfma_chunk<T>(bf[j], af[i], acc[ph][i][j]);  // D[channel][pixel]
        }
        if (h == 0 && !bwave && st < 4 && cb + 1 < ncb) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < HPS; ++q) {
            const int j = st * HPS + q;
            if (j < H_INS) issue_h(cb + 1, j, (cb + 1) & 1);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // B-wave: step s+1's weights landed; H-wave: the next block's halo before its first step
      if (bwave) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (st == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage stg done
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- epilogue: phase (py, px) of input position (y, x) → T(2y+py, 2x+px) ----------------------
  T* __restrict__ Y = (T*)k.t;
  const int TS = DG ? 2 * R : 2 * R + 1, lrow = lane >> 4;
  if constexpr (sizeof(T) == 4) {
    // D[channel][pixel]: lane (frow, fq) holds channels 4·fq … 4·fq+3 of fragment j for pixel
    // x0 + frow — one 16-byte vector per (phase, row, fragment)
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int py = ph >> 1, px = ph & 1;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ty = 2 * (y0 + wm * FM + i) + (DG ? 1 - py : py);
        const int tx = 2 * (x0 + frow) + (DG ? 1 - px : px);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c = n0 + wn * FN * 16 + 16 * j + 4 * fq;
          const size_t off = ((size_t)(n * TS + ty) * TS + tx) * Cout + c;
          f32x4 v = acc[ph][i][j];
          if constexpr (DG) {
            if (k.mask_a) {
              const f32x4 m = *(const f32x4*)((const float*)k.mask_a + off);
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float sl = k.mask_slope ? k.mask_slope[c + e] : 0.f;
                v[e] = m[e] > 0.f ? v[e] : sl * v[e];
              }
            }
            if (k.accumulate) {
              const f32x4 o = *(const f32x4*)((const float*)Y + off);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += o[e];
            }
          }
          *(f32x4*)((float*)Y + off) = v;
        }
      }
    }
    return;
  } else {
  typedef T t2 __attribute__((ext_vector_type(2)));
  float msl[8];
  if constexpr (DG) {
    const int c = n0 + wn * FN * 16 + 16 * (lrow & 1) + 8 * (lrow >> 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) msl[e] = k.mask_slope ? k.mask_slope[c + e] : 0.f;
  }
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) {
    const int py = ph >> 1, px = ph & 1;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ty = 2 * (y0 + wm * FM + i) + (DG ? 1 - py : py);
      const int tx = 2 * (x0 + frow) + (DG ? 1 - px : px);
      unsigned a[2], b[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const t2 ta = {(T)acc[ph][i][0][2 * h], (T)acc[ph][i][0][2 * h + 1]};
        const t2 tb = {(T)acc[ph][i][1][2 * h], (T)acc[ph][i][1][2 * h + 1]};
        const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, ta),
                                                        __builtin_bit_cast(unsigned, tb), false,
                                                        false);
        a[h] = r[0];
        b[h] = r[1];
      }
      // lane row lrow now holds channels [16·(lrow & 1) + 8·(lrow >> 1), +8) of the wave's 32
      const int c = n0 + wn * FN * 16 + 16 * (lrow & 1) + 8 * (lrow >> 1);
      const size_t off = ((size_t)(n * TS + ty) * TS + tx) * Cout + c;
      if constexpr (DG) {
        if (k.mask_a || k.accumulate) {  // 8 channels of this lane: mask, accumulate, repack
          typedef typename Vec<T>::type VT8;
          VT8 v = __builtin_bit_cast(VT8, make_uint4(a[0], a[1], b[0], b[1]));
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = (float)v[e];
          if (k.mask_a) {
            const VT8 m = *(const VT8*)((const T*)k.mask_a + off);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = (float)m[e] > 0.f ? f[e] : msl[e] * f[e];
          }
          if (k.accumulate) {
            const VT8 o = *(const VT8*)(Y + off);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += (float)o[e];
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (T)f[e];
          *(VT8*)(Y + off) = v;
          continue;
        }
      }
      *(uint4*)(Y + off) = make_uint4(a[0], a[1], b[0], b[1]);
    }
  }
  }  // 2-byte epilogue
}

template <typename T, bool PRO, bool DG = false>
static int launch_upconv_halo(UpK& k, hipStream_t st) {
  typedef HaloUp TL;
  k.nbn = k.Cout / TL::BN;
  k.nblk = k.N * (k.R / TL::PH) * (k.R / TL::PW) * k.nbn;
  size_t lds = 2 * (size_t)TL::HBUF + (size_t)TL::STAGES * TL::BSTAGE;
  if (PRO) lds += (size_t)k.Cin * sizeof(T);
  if (lds > 160 * 1024) return set_error("upconv_halo: LDS budget exceeded");
  auto fn = upconv_halo_kernel<T, PRO, DG>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    attr_set = true;
  }
  hipLaunchKernelGGL(fn, dim3(k.nblk), dim3(TL::NT), lds, st, k);
  return check_launch("upconv_halo");
}

bool upconv_halo_eligible(int dtype, int R, int Cin, int Cout) {
  const char* e = getenv("MIA_UPCONV_HALO");  // tuning / A-B switch: 0 = generic phase GEMMs
  if (e && atoi(e) == 0) return false;
  return R % 16 == 0 && Cin % 64 == 0 && Cout % HaloUp::BN == 0 &&
         (int64_t)(2 * R + 1) * (2 * R + 1) < (1LL << 31);
}

int launch_upconv_halo(const void* x, const void* w_up, void* t, int N, int R, int Cin, int Cout,
                       int act_in, const float* style, int dtype, hipStream_t st) {
  UpK k = {};
  k.x = x; k.w = w_up; k.t = t; k.style = style;
  k.N = N; k.R = R; k.Cin = Cin; k.Cout = Cout; k.act_in = act_in;
  const bool pro = style != nullptr || act_in != MIA_ACT_NONE;
  MIA_DISPATCH_DTYPE(dtype, T, {
    return pro ? launch_upconv_halo<T, true, false>(k, st)
               : launch_upconv_halo<T, false, false>(k, st);
  });
  return set_error("upconv_halo: unknown dtype");
}

bool s2_dgrad_halo_eligible(int dtype, int R, int Cg, int Cx) {
  const char* e = getenv("MIA_S2DG_HALO");  // tuning / A-B switch: 0 = generic phase GEMMs
  if (e && atoi(e) == 0) return false;
  return R % 16 == 0 && Cg % 64 == 0 && Cx % HaloUp::BN == 0 &&
         (int64_t)4 * R * R < (1LL << 31);
}

int launch_s2_dgrad_halo(const void* g, const void* w, void* gx, int N, int R, int Cg, int Cx,
                         const void* mask_a, const float* mask_slope, int accumulate, int dtype,
                         hipStream_t st) {
  UpK k = {};
  k.x = g; k.w = w; k.t = gx; k.mask_a = mask_a; k.mask_slope = mask_slope;
  k.N = N; k.R = R; k.Cin = Cg; k.Cout = Cx; k.accumulate = accumulate;
  MIA_DISPATCH_DTYPE(dtype, T, return launch_upconv_halo<T, false, true>(k, st));
  return set_error("s2_dgrad_halo: unknown dtype");
}

}  // namespace mia

using namespace mia;

extern "C" int mia_conv_s2_dgrad_halo(const void* g, const void* w_halo, void* gx, int N, int R,
                                      int Cg, int Cx, const void* mask_a, const float* mask_slope,
                                      int accumulate, int dtype, void* stream) {
  MIA_CHECK_ARG(g && w_halo && gx && N > 0, "bad args");
  MIA_CHECK_ARG(s2_dgrad_halo_eligible(dtype, R, Cg, Cx),
                "needs R % 16 == 0, Cg % 64 == 0, Cx % 64 == 0 "
                "(use mia_conv2d phase groups otherwise)");
  MIA_CHECK_ARG((int64_t)N * R * R * Cg < (1LL << 31), "input too large for 32-bit offsets");
  return launch_s2_dgrad_halo(g, w_halo, gx, N, R, Cg, Cx, mask_a, mask_slope, accumulate, dtype,
                              (hipStream_t)stream);
}
