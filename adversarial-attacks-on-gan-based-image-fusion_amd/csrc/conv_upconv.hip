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

// BN_ = 64 output channels per block (2 row waves × 2 column waves of 4 × 2 fragments) or 32
// (the 32-channel up-conv of the 1024² generator: 4 row waves × 1 column wave of 2 × 2 fragments)
template <int BN_>
struct HaloUpT {
  static constexpr int PH = 8, PW = 16, NW = 4, NT = 256;
  static constexpr int WN = BN_ == 64 ? 2 : 1, WM = NW / WN, FM = PH / WM, FN = 2;
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
  static_assert(WM * FM == PH && WN * FN * 16 == BN_, "");
};
typedef HaloUpT<64> HaloUp;

// K-step st: offset (jy, jx) and the phases of its two weight slots (−1: none)
__device__ __forceinline__ constexpr int up_jy(int st) { return st == 3 || st == 4 ? 1 : 0; }
__device__ __forceinline__ constexpr int up_jx(int st) { return st == 2 || st == 4 ? 1 : 0; }
__device__ __forceinline__ constexpr int up_phase(int st, int slot) {
  return st == 0 ? slot : st == 1 ? 2 + slot : st == 2 ? 2 * slot : st == 3 ? slot : (slot ? -1 : 0);
}

constexpr int UP_MAX_SRC = 8;
struct UpK {
  const void* x;
  const void* w;  // packed [Cin/BK][5][2][Cout][BK]
  void* t;        // (N, 2R+1, 2R+1, Cout); DG: (N, 2R, 2R, Cout)
  const float* style;
  const void* mask_a;       // DG: (N, 2R, 2R, Cout) or NULL
  const float* mask_slope;  // DG: [Cout] or NULL (→ 0)
  int N, R, Cin, Cout, act_in, nbn, nblk, accumulate;
  // the input as nsrc tensors (N, R, R, cin_src) concatenated along channels (Cin = nsrc·cin_src):
  // DG mode sums the input gradients of several stride-2 convs reading the same tensor (the e4e
  // style heads on one FPN map) in one K loop; xs[0] = x otherwise
  const void* xs[UP_MAX_SRC];
  int cin_src;
  const void* w_split;  // fp32: split_f32 of w (the split-once DG kernel), or NULL
};

// k.xs[i] for a wave-uniform i as a select chain over constant indices (a dynamic index into the
// by-value kernel argument would copy the array to scratch)
__device__ __forceinline__ const char* up_src(const UpK& k, int i) {
  const void* p = k.xs[0];
#pragma unroll
  for (int j = 1; j < UP_MAX_SRC; ++j) p = i == j ? k.xs[j] : p;
  return (const char*)p;
}

template <typename T, bool PRO, bool DG, int BN_ = 64>
__global__ __launch_bounds__(256, 2) void upconv_halo_kernel(const UpK k) {
  typedef HaloUpT<BN_> TL;
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
  // H-wave hw owns halo pieces hw + 2·j (in source tensor 0; another source is a uniform delta)
  const int csrc = k.cin_src, cbs = csrc / BK;  // channel blocks per source tensor
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
        src[j] = X + ((size_t)(n * R + y) * R + x) * csrc + ((lane & 7) ^ fsw(hr)) * VEC;
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
    if constexpr (!DG) {  // one source tensor
      const T* a = src[j] ? src[j] + cb * BK : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)a,
                                       (lptr_t)(hbuf + buf * HBUF + (hw + HWAVES * j) * 1024), 16,
                                       0, 0);
      return;
    }
    const int sc = cb / cbs;  // source tensor of channel block cb (wave-uniform)
    const int64_t delta = up_src(k, sc) - (const char*)X;
    const T* a = src[j] ? (const T*)((const char*)(src[j] + (cb - sc * cbs) * BK) + delta) : zero;
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
  // PRO (round 6, as conv_halo.hip): the landed halo of channel block cb modulated in place ONCE —
  // act(x)·s rounded to T exactly as modulate<T> on every fragment read (5 K-steps × 2 column
  // waves) would, so the outputs are bit-identical to the round-5 per-fragment form; zero padding
  // stays zero. bf16 up-conv forwards −28 … −33 % per call, fp16 −3 … −9 %
  // (profiles/r06_upconv_premod_ab.txt)
  auto premod = [&](int cb, int buf) {
    char* hb = hbuf + buf * HBUF;
    for (int c = tid; c < HROWS * 8; c += TL::NT) {
      const int hr = c >> 3, pc = c & 7, lc = pc ^ fsw(hr);
      VT v = *(const VT*)(hb + hr * ROWB + pc * 16);
      const VT sv = *(const VT*)(stab + cb * BK + lc * VEC);
      modulate<T>(v, sv, lrelu_in);
      *(VT*)(hb + hr * ROWB + pc * 16) = v;
    }
  };
  if (bwave) {
    issue_b(0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < H_INS; ++j) issue_h(0, j, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (PRO) {
    premod(0, 0);
    lds_handoff();
  }

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
      if constexpr (PRO) {
        if (st == 4 && cb + 1 < ncb) {  // the next block's halo landed (step 4's wait): modulate it
          premod(cb + 1, (cb + 1) & 1);
          lds_handoff();
        }
      }
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

template <typename T, bool PRO, bool DG = false, int BN_ = 64>
static int launch_upconv_halo(UpK& k, hipStream_t st) {
  typedef HaloUpT<BN_> TL;
  k.nbn = k.Cout / TL::BN;
  k.nblk = k.N * (k.R / TL::PH) * (k.R / TL::PW) * k.nbn;
  size_t lds = 2 * (size_t)TL::HBUF + (size_t)TL::STAGES * TL::BSTAGE;
  if (PRO) lds += (size_t)k.Cin * sizeof(T);
  if (lds > 160 * 1024) return set_error("upconv_halo: LDS budget exceeded");
  auto fn = upconv_halo_kernel<T, PRO, DG, BN_>;
  if (const int rc = ensure_dyn_lds((const void*)fn, 160 * 1024); rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(k.nblk), dim3(TL::NT), lds, st, k);
  return check_launch("upconv_halo");
}

bool upconv_halo_eligible(int dtype, int R, int Cin, int Cout) {
  if (tune(T_UPCONV_HALO) == 0) return false;  // the generic phase GEMMs
  return R % 16 == 0 && Cin % 64 == 0 && Cout % 32 == 0 &&
         (int64_t)(2 * R + 1) * (2 * R + 1) < (1LL << 31);
}

template <bool DG, bool PRO>
static int launch_upconv_x6(UpK& k, hipStream_t st);
static bool upconv_x6_ok(const UpK& k, int dtype);

int launch_upconv_halo(const void* x, const void* w_up, const void* w_up_split, void* t, int N,
                       int R, int Cin, int Cout, int act_in, const float* style, int dtype,
                       hipStream_t st) {
  UpK k = {};
  k.x = x; k.w = w_up; k.t = t; k.style = style;
  k.N = N; k.R = R; k.Cin = Cin; k.Cout = Cout; k.act_in = act_in;
  k.xs[0] = x; k.cin_src = Cin;
  k.w_split = w_up_split;
  const bool pro = style != nullptr || act_in != MIA_ACT_NONE;
  if (upconv_x6_ok(k, dtype))
    return pro ? launch_upconv_x6<false, true>(k, st) : launch_upconv_x6<false, false>(k, st);
  if (Cout % 64) {  // the 32-channel tile (1024² generator: 64 → 32 at 512²)
    MIA_DISPATCH_DTYPE(dtype, T, {
      return pro ? launch_upconv_halo<T, true, false, 32>(k, st)
                 : launch_upconv_halo<T, false, false, 32>(k, st);
    });
  }
  MIA_DISPATCH_DTYPE(dtype, T, {
    return pro ? launch_upconv_halo<T, true, false>(k, st)
               : launch_upconv_halo<T, false, false>(k, st);
  });
  return set_error("upconv_halo: unknown dtype");
}

// ---- fp32 stride-2 input gradient with the operands split once (bf16 matrix pipe) -------------
// DG mode of the kernel above for fp32 (conv_common.h mfma_x6, as conv_halo_x6.hip): the packed
// weights come pre-split from HBM (layouts.split_f32 of the packed tensor: per row of BK = 32 k a
// 128-B [hi|mid] record, then a 64-B lo record), each 32-channel block of the g halo is split in LDS
// once after its DMA lands ([hi|mid] in place + lo into an L buffer) and the main loop is ds_reads
// + 3 MFMAs per fragment pair with no split VALU (the kernel above splits both operands per
// fragment read: ≈ 145 TFLOP/s). Tile: a 16 × 16 patch of g × 64 output channels × the 4 output
// phases, 8 waves (4 row waves of 4 patch rows × 2 column waves of 32 channels), one block per CU:
// LDS = 2 halo buffers (2 × 37 KB, 17 × 17 pixels) + lo (18.5 KB) + a 2-stage pre-split weight ring
// (2 × 24 KB: two phase slots × 64 channels) = 140 KB. DMA roles as conv_halo_x6.hip: waves 0–3
// stream the weights one K-step ahead, waves 4–7 the next channel block's halo during steps 0–3;
// the next block's split follows the last step of the current one. The prologue and epilogue are
// not hidden behind a second block; the longest K loops gain most: the concatenated first-conv
// input gradients of the e4e style heads (K = 9 × 7 × 512 for the 7 fine heads).
struct DgX6 {
  static constexpr int PH = 16, PW = 16, NW = 8, NT = 64 * NW;
  static constexpr int WM = 4, WN = 2, FM = 4, FN = 2;
  static constexpr int BN = WN * FN * 16, BK = 32;              // 64 output channels
  static constexpr int HSIDE = PW + 1, HROWS = (PH + 1) * HSIDE;  // 289 halo pixels
  static constexpr int HPIECES = (HROWS + 7) / 8;                 // 37 pieces of 8 rows
  static constexpr int HBUF = HPIECES * 1024;
  static constexpr int LROWB = 64, LBUF = HROWS * LROWB;
  static constexpr int BROWS = 2 * BN;                            // two phase slots per K-step
  static constexpr int BHM = BROWS * ROWB, BSTAGE = BHM + BROWS * LROWB;
  static constexpr int BWAVES = 4, HWAVES = 4;
  static constexpr int B_HM_INS = BROWS / 8 / BWAVES;             // 4 [hi|mid] pieces per B-wave
  static constexpr int B_L_INS = BROWS / 16 / BWAVES;             // 2 lo pieces per B-wave
  static constexpr int H_INS = (HPIECES + HWAVES - 1) / HWAVES;   // 10
  static constexpr int HPS = (H_INS + 3) / 4;                     // issued over steps 0–3
  static constexpr int NSTEP = 5;
  static constexpr int LDS = 2 * HBUF + LBUF + 2 * BSTAGE;
  static_assert(WM * FM == PH && WN * FN * 16 == BN, "");
  static_assert(B_HM_INS * 8 * BWAVES == BROWS && B_L_INS * 16 * BWAVES == BROWS, "");
  static_assert(LDS <= 160 * 1024, "");
};

template <bool DG, bool PRO, bool EARLY, bool PRIO>
__global__ __launch_bounds__(DgX6::NT, 1) void upconv_x6_kernel(const UpK k) {
  typedef DgX6 TL;
  constexpr int FM = TL::FM, FN = TL::FN, WN = TL::WN, BN = TL::BN, BK = TL::BK, NT = TL::NT;
  constexpr int HSIDE = TL::HSIDE, HROWS = TL::HROWS, HPIECES = TL::HPIECES, HBUF = TL::HBUF;
  constexpr int H_INS = TL::H_INS, HPS = TL::HPS, HWAVES = TL::HWAVES, BSTAGE = TL::BSTAGE;
  constexpr int B_HM_INS = TL::B_HM_INS, B_L_INS = TL::B_L_INS;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                  // 2 halo buffers: raw fp32, then [hi|mid] in place
  char* const lbuf = smem + 2 * HBUF;       // lo of the current channel block
  char* const bring = lbuf + TL::LBUF;      // 2 stages of pre-split weights: [hi|mid] rows, lo rows

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int R = k.R, Cin = k.Cin, Cout = k.Cout;
  const int bl = xcd_remap(blockIdx.x, k.nblk);
  const int mt = bl / k.nbn, n0 = (bl % k.nbn) * BN;
  const int ptx = R / TL::PW, pty = R / TL::PH;
  const int x0 = (mt % ptx) * TL::PW;
  const int y0 = ((mt / ptx) % pty) * TL::PH;
  const int n = mt / (ptx * pty);
  const int ncb = Cin / BK, nk = TL::NSTEP * ncb;
  const int csrc = k.cin_src, cbs = csrc / BK;
  // packed rows: ((cb·5 + step)·2 + slot)·Cout + channel; [hi|mid] 128 B per row, then lo 64 B
  const char* Whm = (const char*)k.w_split;
  const char* Wl = Whm + (size_t)nk * 2 * Cout * ROWB;
  const size_t hm_step = (size_t)2 * Cout * ROWB, l_step = (size_t)2 * Cout * TL::LROWB;
  const char* zero = (const char*)g_zero16;
  const bool bwave = wid < TL::BWAVES;
  const int hw = wid - TL::BWAVES;

  // per-lane DMA sources: B-waves byte offsets of their weight pieces within a K-step's rows;
  // H-waves element offsets of their halo pieces in a source tensor (−1 → zero page)
  constexpr int NSRC = H_INS > B_HM_INS + B_L_INS ? H_INS : B_HM_INS + B_L_INS;
  int off[NSRC];  // (< 2^31: checked at the API)
#pragma unroll
  for (int j = 0; j < NSRC; ++j) {
    off[j] = -1;
    if (bwave) {
      if (j < B_HM_INS) {
        const int row = (wid * B_HM_INS + j) * 8 + (lane >> 3);
        const int slot = row / BN, c = n0 + row % BN;
        off[j] = (slot * Cout + c) * ROWB + ((lane & 7) ^ fsw(row)) * 16;
      } else if (j < B_HM_INS + B_L_INS) {
        const int row = (wid * B_L_INS + j - B_HM_INS) * 16 + (lane >> 2);
        const int slot = row / BN, c = n0 + row % BN;
        off[j] = (slot * Cout + c) * TL::LROWB + ((lane & 3) ^ (lsw(row) >> 1)) * 16;
      }
    } else if (j < H_INS) {
      const int hr = (hw + HWAVES * j) * 8 + (lane >> 3);
      const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
      const int y = y0 + hy - (DG ? 0 : 1), x = x0 + hx - (DG ? 0 : 1);
      if (hr < HROWS && y >= 0 && y < R && x >= 0 && x < R)
        off[j] = ((n * R + y) * R + x) * csrc + ((lane & 7) ^ fsw(hr)) * 4;
    }
  }

  // (the offsets pass through an opaque copy at each use: hoisted out of the loops, the 64-bit
  // per-lane addresses spill)
  auto opaque = [](int v) __attribute__((always_inline)) {
    asm volatile("" : "+v"(v));
    return v;
  };
  auto issue_b = [&](int s, int stg) {
    char* dst = bring + stg * BSTAGE;
    const char* hm = Whm + s * hm_step;
    const char* lo = Wl + s * l_step;
#pragma unroll
    for (int j = 0; j < B_HM_INS; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(hm + opaque(off[j])),
                                       (lptr_t)(dst + (wid * B_HM_INS + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < B_L_INS; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(lo + opaque(off[B_HM_INS + j])),
                                       (lptr_t)(dst + TL::BHM + (wid * B_L_INS + j) * 1024), 16,
                                       0, 0);
  };
  auto issue_h = [&](int cb, int j, int buf) {
    const int sc = cb / cbs;  // source tensor of channel block cb (wave-uniform)
    const float* xb = (const float*)up_src(k, sc) + (cb - sc * cbs) * BK;
    const int o = opaque(off[j]);
    const char* a = o >= 0 ? (const char*)(xb + o) : zero;
    __builtin_amdgcn_global_load_lds((gptr_t)a,
                                     (lptr_t)(hbuf + buf * HBUF + (hw + HWAVES * j) * 1024), 16,
                                     0, 0);
  };
  // split the landed raw halo of channel block cb in place + lo into lbuf (PRO: x̃ = act(x)·s
  // first, rounded as the on-the-fly path)
  const bool lrelu_in = k.act_in == MIA_ACT_LRELU_S2;
  auto convert = [&](int cb) {
    char* hb = hbuf + (cb & 1) * HBUF;
    for (int c = tid; c < HROWS * 8; c += NT) {
      const int hr = c >> 3, pc = c & 7, lc = pc ^ fsw(hr);
      f32x4 v = *(const f32x4*)(hb + hr * ROWB + pc * 16);
      if constexpr (PRO) {
        const float mul = lrelu_in ? SQRT2 : 1.f;
        f32x4 s4 = {1.f, 1.f, 1.f, 1.f};
        if (k.style) s4 = *(const f32x4*)(k.style + (size_t)n * Cin + cb * BK + lc * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float f = v[e];
          if (lrelu_in) f = fmaxf(f, 0.2f * f);
          v[e] = f * (s4[e] * mul);
        }
      }
      u32x4 hm;
      u32x2 lo;
      split_quad(v, hm, lo);
      *(u32x4*)(hb + hr * ROWB + pc * 16) = hm;
      *(u32x2*)(lbuf + hr * TL::LROWB + ((lc ^ lsw(hr)) << 3)) = lo;
    }
  };

  if (bwave) {
    issue_b(0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < H_INS; ++j)
      if (hw + HWAVES * j < HPIECES) issue_h(0, j, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  convert(0);
  __syncthreads();

  f32x4 acc[4][FM][FN];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int cb = 0; cb < ncb; ++cb) {
    const char* ha = hbuf + (cb & 1) * HBUF;
#pragma unroll
    for (int st = 0; st < TL::NSTEP; ++st) {
      const int ln = opaque(lane);  // the fragment addresses are recomputed per K-step
      const int frow = ln & 15, fq = ln >> 4;
      const int s = cb * TL::NSTEP + st;
      const char* sb = bring + (s & 1) * BSTAGE;
      if (bwave && s + 1 < nk) issue_b(s + 1, (s & 1) ^ 1);
      const int jy = up_jy(st), jx = up_jx(st);
      if constexpr (EARLY) {  // the next block's halo pieces before the step's LDS reads
        if (!bwave && st < 4 && cb + 1 < ncb) {
#pragma unroll
          for (int q = 0; q < HPS; ++q) {
            const int j = st * HPS + q;
            if (j < H_INS && hw + HWAVES * j < HPIECES) issue_h(cb + 1, j, (cb + 1) & 1);
          }
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = h * 4 + fq;  // this lane's logical 16-B quad of the K-step
        u32x4 ahm[FM];
        u32x2 al[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int hr = DG ? (wm * FM + i + jy) * HSIDE + frow + jx
                            : (wm * FM + i + 1 - jy) * HSIDE + frow + 1 - jx;
          ahm[i] = *(const u32x4*)(ha + hr * ROWB + ((ch ^ fsw(hr)) << 4));
          al[i] = *(const u32x2*)(lbuf + hr * TL::LROWB + ((ch ^ lsw(hr)) << 3));
        }
#pragma unroll
        for (int slot = 0; slot < 2; ++slot) {
          const int ph = up_phase(st, slot);
          if (ph < 0) continue;
          u32x4 bhm[FN];
          u32x2 blo[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int row = slot * BN + wn * FN * 16 + 16 * j + frow;
            bhm[j] = *(const u32x4*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
            blo[j] = *(const u32x2*)(sb + TL::BHM + row * TL::LROWB + ((ch ^ lsw(row)) << 3));
          }
          if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)  // D[channel][pixel]
              acc[ph][i][j] = mfma_x6(bhm[j], blo[j], ahm[i], al[i], acc[ph][i][j]);
          if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        }
        if (!EARLY && h == 0 && !bwave && st < 4 && cb + 1 < ncb) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < HPS; ++q) {
            const int j = st * HPS + q;
            if (j < H_INS && hw + HWAVES * j < HPIECES) issue_h(cb + 1, j, (cb + 1) & 1);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // B-wave: step s+1's weights landed; H-wave: the next block's halo before the split
      if (bwave || st == TL::NSTEP - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS reads of the step done
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (st == TL::NSTEP - 1 && cb + 1 < ncb) {  // every wave is past its last read of lbuf
        convert(cb + 1);
        __syncthreads();
      }
    }
  }

  // epilogue: phase (py, px) of input position (y, x) → T(2y + py, 2x + px) (DG: g position →
  // gx(2y + 1 − py, 2x + 1 − px)); lane (frow, fq) holds channels 4·fq … 4·fq+3 of fragment j
  // for pixel x0 + frow
  const int frow = lane & 15, fq = lane >> 4;
  float* __restrict__ Y = (float*)k.t;
  const int TS = DG ? 2 * R : 2 * R + 1;
  float msl[FN][4];  // slope of the mask per channel of this lane
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      msl[j][e] = k.mask_slope ? k.mask_slope[n0 + wn * FN * 16 + 16 * j + 4 * fq + e] : 0.f;
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
        const size_t o = ((size_t)(n * TS + ty) * TS + tx) * Cout + c;
        f32x4 v = acc[ph][i][j];
        if (DG && k.mask_a) {
          const f32x4 m = *(const f32x4*)((const float*)k.mask_a + o);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = m[e] > 0.f ? v[e] : msl[j][e] * v[e];
        }
        if (DG && k.accumulate) {
          const f32x4 a = *(const f32x4*)(Y + o);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += a[e];
        }
        *(f32x4*)(Y + o) = v;
      }
    }
  }
}

// ---- the same on an 8 × 16 patch, two blocks per CU (round 4) --------------------------------
// As conv_halo_x6.hip's HaloX6S for the 64-channel stride-1 layers: the kernel above is one 8-wave
// block per CU, so its per-step barriers, channel-block splits, prologue and epilogue stall the
// whole CU. Here a block is an 8 × 16 patch (4 row waves of 2 patch rows × 64 channels × the 4
// phases: the same 128 accumulator VGPRs per wave), LDS = ONE halo buffer + lo + the 2-stage weight
// ring = 77.6 KB, two blocks per CU; every wave streams a share of the weights (6 pieces per
// K-step) and of the next channel block's halo (fetched after the block's last step). Same MFMAs
// in the same order per output as the kernel above (bit-identical).
struct DgX6S {
  static constexpr int PH = 8, PW = 16, NW = 4, NT = 64 * NW;
  static constexpr int WM = 4, WN = 1, FM = 2, FN = 4;
  static constexpr int BN = WN * FN * 16, BK = 32;              // 64 output channels
  static constexpr int HSIDE = PW + 1, HROWS = (PH + 1) * HSIDE;  // 153 halo pixels
  static constexpr int HPIECES = (HROWS + 7) / 8;                 // 20 pieces of 8 rows
  static constexpr int HBUF = HPIECES * 1024;
  static constexpr int LROWB = 64, LBUF = HROWS * LROWB;
  static constexpr int BROWS = 2 * BN;                            // two phase slots per K-step
  static constexpr int BHM = BROWS * ROWB, BSTAGE = BHM + BROWS * LROWB;
  static constexpr int B_HM_INS = BROWS / 8 / NW;                 // 4 [hi|mid] pieces per wave
  static constexpr int B_L_INS = BROWS / 16 / NW;                 // 2 lo pieces per wave
  static constexpr int H_INS = (HPIECES + NW - 1) / NW;           // 5
  static constexpr int NSTEP = 5;
  static constexpr int LDS = HBUF + LBUF + 2 * BSTAGE;
  static_assert(WM * FM == PH && WN * FN * 16 == BN, "");
  static_assert(B_HM_INS * 8 * NW == BROWS && B_L_INS * 16 * NW == BROWS, "");
  static_assert(LDS <= 80 * 1024, "two blocks per CU");
};

template <bool DG, bool PRO>
__global__ __launch_bounds__(DgX6S::NT, 2) void upconv_x6s_kernel(const UpK k) {
  typedef DgX6S TL;
  constexpr int FM = TL::FM, FN = TL::FN, WN = TL::WN, BN = TL::BN, BK = TL::BK, NT = TL::NT;
  constexpr int HSIDE = TL::HSIDE, HROWS = TL::HROWS, HPIECES = TL::HPIECES;
  constexpr int H_INS = TL::H_INS, BSTAGE = TL::BSTAGE;
  constexpr int B_HM_INS = TL::B_HM_INS, B_L_INS = TL::B_L_INS;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                  // the halo: raw fp32, then [hi|mid] in place
  char* const lbuf = smem + TL::HBUF;       // lo of the current channel block
  char* const bring = lbuf + TL::LBUF;      // 2 stages of pre-split weights: [hi|mid] rows, lo rows

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int R = k.R, Cin = k.Cin, Cout = k.Cout;
  const int bl = xcd_remap(blockIdx.x, k.nblk);
  const int mt = bl / k.nbn, n0 = (bl % k.nbn) * BN;
  const int ptx = R / TL::PW, pty = R / TL::PH;
  const int x0 = (mt % ptx) * TL::PW;
  const int y0 = ((mt / ptx) % pty) * TL::PH;
  const int n = mt / (ptx * pty);
  const int ncb = Cin / BK, nk = TL::NSTEP * ncb;
  const int csrc = k.cin_src, cbs = csrc / BK;
  const char* Whm = (const char*)k.w_split;
  const char* Wl = Whm + (size_t)nk * 2 * Cout * ROWB;
  const size_t hm_step = (size_t)2 * Cout * ROWB, l_step = (size_t)2 * Cout * TL::LROWB;
  const char* zero = (const char*)g_zero16;

  // per-lane DMA offsets: this wave's weight pieces (bytes within a K-step's rows) and its halo
  // pieces (elements in a source tensor, −1 → the zero page); < 2^31, checked at the API
  int woff[B_HM_INS + B_L_INS], hoff[H_INS];
#pragma unroll
  for (int j = 0; j < B_HM_INS + B_L_INS; ++j) {
    if (j < B_HM_INS) {
      const int row = (wid * B_HM_INS + j) * 8 + (lane >> 3);
      const int slot = row / BN, c = n0 + row % BN;
      woff[j] = (slot * Cout + c) * ROWB + ((lane & 7) ^ fsw(row)) * 16;
    } else {
      const int row = (wid * B_L_INS + j - B_HM_INS) * 16 + (lane >> 2);
      const int slot = row / BN, c = n0 + row % BN;
      woff[j] = (slot * Cout + c) * TL::LROWB + ((lane & 3) ^ (lsw(row) >> 1)) * 16;
    }
  }
#pragma unroll
  for (int j = 0; j < H_INS; ++j) {
    hoff[j] = -1;
    const int hr = (wid + TL::NW * j) * 8 + (lane >> 3);
    const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
    const int y = y0 + hy - (DG ? 0 : 1), x = x0 + hx - (DG ? 0 : 1);
    if (hr < HROWS && y >= 0 && y < R && x >= 0 && x < R)
      hoff[j] = ((n * R + y) * R + x) * csrc + ((lane & 7) ^ fsw(hr)) * 4;
  }
  auto opaque = [](int v) __attribute__((always_inline)) {
    asm volatile("" : "+v"(v));
    return v;
  };
  auto issue_b = [&](int s, int stg) {
    char* dst = bring + stg * BSTAGE;
    const char* hm = Whm + s * hm_step;
    const char* lo = Wl + s * l_step;
#pragma unroll
    for (int j = 0; j < B_HM_INS; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(hm + opaque(woff[j])),
                                       (lptr_t)(dst + (wid * B_HM_INS + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < B_L_INS; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(lo + opaque(woff[B_HM_INS + j])),
                                       (lptr_t)(dst + TL::BHM + (wid * B_L_INS + j) * 1024), 16,
                                       0, 0);
  };
  auto issue_halo = [&](int cb) {
    const int sc = cb / cbs;  // source tensor of channel block cb (wave-uniform)
    const float* xb = (const float*)up_src(k, sc) + (cb - sc * cbs) * BK;
#pragma unroll
    for (int j = 0; j < H_INS; ++j) {
      if (wid + TL::NW * j >= HPIECES) break;
      const int o = opaque(hoff[j]);
      const char* a = o >= 0 ? (const char*)(xb + o) : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)a, (lptr_t)(hbuf + (wid + TL::NW * j) * 1024), 16,
                                       0, 0);
    }
  };
  const bool lrelu_in = k.act_in == MIA_ACT_LRELU_S2;
  auto convert = [&](int cb) {
    for (int c = tid; c < HROWS * 8; c += NT) {
      const int hr = c >> 3, pc = c & 7, lc = pc ^ fsw(hr);
      f32x4 v = *(const f32x4*)(hbuf + hr * ROWB + pc * 16);
      if constexpr (PRO) {
        const float mul = lrelu_in ? SQRT2 : 1.f;
        f32x4 s4 = {1.f, 1.f, 1.f, 1.f};
        if (k.style) s4 = *(const f32x4*)(k.style + (size_t)n * Cin + cb * BK + lc * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float f = v[e];
          if (lrelu_in) f = fmaxf(f, 0.2f * f);
          v[e] = f * (s4[e] * mul);
        }
      }
      u32x4 hm;
      u32x2 lo;
      split_quad(v, hm, lo);
      *(u32x4*)(hbuf + hr * ROWB + pc * 16) = hm;
      *(u32x2*)(lbuf + hr * TL::LROWB + ((lc ^ lsw(hr)) << 3)) = lo;
    }
  };

  issue_halo(0);
  issue_b(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  convert(0);
  __syncthreads();

  f32x4 acc[4][FM][FN];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int cb = 0; cb < ncb; ++cb) {
#pragma unroll
    for (int st = 0; st < TL::NSTEP; ++st) {
      const int ln = opaque(lane);  // the fragment addresses are recomputed per K-step
      const int frow = ln & 15, fq = ln >> 4;
      const int s = cb * TL::NSTEP + st;
      const char* sb = bring + (s & 1) * BSTAGE;
      if (s + 1 < nk) issue_b(s + 1, (s & 1) ^ 1);
      const int jy = up_jy(st), jx = up_jx(st);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = h * 4 + fq;
        u32x4 ahm[FM];
        u32x2 al[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int hr = DG ? (wm * FM + i + jy) * HSIDE + frow + jx
                            : (wm * FM + i + 1 - jy) * HSIDE + frow + 1 - jx;
          ahm[i] = *(const u32x4*)(hbuf + hr * ROWB + ((ch ^ fsw(hr)) << 4));
          al[i] = *(const u32x2*)(lbuf + hr * TL::LROWB + ((ch ^ lsw(hr)) << 3));
        }
#pragma unroll
        for (int slot = 0; slot < 2; ++slot) {
          const int ph = up_phase(st, slot);
          if (ph < 0) continue;
          u32x4 bhm[FN];
          u32x2 blo[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int row = slot * BN + wn * FN * 16 + 16 * j + frow;
            bhm[j] = *(const u32x4*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
            blo[j] = *(const u32x2*)(sb + TL::BHM + row * TL::LROWB + ((ch ^ lsw(row)) << 3));
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)  // D[channel][pixel]
              acc[ph][i][j] = mfma_x6(bhm[j], blo[j], ahm[i], al[i], acc[ph][i][j]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of step s+1
      lds_handoff();
      __builtin_amdgcn_sched_barrier(0);
    }
    if (cb + 1 < ncb) {  // every wave is past its last read of the halo and lo
      issue_halo(cb + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      convert(cb + 1);
      __syncthreads();
    }
  }

  const int frow = lane & 15, fq = lane >> 4;
  float* __restrict__ Y = (float*)k.t;
  const int TS = DG ? 2 * R : 2 * R + 1;
  float msl[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      msl[j][e] = k.mask_slope ? k.mask_slope[n0 + wn * FN * 16 + 16 * j + 4 * fq + e] : 0.f;
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
        const size_t o = ((size_t)(n * TS + ty) * TS + tx) * Cout + c;
        f32x4 v = acc[ph][i][j];
        if (DG && k.mask_a) {
          const f32x4 m = *(const f32x4*)((const float*)k.mask_a + o);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = m[e] > 0.f ? v[e] : msl[j][e] * v[e];
        }
        if (DG && k.accumulate) {
          const f32x4 a = *(const f32x4*)(Y + o);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += a[e];
        }
        *(f32x4*)(Y + o) = v;
      }
    }
  }
}

template <bool DG, bool PRO>
static int launch_upconv_x6s(UpK& k, hipStream_t st) {
  typedef DgX6S TL;
  k.nbn = k.Cout / TL::BN;
  k.nblk = k.N * (k.R / TL::PH) * (k.R / TL::PW) * k.nbn;
  auto fn = upconv_x6s_kernel<DG, PRO>;
  if (const int rc = ensure_dyn_lds((const void*)fn, 80 * 1024); rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(k.nblk), dim3(TL::NT), TL::LDS, st, k);
  return check_launch("upconv_x6s");
}

template <bool DG, bool PRO, bool EARLY, bool PRIO>
static int launch_upconv_x6_e(UpK& k, hipStream_t st) {
  typedef DgX6 TL;
  k.nbn = k.Cout / TL::BN;
  k.nblk = k.N * (k.R / TL::PH) * (k.R / TL::PW) * k.nbn;
  auto fn = upconv_x6_kernel<DG, PRO, EARLY, PRIO>;
  if (const int rc = ensure_dyn_lds((const void*)fn, 160 * 1024); rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(k.nblk), dim3(TL::NT), TL::LDS, st, k);
  return check_launch("upconv_x6");
}

template <bool DG, bool PRO>
static int launch_upconv_x6(UpK& k, hipStream_t st) {
  // T_UPCONV_X6S = 1 (default): the 8 × 16-patch two-blocks-per-CU form for the stride-2 input
  // gradients with Cin ≤ 512 (≤ 16 channel blocks: their prologue / splits / epilogue are the
  // exposed share); measured (fp32, 128 images, profiles/r04_layers_fp32_b128_e4e_upx6s_*):
  // e4e body / single heads R128 / R64 / R32 / R16 −9 / −12 / −11 / −2 % per call, the long
  // multi-source K loops (7 × 512, 4 × 512 channels) +5 / +4 %, the up-conv forward ±0.5 %
  if (DG && tune(T_UPCONV_X6S) != 0 && k.Cin <= 512) return launch_upconv_x6s<DG, PRO>(k, st);
  // the next block's halo DMA at the step start (as the x6 halo kernel; neutral here against
  // issuing it between the two MFMA halves); no s_setprio (neutral, +1 / −1 % by layer)
  return launch_upconv_x6_e<DG, PRO, true, false>(k, st);
}

// the split-once kernel: fp32 with pre-split weights, R % 16 == 0, Cx % 64 == 0 (T_S2DG_X6 = 0
// disables: tests / tuning). Measured against the on-the-fly split kernel (fp32,
// 128 images, tools/layer_table.py): the 7 concatenated fine heads 146 → 210 TFLOP/s, single
// 512-channel heads at 16² 133 → 197, the bottleneck units (Cg 64 / 128 / 256) 69 / 97 / 122 →
// 96 / 147 / 176 — faster at every shape of the attack despite the exposed prologue / epilogue.
// the split-once kernel for the up-sampling conv forward (fp32, w_up_split given; the last row /
// column still goes to the generic kernel). T_UPCONV_X6 = 0 disables (tests / tuning).
static bool upconv_x6_ok(const UpK& k, int dtype) {
#ifdef MIA_F32_NATIVE
  (void)k;
  (void)dtype;
  return false;
#else
  if (tune(T_UPCONV_X6) == 0) return false;
  return dtype == MIA_F32 && k.w_split && k.R % DgX6::PH == 0 && k.Cout % DgX6::BN == 0 &&
         k.Cin % DgX6::BK == 0;
#endif
}

static bool s2dg_x6_ok(const UpK& k, int dtype) {
#ifdef MIA_F32_NATIVE
  (void)k;
  (void)dtype;
  return false;
#else
  if (tune(T_S2DG_X6) == 0) return false;
  return dtype == MIA_F32 && k.w_split && k.R % DgX6::PH == 0 && k.Cout % DgX6::BN == 0 &&
         k.cin_src % DgX6::BK == 0;
#endif
}

bool s2_dgrad_halo_eligible(int dtype, int R, int Cg, int Cx) {
  if (tune(T_S2DG_HALO) == 0) return false;  // the generic phase GEMMs
  (void)dtype;
  return R % 16 == 0 && Cg % 64 == 0 && Cx % HaloUp::BN == 0 &&
         (int64_t)4 * R * R < (1LL << 31);
}

}  // namespace mia

using namespace mia;

extern "C" int mia_conv_s2_dgrad_halo_multi(const void* const* g, int ng, const void* w_halo,
                                            const void* w_split, void* gx, int N, int R, int Cg,
                                            int Cx, const void* mask_a, const float* mask_slope,
                                            int accumulate, int dtype, void* stream) {
  MIA_CHECK_ARG(g && ng >= 1 && ng <= UP_MAX_SRC && w_halo && gx && N > 0, "bad args");
  for (int i = 0; i < ng; ++i) MIA_CHECK_ARG(g[i], "null source tensor");
  MIA_CHECK_ARG(s2_dgrad_halo_eligible(dtype, R, Cg, Cx),
                "needs R % 16 == 0, Cg % 64 == 0, Cx % 64 == 0 "
                "(use mia_conv2d phase groups otherwise)");
  MIA_CHECK_ARG((int64_t)N * R * R * Cg < (1LL << 31), "input too large for 32-bit offsets");
  UpK k = {};
  k.x = g[0]; k.w = w_halo; k.t = gx; k.mask_a = mask_a; k.mask_slope = mask_slope;
  k.N = N; k.R = R; k.Cin = ng * Cg; k.Cout = Cx; k.accumulate = accumulate;
  for (int i = 0; i < ng; ++i) k.xs[i] = g[i];
  k.cin_src = Cg;
  k.w_split = w_split;
  if (s2dg_x6_ok(k, dtype)) return launch_upconv_x6<true, false>(k, (hipStream_t)stream);
  MIA_DISPATCH_DTYPE(dtype, T, return launch_upconv_halo<T, false, true>(k, (hipStream_t)stream));
  return set_error("s2_dgrad_halo: unknown dtype");
}


extern "C" int mia_conv_s2_dgrad_halo(const void* g, const void* w_halo, void* gx, int N, int R,
                                      int Cg, int Cx, const void* mask_a, const float* mask_slope,
                                      int accumulate, int dtype, void* stream) {
  const void* gs[1] = {g};
  return mia_conv_s2_dgrad_halo_multi(gs, 1, w_halo, nullptr, gx, N, R, Cg, Cx, mask_a,
                                      mask_slope, accumulate, dtype, stream);
}
