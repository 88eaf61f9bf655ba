// Implicit-GEMM convolution on CDNA4 MFMA (gfx950), NHWC.
//
// One kernel serves every dense contraction of the attack step:
//   * VGG conv + bias + ReLU forward        (code/vgg.py:45-62)
//   * VGG conv input-gradient                (flipped/transposed weights; tap-MSE + ReLU mask fused)
//   * ModulatedConv2d forward [ext]          (modulation = per-(n,ci) A-operand scale applied to the
//                                             MFMA fragments, demodulation = per-(n,co) epilogue
//                                             scale: one shared-weight GEMM, never N per-sample
//                                             weight tensors)
//   * up-sampling ModulatedConv2d [ext]      conv_transpose2d(stride 2) as four sub-pixel phase
//                                             GEMMs (2×2, 2×1, 1×2, 1×1 taps) in ONE launch, or the
//                                             blur-folded 4-phase 3×3 variant (shuffle_out)
//   * ModulatedConv2d input/style gradient   (dgrad GEMM, stride 1 or the stride-2 transposed-conv
//                                             adjoint, + Σ_p gx̃·x style reduction in the epilogue)
//
// GEMM view per problem ("group"): M = N·Ho·Wo output pixels, N-dim = Cout,
// K = KH·KW·Cin (tap-major, channel-minor). Input pixel of tap (ty,tx) for output (y,x) is
// (s·y + ty − pad_y, s·x + tx − pad_x); the result lands at (ay·y + by, ax·x + bx).
// Block tile BM×BN×BK, 256 threads = 4 waves (2×2), each wave FM×FN MFMA 16×16 fragments.
//   f16/bf16: v_mfma_f32_16x16x32_{f16,bf16}, BK = 64;  f32: v_mfma_f32_16x16x4_f32, BK = 32.
// Every tile row (a pixel's or an output channel's K-slice) is 128 B = 8 chunks of 16 B.
//
// Staging: both operands go global → LDS by LDS-DMA (global_load_lds_dwordx4), a 2-stage ring:
// the loads of K-step k+1 are issued before the MFMAs of step k and retired by the barrier at its
// end. The im2col gather is the per-lane SOURCE address (one pixel row + tap offset); lanes whose
// tap falls outside the input (or whose row is past M / Cout) read a 16-byte zero vector, so the
// loop has no branches. For Cin ≥ BK the tap is uniform per K-step and each DMA costs one 64-bit
// add. LDS-DMA writes lane-linearly, so the bank swizzle (conv_common.h fsw(),
// conflict-free for the ds_read_b128 fragment lane groups on 128-B rows) is applied by permuting
// which chunk each lane fetches (guide rule 21). The modulation prologue x̃ = act(x)·s[n][ci] is
// applied to A fragments after ds_read, with s held in an LDS table for the (≤ 9) images a tile
// spans. The epilogue stages the fp32 tile through LDS and then works on 8-channel vectors
// (16-byte loads of every aux operand, 16-byte stores).
#include "conv_common.h"
#include <cstdio>
#include "halo_epilogue.h"

#ifndef MIA_F32_PRO_SMALLTILE  // tile-count threshold of the fp32 PRO 64×64 tile (0 = off; A/B)
#define MIA_F32_PRO_SMALLTILE 128
#endif

namespace mia {

// s_waitcnt leaving at most `steps` K-steps of DMA (PER vm instructions each) in flight
template <int PER>
__device__ __forceinline__ void wait_dma_steps(int steps) {
  static_assert(3 * PER <= 63, "vmcnt field");
  if (steps <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (steps == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
  else if (steps == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory");
}

// EPI: −2 = LDS-staged shared epilogue (conv_epilogue); ≥ 0 = the register epilogue specialised
// for feature mask EPI (halo_epilogue_f; MFMAs computed transposed, D[channel][pixel]), for
// single-image tiles of whole 16-pixel rows with identity placement (see reg_epi_ok).
// X6B (fp32 only): the weights come pre-split from HBM (mia_conv_group.w_split): a B stage holds
// [hi|mid] rows (the fp32 row geometry) + 64-B lo rows, B fragments are read pre-split, and only
// the A fragments are split on the fly (conv_common.h split_quad) — half the split VALU of the
// mfma_chunk<float> path, whose VALU bound this lowers.
template <typename T, int BM, int BN, bool X6B>
struct StageBytes {
  static constexpr int v = (BM + BN) * ROWB;
};
template <int BM, int BN>
struct StageBytes<float, BM, BN, true> {
  static constexpr int v = BM * ROWB + BN * (ROWB + 64);
};

template <typename T, typename TL, bool PRO, bool SMALLC, int EPI = -2, bool X6B = false>
__global__ __launch_bounds__(TL::NT, TL::NW == 4 && TL::STAGES <= 3 ? (TL::BM < 128 ? 4 : 2) : 1) void conv_kernel(
    const ConvK k) {
  typedef typename Vec<T>::type VT;
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = ROWB / (int)sizeof(T);
  constexpr int WN = TL::WN, FM = TL::FM, FN = TL::FN, NT = TL::NT;
  constexpr int BM = TL::BM, BN = TL::BN, A_INS = TL::A_INS, B_INS = TL::B_INS;
  constexpr bool X6 = X6B && std::is_same<T, float>::value;
  constexpr int STAGE = StageBytes<T, BM, BN, X6>::v, STAGES = TL::STAGES;
  constexpr int B_L_INS = X6 ? BN / (16 * TL::NW) : 0;  // lo-row pieces (16 rows) per wave
  static_assert(!X6 || B_L_INS * 16 * TL::NW == BN, "");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform → scalar LDS bases
  const int wm = wid / WN, wn = wid % WN;
  const int bl = xcd_remap(blockIdx.x, k.nblk);
  int gi = 0;
#pragma unroll
  for (int g = 1; g < MIA_MAX_GROUPS; ++g)
    if (g < k.ng && bl >= k.g[g].blk0) gi = g;
  const ConvGroup G = k.g[gi];  // by value: scalar registers for the whole kernel
  const int b = bl - G.blk0;
  const int m0 = (b / k.nbn) * BM, n0 = (b % k.nbn) * BN;
  const int Hin = p.H, Win = p.W, Cin = p.Cin;
  const int HWo = G.ho * G.wo;
  const int ntap = G.kh * G.kw;

  const T* __restrict__ X = (const T*)p.x;
  // X6: the [hi|mid] words of the pre-split weights have the fp32 row geometry (4 B per k)
  const T* __restrict__ Wt = X6 ? (const T*)G.w_split : (const T*)G.w;
  const T* zero = (const T*)g_zero16;

  // ---- per-lane DMA source state -----------------------------------------------------------
  const T* a_ptr[A_INS];
  int a_base[A_INS], a_koff[A_INS], a_mask[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wid * A_INS + j) * 8 + (lane >> 3);
    a_koff[j] = ((lane & 7) ^ fsw(row)) * VEC;
    const int m = m0 + row;
    int msk = 0, base = 0;
    if (m < G.m) {
      const int ng = m / HWo;  // image within the group
      const int rem = m - ng * HWo;
      const int n = ng + G.n_in;
      const int y = rem / G.wo, x = rem - (rem / G.wo) * G.wo;
      const int iy0 = k.stride * y - G.pad_y, ix0 = k.stride * x - G.pad_x;
      base = ((n * Hin + iy0) * Win + ix0) * Cin;
      for (int t = 0; t < ntap; ++t) {
        const int ty = div_kw(t, G.kw), tx = t - ty * G.kw;
        const int yy = iy0 + ty, xx = ix0 + tx;
        if (yy >= 0 && yy < Hin && xx >= 0 && xx < Win) msk |= 1 << t;
      }
    }
    a_base[j] = base;
    a_mask[j] = msk;
    a_ptr[j] = X + base + a_koff[j];
  }
  const T* b_ptr[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wid * B_INS + j) * 8 + (lane >> 3);
    const int c = n0 + row;
    b_ptr[j] = c < p.Cout ? Wt + (size_t)c * G.kpad + ((lane & 7) ^ fsw(row)) * VEC : zero;
  }
  const char* bl_ptr[B_L_INS > 0 ? B_L_INS : 1];
  if constexpr (X6) {
    const __bf16* Wl = (const __bf16*)((const unsigned*)G.w_split + (size_t)p.Cout * G.kpad);
#pragma unroll
    for (int j = 0; j < B_L_INS; ++j) {
      const int row = (wid * B_L_INS + j) * 16 + (lane >> 2);
      const int c = n0 + row;
      bl_ptr[j] = c < p.Cout ? (const char*)(Wl + (size_t)c * G.kpad +
                                             ((lane & 3) ^ (lsw(row) >> 1)) * 8)
                             : nullptr;
    }
  }

  // K-step state for the DMA issue (uniform across the block)
  int is_tap = 0, is_cb = 0;
  const int ncb = SMALLC ? 1 : Cin / BK;

  auto issue = [&](int kb, int st) {
    char* sa = smem + st * STAGE;
    char* sb = sa + BM * ROWB;
    if constexpr (SMALLC) {
#pragma unroll
      for (int j = 0; j < A_INS; ++j) {
        const int kk = kb * BK + a_koff[j];
        const int tap = kk >> k.log2cin;
        const int ci = kk & (Cin - 1);
        const int ty = div_kw(tap, G.kw), tx = tap - ty * G.kw;
        const T* src = ((a_mask[j] >> tap) & 1) ? X + (a_base[j] + (ty * Win + tx) * Cin + ci)
                                                 : zero;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(sa + (wid * A_INS + j) * 1024), 16,
                                         0, 0);
      }
    } else {
      const int ty = div_kw(is_tap, G.kw), tx = is_tap - ty * G.kw;
      const int off = (ty * Win + tx) * Cin + is_cb * BK;  // uniform
#pragma unroll
      for (int j = 0; j < A_INS; ++j) {
        const T* src = ((a_mask[j] >> is_tap) & 1) ? a_ptr[j] + off : zero;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(sa + (wid * A_INS + j) * 1024), 16,
                                         0, 0);
      }
      if (++is_cb == ncb) { is_cb = 0; ++is_tap; }
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const T* src = b_ptr[j] == zero ? zero : b_ptr[j] + (size_t)kb * BK;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(sb + (wid * B_INS + j) * 1024), 16,
                                       0, 0);
    }
    if constexpr (X6) {
#pragma unroll
      for (int j = 0; j < B_L_INS; ++j) {
        const char* src = bl_ptr[j] ? bl_ptr[j] + (size_t)kb * BK * 2 : (const char*)zero;
        __builtin_amdgcn_global_load_lds(
            (gptr_t)src, (lptr_t)(sb + BN * ROWB + (wid * B_L_INS + j) * 1024), 16, 0, 0);
      }
    }
  };

  // ---- modulation table (PRO): s[n][ci] (·√2 for lrelu inputs) for the images of this tile ----
  const int n_first = m0 / HWo;
  T* stab = (T*)(smem + STAGES * STAGE);
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;
  int a_nl[FM];
  if constexpr (PRO) {
    const int n_last = (min(m0 + BM, G.m) - 1) / HWo;
    const int cnt = (n_last - n_first + 1) * Cin;
    const float mul = lrelu_in ? SQRT2 : 1.f;
    for (int i = tid; i < cnt; i += NT) {
      const float sv = p.in_scale ? p.in_scale[(size_t)(n_first + G.n_in) * Cin + i] : 1.f;
      stab[i] = from_f<T>(sv * mul);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = min(m0 + wm * FM * 16 + 16 * i + (lane & 15), G.m - 1);
      a_nl[i] = (m / HWo - n_first) * Cin;
    }
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K-steps of this group's taps (= kpad / BK for a full weight row; an edge group of the up-conv
  // runs only the leading taps of its rows, kpad staying the row stride)
  const int nk = (ntap * Cin + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);
  if constexpr (STAGES == 2) {
    __syncthreads();
  } else {
    static_assert(!X6, "X6B: 2-stage tiles only");
    // retire step 0 (the later prologue steps may stay in flight), then make every wave's DMA
    // visible
    wait_dma_steps<A_INS + B_INS>(min(nk, STAGES - 1) - 1);
    __syncthreads();
  }
  const int frow = lane & 15, fq = lane >> 4;
  int st = 0;
  for (int kb = 0; kb < nk; ++kb) {
    const int ahead = kb + STAGES - 1;
    const int st_ahead = st == 0 ? STAGES - 1 : st - 1;  // (kb + STAGES - 1) % STAGES
    if (ahead < nk) issue(ahead, st_ahead);
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
      if constexpr (X6) {
        u32x4 ahm[FM], bhm[FN];
        u32x2 alo[FM], blo[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * FN * 16 + 16 * j + frow;
          bhm[j] = *(const u32x4*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
          blo[j] = *(const u32x2*)(sb + BN * ROWB + row * 64 + ((ch ^ lsw(row)) << 3));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#ifdef MIA_PROBE_NOSPLIT_A  // timing probe only (wrong numerics): the A split's VALU removed
          const u32x4 u = __builtin_bit_cast(u32x4, af[i]);  // hi = truncated bf16, mid = lo = 0
          ahm[i] = u32x4{__builtin_amdgcn_perm(u[1], u[0], 0x07060302u),
                         __builtin_amdgcn_perm(u[3], u[2], 0x07060302u), 0u, 0u};
          alo[i] = u32x2{0u, 0u};
#else
          split_quad(af[i], ahm[i], alo[i]);
#endif
        }
        if (k.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = EPI == -2 ? mfma_x6(ahm[i], alo[i], bhm[j], blo[j], acc[i][j])
                                  : mfma_x6(bhm[j], blo[j], ahm[i], alo[i], acc[i][j]);
        if (k.prio) __builtin_amdgcn_s_setprio(0);
        continue;
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
        for (int j = 0; j < FN; ++j)
          acc[i][j] = EPI == -2 ? mfma_chunk<T>(af[i], bf[j], acc[i][j])   // D[pixel][channel]
                                : mfma_chunk<T>(bf[j], af[i], acc[i][j]);  // D[channel][pixel]
    }
    if constexpr (STAGES == 2) {
      __syncthreads();  // retires the DMA of step kb+1 (vmcnt(0)) and frees stage st
    } else {
      // step kb+1 must have landed; steps kb+2 … (issued up to this iteration) may stay in flight
      wait_dma_steps<A_INS + B_INS>(min(STAGES - 2, nk - 2 - kb));
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS reads of stage st done
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    st = st + 1 == STAGES ? 0 : st + 1;
  }
  if constexpr (STAGES != 2) __syncthreads();

  // ---- epilogue ---------------------------------------------------------------------------
  if constexpr (EPI >= 0) {
    const int n_img = m0 / HWo;  // the whole tile is in this image (reg_epi_ok)
    halo_epilogue_f<T, TL, EPI>(k, acc, n_img, (m0 - n_img * HWo) >> 4, 0, n0, wm, wn, lane,
                                HWo >> 4, 16, nullptr, k.prered ? (float*)smem : nullptr, TL::WM,
                                TL::BN);
  } else {
    const int last = min(m0 + BM, G.m) - 1;
    const int n_first_img = m0 / HWo;
    // sums: one partial per channel per tile (slot = the tile's index within its image) when
    // the images are whole tiles, else one per output pixel (k.red_px: small images)
    const bool single = n_first_img == last / HWo && !k.red_px;
    const int gm = G.m;
    conv_epilogue<T, TL>(k, G, acc, smem, n0, single, n_first_img, [=](int r) {
      const int m = m0 + r;
      return m < gm ? m : -1;
    }, (m0 - n_first_img * HWo) / BM);
  }
}

template <typename T, typename TL, bool PRO, bool SMALLC, int EPI = -2, bool X6B = false>
static int launch_tile(ConvK& k, hipStream_t st) {
  k.nbn = (k.a.Cout + TL::BN - 1) / TL::BN;
  int blk = 0;
  for (int g = 0; g < k.ng; ++g) {
    k.g[g].nbm = (k.g[g].m + TL::BM - 1) / TL::BM;
    k.g[g].blk0 = blk;
    blk += k.g[g].nbm * k.nbn;
  }
  k.nblk = blk;
  size_t lds = (size_t)TL::STAGES * StageBytes<T, TL::BM, TL::BN, X6B>::v;
  if (PRO) lds += (size_t)k.n_first_max * k.a.Cin * sizeof(T);
  lds = std::max(lds, (size_t)TL::EROWS * TL::ES * 4);
  lds = std::max(lds, (size_t)TL::NW * TL::BN * 4);
  if (lds > 160 * 1024) return set_error("conv: LDS budget exceeded");
  auto fn = conv_kernel<T, TL, PRO, SMALLC, EPI, X6B>;
  if (const int rc = ensure_dyn_lds((const void*)fn, 160 * 1024); rc != MIA_OK) return rc;
  k.prered = EPI >= 0 && (EPI & epi::CSUM);
  // X6B: s_setprio(1) around the MFMA blocks measured 1-2 % slower on this 2-blocks-per-CU tile
  k.prio = 0;
  // deterministic sums: contributor slots per (image, channel) (sums need one group, identity
  // placement: run_conv)
  const int HWo = k.g[0].ho * k.g[0].wo;
  int nslots;
  if constexpr (EPI >= 0) {  // register epilogue on the virtual (HWo/16 × 16) grid
    nslots = halo_red_slots(HWo / 16, 16, TL::FM, TL::WM, k.prered);
  } else {
    k.red_px = HWo % TL::BM != 0;
    nslots = k.red_px ? HWo : HWo / TL::BM;
  }
  RedQ r;
  int rc = conv_red_begin(k, r, nslots, st);
  if (rc != MIA_OK) return rc;
#ifdef MIA_DEBUG_LAUNCH  // diagnostic builds only (make variant): which tile / epilogue a launch takes
  fprintf(stderr, "MIA_LAUNCH conv_kernel bytes=%d BM=%d BN=%d PRO=%d SMALLC=%d EPI=%d X6B=%d "
                  "mask=%d N=%d H=%d W=%d Cin=%d Cout=%d stride=%d ng=%d ho=%d wo=%d\n",
          (int)sizeof(T), TL::BM, TL::BN, (int)PRO, (int)SMALLC, EPI, (int)X6B, epi_mask(k), k.a.N,
          k.a.H, k.a.W, k.a.Cin, k.a.Cout, k.stride, k.ng, k.g[0].ho, k.g[0].wo);
#endif
  hipLaunchKernelGGL(fn, dim3(blk), dim3(TL::NT), lds, st, k);
  rc = check_launch("conv");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

typedef Tile<2, 2, 4, 2, 2> Tile128x64;
typedef Tile<2, 2, 4, 4, 2> Tile128x128;
typedef Tile<2, 2, 2, 2, 2> Tile64x64;

// Register epilogue on the 128x128 tile: 2-byte types, one group, identity output placement,
// every tile inside one image (HWo % 128 == 0), the feature masks of the heavy short-K launches
// (the StyleGAN2 up-conv adjoint with its fused backward front; the e4e style-head convs).
// T_CONV_REGEPI = 0 disables (tests / tuning).
static int reg_epi_mask(const ConvK& k, int bytes) {
  (void)bytes;
  if (tune(T_CONV_REGEPI) == 0 || k.ng != 1 || k.batched || k.a.shuffle_out) return -1;
  const ConvGroup& G = k.g[0];
  if (G.ay != 1 || G.ax != 1 || G.by != 0 || G.bx != 0 || G.ho != k.HT || G.wo != k.WT ||
      (G.ho * G.wo) % 128 != 0)
    return -1;
  using namespace epi;
  const int f = epi_mask(k);
  switch (f) {
    case OSC | SDOT: case OSC | SDOT | ACC: case OSC | SDOT | BAB: case OSC | SDOT | ACC | BAB:
    case BIAS | PRELU:
    // the e4e encoder's stride-2 body convs and 1×1 shortcuts (folded BN: bias) and the FPN
    // laterals accumulating onto the up-sampled map
    case BIAS: case ACC: case BIAS | ACC:
      return f;
    default:
      return -1;
  }
}

template <typename T, bool PRO, bool SMALLC>
static int launch_bn(ConvK& k, hipStream_t st) {
  int64_t m = 0;
  for (int g = 0; g < k.ng; ++g) m += k.g[g].m;
  // (a 256x128 3-stage tile measured slower than 128x128 on every StyleGAN2 / VGG shape of the
  // 256² attack step — 2 blocks per CU hide each other's DMA waits better than 1 deeper ring —
  // and was removed in round 5)
  if (k.a.Cout <= 64) {
    // the 64-column tile with the specialised register epilogue for the same feature masks as
    // the 128-column tile below (the 512² StyledConv input gradients and the up-conv adjoints of
    // the 1024² generator: the LDS-staged generic epilogue with its sums cost ≈ as much as the
    // tile's short K loop)
    if constexpr (!PRO) {
      using namespace epi;
      switch (reg_epi_mask(k, sizeof(T))) {
        case OSC | SDOT: return launch_tile<T, Tile128x64, PRO, SMALLC, OSC | SDOT>(k, st);
        case OSC | SDOT | ACC:
          return launch_tile<T, Tile128x64, PRO, SMALLC, OSC | SDOT | ACC>(k, st);
        case OSC | SDOT | BAB:
          return launch_tile<T, Tile128x64, PRO, SMALLC, OSC | SDOT | BAB>(k, st);
        case OSC | SDOT | ACC | BAB:
          return launch_tile<T, Tile128x64, PRO, SMALLC, OSC | SDOT | ACC | BAB>(k, st);
        case BIAS | PRELU: return launch_tile<T, Tile128x64, PRO, SMALLC, BIAS | PRELU>(k, st);
        case BIAS: return launch_tile<T, Tile128x64, PRO, SMALLC, BIAS>(k, st);
        case ACC: return launch_tile<T, Tile128x64, PRO, SMALLC, ACC>(k, st);
        case BIAS | ACC: return launch_tile<T, Tile128x64, PRO, SMALLC, BIAS | ACC>(k, st);
        default: break;
      }
    }
    return launch_tile<T, Tile128x64, PRO, SMALLC>(k, st);
  }
  // Launches with fewer 128x128 tiles than 2 per CU (the e4e style heads at 8²…1² outputs,
  // K = 9·512) run one block per CU and serialise each wave's LDS reads, MFMAs and the step
  // barrier; 64x64 tiles put 4× the blocks (and waves) on the chip. T_CONV_SMALLTILE = the
  // 128x128-tile count below which this applies (T_CONV_SMALLTILE; 0 disables).
  int64_t tiles = 0;
  for (int g = 0; g < k.ng; ++g) tiles += (k.g[g].m + 127) / 128;
  tiles *= (k.a.Cout + 127) / 128;
  const int64_t small_below = tune(T_CONV_SMALLTILE);
  // (2-byte types only: fp32's small launches — the e4e style heads — have pre-split weights and
  // take the X6B 128×128 tile in launch_conv before reaching here; the 64×64 tile has no
  // pre-split-B form, and on the on-the-fly split it would double the split VALU per MFMA)
  if (sizeof(T) == 2 && tiles < small_below) return launch_tile<T, Tile64x64, PRO, SMALLC>(k, st);
  // fp32 modulated-input launches of < 128 128×128 tiles (the generator's first StyledConv, 4²:
  // 64 tiles, one block per four CUs on the K = 9·512 loop) on 64×64 tiles: 352 → 186 µs per
  // call. From 256 tiles on (the 8² StyledConv, the 4 → 8 and 8 → 16 up-convs, the up-conv
  // edges) the 64×64 tile's doubled split VALU per MFMA costs more than its blocks gain
  // (profiles/r06_f32_small_pro_tile_ab.txt)
  if (sizeof(T) == 4 && PRO && tiles < MIA_F32_PRO_SMALLTILE)
    return launch_tile<T, Tile64x64, PRO, SMALLC>(k, st);
  if constexpr (!SMALLC && !PRO) {
    using namespace epi;
    switch (reg_epi_mask(k, sizeof(T))) {
      case OSC | SDOT: return launch_tile<T, Tile128x128, PRO, SMALLC, OSC | SDOT>(k, st);
      case OSC | SDOT | ACC: return launch_tile<T, Tile128x128, PRO, SMALLC, OSC | SDOT | ACC>(k, st);
      case OSC | SDOT | BAB: return launch_tile<T, Tile128x128, PRO, SMALLC, OSC | SDOT | BAB>(k, st);
      case OSC | SDOT | ACC | BAB:
        return launch_tile<T, Tile128x128, PRO, SMALLC, OSC | SDOT | ACC | BAB>(k, st);
      case BIAS | PRELU: return launch_tile<T, Tile128x128, PRO, SMALLC, BIAS | PRELU>(k, st);
      case BIAS: return launch_tile<T, Tile128x128, PRO, SMALLC, BIAS>(k, st);
      case ACC: return launch_tile<T, Tile128x128, PRO, SMALLC, ACC>(k, st);
      case BIAS | ACC: return launch_tile<T, Tile128x128, PRO, SMALLC, BIAS | ACC>(k, st);
      default: break;
    }
  }
  return launch_tile<T, Tile128x128, PRO, SMALLC>(k, st);
}

// fp32, every group pre-split, unmodulated, Cin ≥ 32, Cout > 64: the X6B 128×128 tile (2 stages,
// exactly 80 KB of LDS, 2 blocks per CU): e4e style-head convs 155 / 175 TFLOP/s vs 142 / 150 on
// the on-the-fly split (64²→32² / 32²→16², 512 → 512). At Cout ≤ 64 (128×64 tile, two B
// fragments per wave) it measured 2–11 % slower and is not used. MIA_CONV_X6=0 disables (A/B).
static bool x6b_ok(const ConvK& k) {
#ifdef MIA_F32_NATIVE
  (void)k;
  return false;
#else
  if (tune(T_CONV_X6) == 0) return false;
  for (int g = 0; g < k.ng; ++g)
    if (!k.g[g].w_split) return false;
  return k.a.in_scale == nullptr && k.a.act_in == MIA_ACT_NONE && k.a.Cin >= 32 && k.a.Cout > 64;
#endif
}

template <typename T>
static int launch_conv(ConvK& k, hipStream_t st) {
  if constexpr (std::is_same<T, float>::value) {
    if (x6b_ok(k)) {
      // the specialised register epilogues where they apply (the up-conv adjoints with their
      // fused backward front, the style-head convs), else the LDS-staged one
      using namespace epi;
      switch (reg_epi_mask(k, 4)) {
        case OSC | SDOT: return launch_tile<T, Tile128x128, false, false, OSC | SDOT, true>(k, st);
        case OSC | SDOT | ACC:
          return launch_tile<T, Tile128x128, false, false, OSC | SDOT | ACC, true>(k, st);
        case OSC | SDOT | BAB:
          return launch_tile<T, Tile128x128, false, false, OSC | SDOT | BAB, true>(k, st);
        case OSC | SDOT | ACC | BAB:
          return launch_tile<T, Tile128x128, false, false, OSC | SDOT | ACC | BAB, true>(k, st);
        case BIAS | PRELU: return launch_tile<T, Tile128x128, false, false, BIAS | PRELU, true>(k, st);
        case BIAS: return launch_tile<T, Tile128x128, false, false, BIAS, true>(k, st);
        case ACC: return launch_tile<T, Tile128x128, false, false, ACC, true>(k, st);
        case BIAS | ACC: return launch_tile<T, Tile128x128, false, false, BIAS | ACC, true>(k, st);
        default: break;
      }
      return launch_tile<T, Tile128x128, false, false, -2, true>(k, st);
    }
  }
  const bool pro = k.a.in_scale != nullptr || k.a.act_in != MIA_ACT_NONE;
  const bool small = k.a.Cin < ROWB / (int)sizeof(T);
  if (pro) return small ? launch_bn<T, true, true>(k, st) : launch_bn<T, true, false>(k, st);
  return small ? launch_bn<T, false, true>(k, st) : launch_bn<T, false, false>(k, st);
}

int conv_red_begin(ConvK& k, RedQ& r, int nslots, hipStream_t st, bool zero) {
  const mia_conv_args& a = k.a;
  const int count = a.N * a.Cout;
  const int rc = red_begin(r, a.sdot, a.bab_demod ? a.bab_q : nullptr, a.csum, nslots, count, st,
                           zero);
  k.red_part = r.part;
  k.red_nslots = nslots;
  k.red_count = count;
  return rc;
}

static int bk_for(int dtype) { return dtype == MIA_F32 ? 32 : 64; }

// the up-conv edge groups on their leading (in-range) taps only; tuning A/B: =0 the full windows
#ifndef MIA_UPCONV_EDGE_TRIM
#define MIA_UPCONV_EDGE_TRIM 1
#endif

static int kpad_for(int k, int dtype) {
  const int bk = bk_for(dtype);
  return (k + bk - 1) / bk * bk;
}

// Shared validation + dispatch for a filled ConvK (groups set up by the caller).
static int run_conv(ConvK& k, int dtype, hipStream_t st) {
  const mia_conv_args& a = k.a;
  MIA_CHECK_ARG(a.x, "x is required");
  MIA_CHECK_ARG(a.N > 0 && a.H > 0 && a.W > 0 && a.Cin > 0 && a.Cout > 0, "bad shape");
  MIA_CHECK_ARG(dtype == MIA_F32 || dtype == MIA_F16 || dtype == MIA_BF16, "bad dtype");
  const int vec = dtype == MIA_F32 ? 4 : 8;
  MIA_CHECK_ARG(a.Cin >= vec && (a.Cin & (a.Cin - 1)) == 0,
                "Cin must be a power of two ≥ the 16-byte vector");
  MIA_CHECK_ARG(a.Cout % 8 == 0, "Cout must be a multiple of 8");
  MIA_CHECK_ARG(!a.shuffle_out || (a.Cout % 32 == 0 && k.ng == 1), "shuffle_out: Cout % 32, 1 group");
  MIA_CHECK_ARG(!a.sdot || a.aux_x, "sdot needs aux_x");
  MIA_CHECK_ARG(!a.bab_demod || (a.aux_x && a.act_aux == MIA_ACT_NONE && a.bab_q && a.y &&
                                 !a.shuffle_out),
                "bab_demod needs aux_x (stored activations, act_aux NONE), bab_q and y");
  MIA_CHECK_ARG(!a.tap_a || a.tap_t, "tap_a needs tap_t");
  MIA_CHECK_ARG(a.act_out != MIA_ACT_PRELU || a.act_slope, "MIA_ACT_PRELU needs act_slope");
  MIA_CHECK_ARG(!a.csum || (a.y && !a.shuffle_out && k.ng == 1 &&
                             k.g[0].ho * k.g[0].wo == k.HT * k.WT),
                "csum needs y (un-shuffled), one group with an identity output placement");
  MIA_CHECK_ARG(!a.shuffle_out || !(a.tap_a || a.mask_a || a.sdot),
                "aux inputs need un-shuffled output");
  MIA_CHECK_ARG((int64_t)a.N * a.H * a.W * a.Cin < (1LL << 31), "input too large for 32-bit offsets");
  MIA_CHECK_ARG(a.in_scale == nullptr || a.Cin <= 2048, "modulated Cin ≤ 2048");
  MIA_CHECK_ARG(k.ng >= 1 && k.ng <= (k.batched ? MIA_MAX_GROUPS : 4), "1..4 groups (16 batched)");
  for (int g = 0; g < k.ng; ++g) {
    const ConvGroup& G = k.g[g];
    MIA_CHECK_ARG(G.w, "w is required");
    MIA_CHECK_ARG(G.kh >= 1 && G.kh <= 3 && G.kw >= 1 && G.kw <= 3, "taps 1..3");
    MIA_CHECK_ARG(G.kpad >= kpad_for(G.kh * G.kw * a.Cin, dtype) && G.kpad % bk_for(dtype) == 0,
                  "Kpad must be mia_conv_kpad()");
    MIA_CHECK_ARG(G.ho > 0 && G.wo > 0, "empty output grid");
    MIA_CHECK_ARG((int64_t)a.N * G.ho * G.wo < (1LL << 31), "too many pixels");
    MIA_CHECK_ARG(!(a.sdot || a.bab_demod) || (k.ng == 1 && G.ho * G.wo == k.HT * k.WT),
                  "sdot / bab need one group with an identity output placement");
    MIA_CHECK_ARG(G.ay * (G.ho - 1) + G.by < k.HT && G.ax * (G.wo - 1) + G.bx < k.WT &&
                      G.by >= 0 && G.bx >= 0,
                  "output placement outside the output grid");
  }
  int lc = 0;
  while ((1 << lc) < a.Cin) ++lc;
  k.log2cin = lc;
  int hw_min = 1 << 30;
  for (int g = 0; g < k.ng; ++g) hw_min = std::min(hw_min, k.g[g].ho * k.g[g].wo);
  k.n_first_max = std::min(a.N, (256 + hw_min - 1) / hw_min + 1);

  if (k.batched) {  // the generic tile only (its LDS-staged epilogue applies the offsets)
    MIA_CHECK_ARG(!a.shuffle_out && !a.sdot && !a.bab_demod && !a.csum,
                  "batched groups: no shuffle_out / sdot / bab / csum");
    MIA_DISPATCH_DTYPE(dtype, T, return launch_conv<T>(k, st));
  }
  if (conv_thin_eligible(k, dtype)) return launch_conv_thin(k, dtype, st);
  if (conv_wres32_eligible(k, dtype)) return launch_conv_wres32(k, dtype, st);
  if (conv_thin32_eligible(k, dtype)) return launch_conv_thin32(k, dtype, st);
  if (conv_wres_eligible(k, dtype)) return launch_conv_wres(k, dtype, st);
  if (conv_wres128_eligible(k, dtype)) return launch_conv_wres128(k, dtype, st);
  if (conv_halo_x6_eligible(k, dtype)) return launch_conv_halo_x6(k, st);
  if (conv_halo_eligible(k, dtype)) return launch_conv_halo(k, dtype, st);
  MIA_DISPATCH_DTYPE(dtype, T, return launch_conv<T>(k, st));
  return MIA_OK;
}

}  // namespace mia

using namespace mia;

extern "C" int mia_conv_kpad(int cin, int dtype) { return kpad_for(9 * cin, dtype); }

extern "C" int mia_conv3x3(const mia_conv_args* args, int dtype, void* stream) {
  MIA_CHECK_ARG(args != nullptr, "null args");
  const mia_conv_args& a = *args;
  MIA_CHECK_ARG(a.Kpad == kpad_for(9 * a.Cin, dtype), "Kpad must be mia_conv_kpad()");
  ConvK k = {};
  k.a = a;
  k.stride = 1;
  k.ng = 1;
  ConvGroup& G = k.g[0];
  G.w = a.w;
  G.w_split = a.w_split;
  G.kpad = a.Kpad;
  G.kh = G.kw = 3;
  G.pad_y = G.pad_x = 1;
  G.ho = a.H;
  G.wo = a.W;
  G.ay = G.ax = 1;
  G.m = pixels_clamped(a.N, a.H, a.W);
  k.HT = a.shuffle_out ? 2 * a.H : a.H;
  k.WT = a.shuffle_out ? 2 * a.W : a.W;
  k.cout_mod = a.shuffle_out ? a.Cout / 4 : a.Cout;
  k.ystride = a.y_cstride > 0 ? a.y_cstride : k.cout_mod;
  MIA_CHECK_ARG(k.ystride >= k.cout_mod, "y_cstride < Cout");
  return run_conv(k, dtype, (hipStream_t)stream);
}

extern "C" int mia_conv2d_kpad(int taps, int cin, int dtype) { return kpad_for(taps * cin, dtype); }

static int conv2d_impl(const mia_conv_args* args, int stride, const mia_conv_group* groups,
                       const mia_conv_batch* batch, int ngroups, int out_h, int out_w, int dtype,
                       void* stream, int ysplit = 0, int64_t yplane = 0);

extern "C" int mia_conv2d(const mia_conv_args* args, int stride, const mia_conv_group* groups,
                          int ngroups, int out_h, int out_w, int dtype, void* stream) {
  MIA_CHECK_ARG(ngroups >= 1 && ngroups <= 4, "1..4 groups");
  return conv2d_impl(args, stride, groups, nullptr, ngroups, out_h, out_w, dtype, stream);
}

extern "C" int mia_conv2d_batched(const mia_conv_args* args, int stride,
                                  const mia_conv_group* groups, const mia_conv_batch* batch,
                                  int ngroups, int out_h, int out_w, int dtype, void* stream) {
  MIA_CHECK_ARG(batch != nullptr, "null batch");
  MIA_CHECK_ARG(ngroups >= 1 && ngroups <= MIA_MAX_GROUPS, "1..16 groups");
  for (int g = 0; g < ngroups; ++g)
    MIA_CHECK_ARG(batch[g].n_in >= 0 && batch[g].n_out >= 0 && batch[g].c_off >= 0 &&
                      batch[g].c_off % 8 == 0,
                  "batch offsets must be ≥ 0 (c_off a multiple of 8)");
  return conv2d_impl(args, stride, groups, batch, ngroups, out_h, out_w, dtype, stream);
}

extern "C" int mia_conv2d_planes(const mia_conv_args* args, int stride,
                                 const mia_conv_group* groups, int out_h, int out_w,
                                 int plane_channels, int64_t plane_stride, int dtype,
                                 void* stream) {
  MIA_CHECK_ARG(args != nullptr && groups != nullptr, "null args");
  const mia_conv_args& a = *args;
  MIA_CHECK_ARG(stride == 2, "plane-split output: the stride-2 convs (generic tile) only");
  MIA_CHECK_ARG(plane_channels > 0 && plane_channels % 128 == 0 && a.Cout % plane_channels == 0,
                "plane_channels must be a multiple of 128 dividing Cout");
  MIA_CHECK_ARG(a.y_cstride == 0 || a.y_cstride == plane_channels, "y_cstride = plane_channels");
  MIA_CHECK_ARG(plane_stride >= (int64_t)a.N * out_h * out_w * plane_channels,
                "plane_stride < N·out_h·out_w·plane_channels");
  MIA_CHECK_ARG(a.y && !a.sdot && !a.bab_demod && !a.csum && !a.mask_a && !a.tap_a && !a.aux_x &&
                    !a.accumulate && !a.out_scale && !a.noise,
                "plane-split output: bias / act epilogues only");
  return conv2d_impl(args, stride, groups, nullptr, 1, out_h, out_w, dtype, stream,
                     plane_channels, plane_stride);
}

static int conv2d_impl(const mia_conv_args* args, int stride, const mia_conv_group* groups,
                       const mia_conv_batch* batch, int ngroups, int out_h, int out_w, int dtype,
                       void* stream, int ysplit, int64_t yplane) {
  MIA_CHECK_ARG(args != nullptr && groups != nullptr, "null args");
  MIA_CHECK_ARG(stride == 1 || stride == 2, "stride 1 or 2");
  MIA_CHECK_ARG(out_h > 0 && out_w > 0, "empty output");
  MIA_CHECK_ARG(!args->shuffle_out, "shuffle_out is a mia_conv3x3 feature");
  const mia_conv_args& a = *args;
  ConvK k = {};
  k.a = a;
  k.stride = stride;
  k.ng = ngroups;
  k.batched = batch != nullptr;
  k.HT = out_h;
  k.WT = out_w;
  k.cout_mod = a.Cout;
  k.ystride = a.y_cstride > 0 ? a.y_cstride : a.Cout;
  k.ysplit = ysplit;
  k.yplane = yplane;
  if (ysplit > 0) k.ystride = ysplit;  // each plane holds ysplit channels per pixel
  MIA_CHECK_ARG(ysplit > 0 || k.ystride >= a.Cout, "y_cstride < Cout");
  for (int g = 0; g < ngroups; ++g) {
    const mia_conv_group& s = groups[g];
    ConvGroup& G = k.g[g];
    G.w = s.w;
    G.w_split = s.w_split;
    G.kh = s.kh;
    G.kw = s.kw;
    G.kpad = kpad_for(s.kh * s.kw * a.Cin, dtype);
    G.pad_y = s.pad_y;
    G.pad_x = s.pad_x;
    G.ho = s.ho;
    G.wo = s.wo;
    G.ay = s.ay;
    G.by = s.by;
    G.ax = s.ax;
    G.bx = s.bx;
    G.m = pixels_clamped(a.N, s.ho, s.wo);
    if (batch) {
      G.n_in = batch[g].n_in;
      G.n_out = batch[g].n_out;
      G.c_off = batch[g].c_off;
    }
  }
  return run_conv(k, dtype, (hipStream_t)stream);
}

extern "C" int mia_upconv_kpad(int cin, int phase, int dtype) {
  const int kh = 2 - (phase >> 1), kw = 2 - (phase & 1);
  return kpad_for(kh * kw * cin, dtype);
}

extern "C" int mia_upconv_fwd(const void* x, const void* const* w_phase, void* t_out, int N,
                              int R, int Cin, int Cout, int act_in, const float* style, int dtype,
                              void* stream) {
  MIA_CHECK_ARG(w_phase && t_out, "bad args");
  mia_conv_args a = {};
  a.x = x; a.y = t_out; a.N = N; a.H = R; a.W = R; a.Cin = Cin; a.Cout = Cout;
  a.act_in = act_in; a.in_scale = style;
  ConvK k = {};
  k.a = a;
  k.stride = 1;
  k.ng = 4;
  k.HT = k.WT = 2 * R + 1;
  k.cout_mod = Cout;
  k.ystride = Cout;
  for (int ph = 0; ph < 4; ++ph) {
    const int py = ph >> 1, px = ph & 1;
    ConvGroup& G = k.g[ph];
    G.w = w_phase[ph];
    G.kh = 2 - py;
    G.kw = 2 - px;
    G.kpad = kpad_for(G.kh * G.kw * Cin, dtype);
    G.pad_y = G.kh - 1;
    G.pad_x = G.kw - 1;
    G.ho = R + 1 - py;
    G.wo = R + 1 - px;
    G.ay = G.ax = 2;
    G.by = py;
    G.bx = px;
    G.m = pixels_clamped(N, G.ho, G.wo);
  }
  return run_conv(k, dtype, (hipStream_t)stream);
}

extern "C" int mia_upconv_fwd_halo(const void* x, const void* const* w_phase, const void* w_up,
                                   void* t_out, int N, int R, int Cin, int Cout, int act_in,
                                   const float* style, int dtype, void* stream) {
  return mia_upconv_fwd_halo_split(x, w_phase, w_up, nullptr, t_out, N, R, Cin, Cout, act_in, style,
                                   dtype, stream);
}

extern "C" int mia_upconv_fwd_halo_split(const void* x, const void* const* w_phase,
                                         const void* w_up, const void* w_up_split, void* t_out,
                                         int N, int R, int Cin, int Cout, int act_in,
                                         const float* style, int dtype, void* stream) {
  if (!w_up || !upconv_halo_eligible(dtype, R, Cin, Cout))
    return mia_upconv_fwd(x, w_phase, t_out, N, R, Cin, Cout, act_in, style, dtype, stream);
  MIA_CHECK_ARG(x && w_phase && t_out && N > 0 && Cout % 8 == 0, "bad args");
  MIA_CHECK_ARG((int64_t)N * R * R * Cin < (1LL << 31), "input too large for 32-bit offsets");
  const int rc = launch_upconv_halo(x, w_up, w_up_split, t_out, N, R, Cin, Cout, act_in, style,
                                    dtype, (hipStream_t)stream);
  if (rc) return rc;
  // the last row / column of the even phase grids (y = R or x = R): four one-row / one-column
  // groups on the generic kernel; the group's input window starts at R − 1 (pad = 1 − R) and its
  // outputs land at T row / column 2R
  mia_conv_args a = {};
  a.x = x; a.y = t_out; a.N = N; a.H = R; a.W = R; a.Cin = Cin; a.Cout = Cout;
  a.act_in = act_in; a.in_scale = style;
  ConvK k = {};
  k.a = a;
  k.stride = 1;
  k.ng = 4;
  k.HT = k.WT = 2 * R + 1;
  k.cout_mod = Cout;
  k.ystride = Cout;
  // {phase, row group?}: (0,0) row y = R (x ∈ [0,R]), (0,1) row y = R (x ∈ [0,R)),
  //                      (0,0) column x = R (y ∈ [0,R)), (1,0) column x = R (y ∈ [0,R)).
  // Only the window's first tap row (row groups) / column (columns) lies inside the input; where
  // those taps lead the weight row (both row groups, the (1,0) column) the group runs just them
  // (kh or kw = 1, the row stride kept in kpad): the MFMAs on the zero taps are skipped, the
  // sums unchanged (each skipped product was an exact zero). The (0,0) column's valid taps
  // (t = 0, 2) are not contiguous in K and keep the full window.
  const int phs[4] = {0, 1, 0, 2};
  const bool rowg[4] = {true, true, false, false};
  for (int g = 0; g < 4; ++g) {
    const int ph = phs[g], py = ph >> 1, px = ph & 1;
    ConvGroup& G = k.g[g];
    G.w = w_phase[ph];
    G.kh = 2 - py;
    G.kw = 2 - px;
    G.kpad = kpad_for(G.kh * G.kw * Cin, dtype);
    G.ay = G.ax = 2;
    if (rowg[g]) {
      G.ho = 1; G.wo = R + 1 - px;
      G.pad_y = (G.kh - 1) - R; G.pad_x = G.kw - 1;
      G.by = 2 * R + py; G.bx = px;
      if (MIA_UPCONV_EDGE_TRIM) G.kh = 1;  // taps ty = 0 (input row R − 1) lead the row
    } else {
      G.ho = R; G.wo = 1;
      G.pad_y = G.kh - 1; G.pad_x = (G.kw - 1) - R;
      G.by = py; G.bx = 2 * R + px;
      if (MIA_UPCONV_EDGE_TRIM && G.kh == 1) G.kw = 1;  // tap tx = 0 (input column R − 1)
    }
    G.m = pixels_clamped(N, G.ho, G.wo);
  }
  return run_conv(k, dtype, (hipStream_t)stream);
}

static int upconv_dgrad_impl(const mia_conv_args& a, const void* w_t, int N, int R, int Cout,
                             int Cin, int dtype, void* stream);

extern "C" int mia_upconv_dgrad(const void* g_t, const void* w_t, void* gx, int N, int R, int Cout,
                                int Cin, const void* x_fwd, int act_x, const float* style,
                                float* sdot, int dtype, void* stream) {
  mia_conv_args a = {};
  a.x = g_t; a.y = gx; a.N = N; a.H = 2 * R + 1; a.W = 2 * R + 1; a.Cin = Cout; a.Cout = Cin;
  a.out_scale = style; a.aux_x = x_fwd; a.act_aux = act_x; a.sdot = sdot;
  return upconv_dgrad_impl(a, w_t, N, R, Cout, Cin, dtype, stream);
}

extern "C" int mia_upconv_dgrad_fused(const void* g_t, const void* w_t, void* gx, int N, int R,
                                      int Cout, int Cin, const void* x_fwd, const float* style,
                                      float* sdot, int accumulate, const float* bab_demod,
                                      const float* bab_noise, float bab_noise_w,
                                      const float* bab_bias, float* bab_q, int dtype,
                                      void* stream) {
  return mia_upconv_dgrad_fused_split(g_t, w_t, nullptr, gx, N, R, Cout, Cin, x_fwd, style, sdot,
                                      accumulate, bab_demod, bab_noise, bab_noise_w, bab_bias,
                                      bab_q, dtype, stream);
}

extern "C" int mia_upconv_dgrad_fused_split(const void* g_t, const void* w_t,
                                            const void* w_t_split, void* gx, int N, int R,
                                            int Cout, int Cin, const void* x_fwd,
                                            const float* style, float* sdot, int accumulate,
                                            const float* bab_demod, const float* bab_noise,
                                            float bab_noise_w, const float* bab_bias, float* bab_q,
                                            int dtype, void* stream) {
  mia_conv_args a = {};
  a.w_split = w_t_split;
  a.x = g_t; a.y = gx; a.N = N; a.H = 2 * R + 1; a.W = 2 * R + 1; a.Cin = Cout; a.Cout = Cin;
  a.out_scale = style; a.aux_x = x_fwd; a.act_aux = MIA_ACT_NONE; a.sdot = sdot;
  a.accumulate = accumulate;
  a.bab_demod = bab_demod; a.bab_noise = bab_noise; a.bab_noise_w = bab_noise_w;
  a.bab_bias = bab_bias; a.bab_q = bab_q;
  return upconv_dgrad_impl(a, w_t, N, R, Cout, Cin, dtype, stream);
}

static int upconv_dgrad_impl(const mia_conv_args& a, const void* w_t, int N, int R, int Cout,
                             int Cin, int dtype, void* stream) {
  ConvK k = {};
  k.a = a;
  k.stride = 2;
  k.ng = 1;
  ConvGroup& G = k.g[0];
  G.w = w_t;
  G.w_split = a.w_split;
  G.kh = G.kw = 3;
  G.kpad = kpad_for(9 * Cout, dtype);
  G.pad_y = G.pad_x = 0;
  G.ho = G.wo = R;
  G.ay = G.ax = 1;
  G.m = pixels_clamped(N, R, R);
  k.HT = k.WT = R;
  k.cout_mod = Cin;
  k.ystride = Cin;
  return run_conv(k, dtype, (hipStream_t)stream);
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

extern "C" int mia_vgg_conv_relu_dgrad(const void* g, const void* w_t, void* gx, int N, int H,
                                       int W, int Cin_g, int Cout_g, int Kpad, const void* tap_a,
                                       const void* tap_t, float tap_coef, const void* mask_a,
                                       int dtype, void* stream) {
  return mia_vgg_conv_dgrad(g, w_t, gx, N, H, W, Cin_g, Cout_g, Kpad, tap_a, tap_t, tap_coef,
                            mask_a, dtype, stream);
}
