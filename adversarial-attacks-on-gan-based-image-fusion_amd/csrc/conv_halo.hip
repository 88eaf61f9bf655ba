// Halo-tiled implicit-GEMM convolution for the stride-1, pad-1 3×3 layers (NHWC), CDNA4 MFMA.
//
// Serves the bulk of the attack step's FLOPs (SURVEY.md §2.1 K1, K7, K15 at 16²…256²): VGG conv
// forward and input-gradient, StyledConv forward (modulation on the A fragments, demodulation in
// the epilogue) and StyledConv input/style gradient. Up-sampling convs and the stride-2 adjoint
// stay on the generic im2col kernel (conv_mfma.hip).
//
// Why a second kernel: the generic kernel re-gathers every input pixel once per tap (9× the
// activation bytes through the LDS-DMA path), and a CU fills LDS at only ≈70 GB/s from L2
// (MI355X_MICROARCH.md, gather-into-LDS table), which caps a 128×128 im2col tile at ≈64 FLOP per
// staged byte ≈ 45 % of the MFMA peak. Here a block owns a 16×16 output patch of one image:
//   * per 64-channel block (BK), the (16+2)×(16+2) input halo is DMA'd once into LDS and read by
//     all 9 taps (A traffic ÷ 7 vs im2col);
//   * the weights stream per (tap, channel block) K-step through a 3-stage ring with two K-steps
//     in flight behind a counted vmcnt;
//   * the next channel block's halo is DMA'd into the other halo buffer one piece per wave per
//     K-step during the first taps of the current block.
// GEMM view: M = 256 patch pixels (wave wm owns patch rows 4·wm … 4·wm+3, one MFMA fragment per
// row), N = BN output channels (64 or 128), K = 9·Cin in (channel block, tap) order; the weight
// matrix is the same tap-major [Cout][Kpad] layout as the generic kernel, so only the K-offset of
// a step differs. The epilogue (demod, noise, bias, tap-MSE, ReLU mask, act, sdot) is shared.
#include <cstring>

#include "conv_common.h"
#include "halo_epilogue.h"

// PRO launches: 1 = the landed halo modulated once in LDS (default); 0 = every fragment read
// modulated (round-2 form, tuning A/B: `make variant VARIANT_FLAGS=-DMIA_HALO_PREMOD=0`).
#ifndef MIA_HALO_PREMOD
#define MIA_HALO_PREMOD 1
#endif


namespace mia {

// Tile: a PH × 16 output patch (PH = 16: 8 waves, 1 block per CU; PH = 8: 4 waves, 2 blocks per
// CU so that one block's prologue/epilogue overlaps the other's main loop) × BN output channels.
// Each wave owns FM = 4 patch rows (one 16-pixel MFMA fragment per row) × BN/2 channels.
// NHBUF = 1: a single halo buffer, for Cin = one channel block only (no next-block prefetch).
// FM = 8: each wave owns 8 patch rows (a 16×16 patch on 4 waves, one block per CU): the weights
// staged per K-step feed twice the MFMAs.
template <int BN_, int PH_, int STAGES_, int NHBUF_ = 2, int FM_ = 4>
struct HaloTile {
  static constexpr int FM = FM_, WM = PH_ / FM_, WN = 2, FN = BN_ / 32;
  static constexpr int PH = PH_, PW = 16, NW = WM * WN, NT = 64 * NW, BM = PH * PW, BN = BN_;
  static constexpr int WAVES_PER_SIMD = (NW == 4 && FM == 4) ? 2 : 1;  // launch-bounds hint
  static constexpr int STAGES = STAGES_;
  static constexpr int NHBUF = NHBUF_;
  static constexpr int HW = PW + 2, HROWS = (PH + 2) * HW;  // 324 / 180 halo pixels
  static constexpr int HPIECES = (HROWS + 7) / 8;          // DMA pieces of 8 rows (1 KB)
  static constexpr int HBUF = HPIECES * 8 * ROWB;          // per halo buffer
  // DMA roles: the first half of the waves stream the weights, the second half the halos.
  // vmcnt retires in issue order, so a wave that mixed both would hold every L2-fast weight
  // piece behind an HBM-slow halo piece.
  static constexpr int BWAVES = NW / 2, HWAVES = NW - BWAVES;
  static constexpr int B_INS = BN / (8 * BWAVES);                // weight pieces per B-wave per step
  static constexpr int H_INS = (HPIECES + HWAVES - 1) / HWAVES;  // halo pieces per H-wave
  static constexpr int H_PER_STEP = (H_INS + 3) / 4;             // next-block halo by tap 3
  static constexpr int BSTAGE = BN * ROWB;
  static constexpr int EROWS = BM < 128 ? BM : 128, ES = BN + 4;  // shared epilogue staging
  static_assert(B_INS >= 1 && B_INS * 8 * BWAVES == BN, "");
  static_assert(WM * FM * 16 == BM && WN * FN * 16 == BN, "");
};

#ifdef MIA_HALO_TIMING
// phase cycle sums of wave 0 over all blocks (tuning builds only: scratch/, never shipped)
// one row per 4096th block: the atomics of one launch spread over 4096 addresses (a single row
// serialised every block's end on 8 addresses and slowed the launch 4×)
constexpr int HT_SLOTS = 4096;
__device__ unsigned long long g_halo_dbg[HT_SLOTS][8];
#define HT_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define HT_STAMP(v)
#endif
#if defined(MIA_HALO_TIMING) && !defined(MIA_HALO_TIMING_COARSE)
#define HT_STEP_STAMP(v) HT_STAMP(v)
#define HT_STEPS 1
#else
#define HT_STEP_STAMP(v)
#define HT_STEPS 0
#endif

// EPI: −2 = LDS-staged shared epilogue (conv_epilogue), −1 = register epilogue with runtime
// features (halo_epilogue), ≥ 0 = register epilogue specialised for feature mask EPI.
template <typename T, typename TL, bool PRO, int EPI>
__global__ __launch_bounds__(TL::NT, TL::WAVES_PER_SIMD) void conv_halo_kernel(const ConvK k) {
  HT_STAMP(t_start);
  typedef typename Vec<T>::type VT;
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = ROWB / (int)sizeof(T);
  constexpr int WN = TL::WN, FM = TL::FM, FN = TL::FN, NT = TL::NT, BN = TL::BN;
  constexpr int H_INS = TL::H_INS, B_INS = TL::B_INS, HBUF = TL::HBUF, BSTAGE = TL::BSTAGE;
  constexpr int STAGES = TL::STAGES, PH = TL::PH, PW = TL::PW, HSIDE = TL::HW, HROWS = TL::HROWS;
  constexpr int HPIECES = TL::HPIECES, BWAVES = TL::BWAVES, HWAVES = TL::HWAVES;
  constexpr int HPS = TL::H_PER_STEP;

  // AUXP: the StyledConv forward (demod, noise, bias, lrelu — modulated input, or per-image
  // modulated weights without the demod) prefetches its epilogue operands into the free halo
  // buffer during the last channel block
  constexpr bool AUXP = ((PRO && EPI == (epi::OSC | epi::NOISE | epi::BIAS | epi::LRELU)) ||
                         (!PRO && EPI == (epi::NOISE | epi::BIAS | epi::LRELU))) &&
                        TL::NHBUF == 2 && TL::BN == 128 && TL::FM <= 4;
  constexpr int AUX_OFF = 4096;  // past the LDS pre-reduction rows (3 × WM × BN floats)
  static_assert(!AUXP || (AUX_OFF + 2048 <= TL::HBUF && 3 * TL::WM * TL::BN * 4 <= AUX_OFF &&
                          4 * TL::PH <= 32),
                "aux prefetch layout");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                        // 2 halo buffers
  char* const bring = smem + TL::NHBUF * HBUF;    // weight ring
  T* const stab = (T*)(bring + STAGES * BSTAGE);  // PRO: style row of the patch's image

  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const ConvGroup G = k.g[0];
  const int H = p.H, W = p.W, Cin = p.Cin, Cout = p.Cout;
  const int bl = xcd_remap(blockIdx.x, k.nblk);
  const int mt = bl / k.nbn, n0 = (bl % k.nbn) * BN;
  const int ptx = W / PW, pty = H / PH;
  const int x0 = (mt % ptx) * PW;
  const int y0 = ((mt / ptx) % pty) * PH;
  const int n = mt / (ptx * pty);

  const T* __restrict__ X = (const T*)p.x;
  const T* __restrict__ Wt = (const T*)G.w + (size_t)n * k.wn;  // per-image weights (wmod)
  const T* zero = (const T*)g_zero16;
  const bool bwave = wid < BWAVES;  // wave-uniform role
  const int hw = wid - BWAVES;      // H-wave index
  const int my_pieces = bwave ? 0 : (HPIECES - hw + HWAVES - 1) / HWAVES;

  // ---- per-lane DMA sources ------------------------------------------------------------------
  // H-wave hw owns halo pieces hw + 4·j (8 halo rows each); B-wave w owns weight rows
  // (w·B_INS + j)·8 + lane/8. Lane → (row, 16-B chunk), the chunk swizzled through the source so
  // that the lane-linear LDS image is bank-swizzled (fsw).
  const T* src[H_INS > B_INS ? H_INS : B_INS];
  constexpr int NSRC = H_INS > B_INS ? H_INS : B_INS;
#pragma unroll
  for (int j = 0; j < NSRC; ++j) {
    src[j] = nullptr;
    if (bwave) {
      if (j < B_INS) {
        const int row = (wid * B_INS + j) * 8 + (lane >> 3);
        if (n0 + row < Cout)
          src[j] = Wt + (size_t)(n0 + row) * G.kpad + ((lane & 7) ^ fsw(row)) * VEC;
      }
    } else if (j < H_INS) {
      const int hr = (hw + HWAVES * j) * 8 + (lane >> 3);
      const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
      const int y = y0 + hy - 1, x = x0 + hx - 1;
      if (hr < HROWS && y >= 0 && y < H && x >= 0 && x < W)
        src[j] = X + ((size_t)(n * H + y) * W + x) * Cin + ((lane & 7) ^ fsw(hr)) * VEC;
    }
  }
  const int ncb = Cin / BK, nk = 9 * ncb;
  auto issue_b = [&](int s, int st) {  // B-wave: its weight pieces of K-step s = (cb, tap)
    const int cb = s / 9, t = s - (s / 9) * 9;
    const int koff = t * Cin + cb * BK;
    char* dst = bring + st * BSTAGE;
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const T* a = src[j] ? src[j] + koff : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)a, (lptr_t)(dst + (wid * B_INS + j) * 1024), 16, 0,
                                       0);
    }
  };
  auto issue_h = [&](int cb, int j, int buf) {  // H-wave: its halo piece j of channel block cb
    const T* a = src[j] ? src[j] + cb * BK : zero;
    __builtin_amdgcn_global_load_lds((gptr_t)a,
                                     (lptr_t)(hbuf + buf * HBUF + (hw + HWAVES * j) * 1024), 16,
                                     0, 0);
  };

  // PRO: modulate the landed halo of channel block cb (buffer buf) in place ONCE — act(x)·s
  // rounded to T exactly as modulate<T> would on every fragment read (9 taps × 2 column waves).
  // Zero padding stays zero.
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;
  auto premod = [&](int cb, int buf) {
    char* hb = hbuf + buf * HBUF;
    for (int c = tid; c < HROWS * 8; c += NT) {
      const int hr = c >> 3, pc = c & 7, lc = pc ^ fsw(hr);
      VT v = *(const VT*)(hb + hr * ROWB + pc * 16);
      const VT sv = *(const VT*)(stab + cb * BK + lc * VEC);
      modulate<T>(v, sv, lrelu_in);
      *(VT*)(hb + hr * ROWB + pc * 16) = v;
    }
  };

  // ---- prologue: halo of channel block 0, weights of steps 0 … STAGES−2, style row -----------
  // (the style row after the DMA issue: its load latency overlaps the DMA's instead of preceding
  // it; with the epilogue-operand prefetch below +0.1 … +1.3 % on the modulated forward,
  // bit-identical, r03 A/B)
  if (bwave) {
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) issue_b(s, s);  // nk ≥ 9
  } else {
#pragma unroll
    for (int j = 0; j < H_INS; ++j)
      if (j < my_pieces) issue_h(0, j, 0);
  }
  if constexpr (PRO) {
    const float mul = lrelu_in ? SQRT2 : 1.f;
    for (int i = tid; i < Cin; i += NT) {
      const float sv = p.in_scale ? p.in_scale[(size_t)n * Cin + i] : 1.f;
      stab[i] = from_f<T>(sv * mul);
    }
  }
  if (bwave) wait_vmcnt((STAGES - 2) * B_INS);  // step 0 landed, 1, 2 may stay in flight
  else wait_vmcnt(0);
  __syncthreads();
  if constexpr (PRO && MIA_HALO_PREMOD) {
    premod(0, 0);
    __syncthreads();
  }
  HT_STAMP(t_pro);
#ifdef MIA_HALO_TIMING
  unsigned long long c_vm = 0, c_mma = 0, c_bar = 0;
#endif

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fq = lane >> 4;
  if constexpr (EPI >= 0) {
    // The taps unrolled (the specialised-epilogue launches): every fragment address is a
    // lane-constant LDS offset — for the A fragments one per (row shift q = i + dy, column shift
    // dx), for the B fragments one per column fragment — computed once here instead of ≈ 6 VALU
    // per fragment per step; the second MFMA half reads chunk ^ 4 (byte offset ^ 64). Same reads
    // and MFMAs in the same order as the rolled loop below (bit-identical outputs).
    int oh[FM + 2][3], ob[FN];
#pragma unroll
    for (int q = 0; q < FM + 2; ++q)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int hr = (wm * FM + q) * HSIDE + frow + c;
        int v = hr * ROWB + ((fq ^ fsw(hr)) << 4);
        asm volatile("" : "+v"(v));  // kept in registers, not recomputed per step
        oh[q][c] = v;
      }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * FN * 16 + 16 * j + frow;
      int v = row * ROWB + ((fq ^ fsw(row)) << 4);
      asm volatile("" : "+v"(v));
      ob[j] = v;
    }
    // The StyledConv forward's epilogue operands (demod, bias: BN floats each; the patch's noise:
    // PH rows × 16 floats) are DMA'd by H-wave 0 into the halo buffer the last channel block leaves
    // free (past the LDS pre-reduction rows), at its first tap: they land under its MFMAs instead
    // of one dependent round trip in the epilogue.
    char* const aux = hbuf + (ncb & (TL::NHBUF - 1)) * HBUF + AUX_OFF;
    auto issue_aux = [&]() {
      const int l = lane & 31;
      const float* a0;
      if (lane < 32) {  // demod (out_scale) | noise rows
        a0 = (EPI & epi::OSC) && n0 + 4 * l < Cout
                 ? p.out_scale + (size_t)n * k.cout_mod + n0 + 4 * l
                 : (const float*)g_zero16;
      } else {          // bias
        a0 = n0 + 4 * l < Cout ? p.bias + n0 + 4 * l : (const float*)g_zero16;
      }
      __builtin_amdgcn_global_load_lds((gptr_t)a0, (lptr_t)aux, 16, 0, 0);
      const float* a1 = lane < 4 * PH ? p.noise + (size_t)(y0 + (l >> 2)) * W + x0 + 4 * (l & 3)
                                      : (const float*)g_zero16;
      __builtin_amdgcn_global_load_lds((gptr_t)a1, (lptr_t)(aux + 1024), 16, 0, 0);
    };
    int st = 0;
    for (int cb = 0; cb < ncb; ++cb) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int s = cb * 9 + t;
        if constexpr (AUXP) {
          if (t == 0 && cb + 1 == ncb && !bwave && hw == 0) issue_aux();
        }
        int hoff = (cb & (TL::NHBUF - 1)) * HBUF, soff = st * BSTAGE, x1 = 64;
        asm volatile("" : "+s"(hoff), "+s"(soff), "+s"(x1));
        const char* ha = hbuf + hoff;
        const char* sb = bring + soff;
        const int dy = t / 3, dx = t % 3;
        if (bwave && s + STAGES - 1 < nk) issue_b(s + STAGES - 1, st == 0 ? STAGES - 1 : st - 1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          VT af[FM], bf[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i)
            af[i] = *(const VT*)(ha + (h ? oh[i + dy][dx] ^ x1 : oh[i + dy][dx]));
#pragma unroll
          for (int j = 0; j < FN; ++j) bf[j] = *(const VT*)(sb + (h ? ob[j] ^ x1 : ob[j]));
          if constexpr (PRO && !MIA_HALO_PREMOD) {
            const VT sv = *(const VT*)(stab + cb * BK + (h * 4 + fq) * VEC);
#pragma unroll
            for (int i = 0; i < FM; ++i) modulate<T>(af[i], sv, lrelu_in);
          }
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = mfma_chunk<T>(bf[j], af[i], acc[i][j]);  // D[channel][pixel]
          __builtin_amdgcn_s_setprio(0);
          if (h == 0 && !bwave && TL::NHBUF > 1 && cb + 1 < ncb && t * HPS < H_INS) {
            // H-waves: the next block's halo between the two MFMA halves, HPS pieces per tap
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < HPS; ++q) {
              const int j = t * HPS + q;
              if (j < H_INS && j < my_pieces) issue_h(cb + 1, j, (cb + 1) & (TL::NHBUF - 1));
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if (bwave) wait_vmcnt(B_INS * max(0, min(STAGES - 2, nk - 2 - s)));
        else if (t == 8) wait_vmcnt(0);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage st are done
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PRO && MIA_HALO_PREMOD && TL::NHBUF > 1) {
          if (t == 8 && cb + 1 < ncb) {  // the next block's halo landed: modulate it once
            premod(cb + 1, (cb + 1) & 1);
            __syncthreads();
          }
        }
        st = st + 1 == STAGES ? 0 : st + 1;
      }
    }
  } else {
  int st = 0, cb = 0, t = 0;
  for (int s = 0; s < nk; ++s) {
    HT_STEP_STAMP(ts1);
    const char* ha = hbuf + (cb & (TL::NHBUF - 1)) * HBUF;
    const char* sb = bring + st * BSTAGE;
    const int dy = t >= 6 ? 2 : (t >= 3 ? 1 : 0), dx = t - 3 * dy;
    // B-waves issue the weights STAGES−1 steps ahead right away (their partner H-wave on the
    // same SIMD keeps the MFMA pipe busy if the address unit queue stalls them)
    if (bwave && s + STAGES - 1 < nk) {
      issue_b(s + STAGES - 1, st == 0 ? STAGES - 1 : st - 1);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = h * 4 + fq;
      VT af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int hr = (wm * FM + i + dy) * HSIDE + frow + dx;
        af[i] = *(const VT*)(ha + hr * ROWB + ((ch ^ fsw(hr)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * FN * 16 + 16 * j + frow;
        bf[j] = *(const VT*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
      }
      if constexpr (PRO && !MIA_HALO_PREMOD) {
        const VT sv = *(const VT*)(stab + cb * BK + ch * VEC);
#pragma unroll
        for (int i = 0; i < FM; ++i) modulate<T>(af[i], sv, lrelu_in);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = EPI != -2 ? mfma_chunk<T>(bf[j], af[i], acc[i][j])  // D[channel][pixel]
                          : mfma_chunk<T>(af[i], bf[j], acc[i][j]);  // D[pixel][channel]
      if (h == 0 && !bwave) {
        // H-waves issue between the two MFMA halves: the texture-address unit takes ≈16 cycles
        // per 1-KB LDS-DMA instruction; here the queue overlaps the partner B-wave's MFMAs.
        __builtin_amdgcn_sched_barrier(0);
        if (TL::NHBUF > 1 && cb + 1 < ncb) {  // next block's halo, HPS pieces per step from tap 0
          // branch per tap so that every piece index is a compile-time constant (src[] stays in
          // registers; a runtime index would move it to scratch)
#pragma unroll
          for (int tt = 0; tt < (H_INS + HPS - 1) / HPS; ++tt) {
            if (t == tt) {
#pragma unroll
              for (int q = 0; q < HPS; ++q) {
                const int j = tt * HPS + q;
                if (j < H_INS && j < my_pieces) issue_h(cb + 1, j, (cb + 1) & (TL::NHBUF - 1));
              }
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    HT_STEP_STAMP(ts2);
    // B-wave: step s+1's weights must have landed; the weights of steps s+2 … s+STAGES−1
    // (issued later; B-waves issue nothing else) may stay in flight. H-wave: the next block's
    // halo must have landed before its first tap (issued by tap 3, waited at tap 8).
    if (bwave) wait_vmcnt(B_INS * max(0, min(STAGES - 2, nk - 2 - s)));
    else if (t == 8) wait_vmcnt(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of stage st are done
    HT_STEP_STAMP(ts3);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#if HT_STEPS
    HT_STEP_STAMP(ts4);
    c_mma += ts2 - ts1;
    c_vm += ts3 - ts2;
    c_bar += ts4 - ts3;
#endif
    if constexpr (PRO && MIA_HALO_PREMOD && TL::NHBUF > 1) {
      if (t == 8 && cb + 1 < ncb) {  // the next block's halo landed: modulate it once
        premod(cb + 1, (cb + 1) & 1);
        __syncthreads();
      }
    }
    st = st + 1 == STAGES ? 0 : st + 1;
    if (++t == 9) { t = 0; ++cb; }
  }
  }  // rolled loop
  HT_STAMP(t_loop);
  if constexpr (AUXP) {
    // the prefetched operands (landed: H-wave 0 drained them before the last step's barrier)
    const char* aux = hbuf + (ncb & (TL::NHBUF - 1)) * HBUF + AUX_OFF;
    EpiChan<FN> E;
    EpiRows<T, FM, FN> R;
    const int cl = n0 + wn * FN * 16 + ((lane >> 4) << 2);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = cl + 16 * j - n0;
      E.osc[j] = *(const f32x4*)(aux + 4 * c);
      E.bia[j] = *(const f32x4*)(aux + 512 + 4 * c);
      E.dmv[j] = E.bbv[j] = E.msl[j] = E.asl[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      R.nz[i] = p.noise_w * *(const float*)(aux + 1024 + 4 * ((wm * FM + i) * 16 + (lane & 15)));
      R.bnz[i] = 0.f;
    }
    halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, n0, wm, wn, lane, -1, -1, &R, nullptr,
                                TL::WM, TL::BN, nullptr, &E);
  } else if constexpr (EPI >= 0) {
    // (the LDS is idle after the main loop's last barrier: the pre-reduction reuses it)
    halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, n0, wm, wn, lane, -1, -1, nullptr,
                                k.prered ? (float*)smem : nullptr, TL::WM, TL::BN);
  } else if constexpr (EPI == -1) {
    halo_epilogue<T, TL>(k, acc, n, y0, x0, n0, wm, wn, lane);
  } else {
    __syncthreads();
    const int img_row = n * H + y0;
    conv_epilogue<T, TL>(k, G, acc, smem, n0, true, n, [=](int r) {
      return (img_row + (r >> 4)) * W + x0 + (r & 15);
    }, (y0 / TL::PH) * (W / TL::PW) + x0 / TL::PW);  // the patch's reduction slot
  }
#ifdef MIA_HALO_TIMING
  HT_STAMP(t_end);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  HT_STAMP(t_drain);
  if (tid == 0) {
    unsigned long long* d = g_halo_dbg[blockIdx.x % HT_SLOTS];
    atomicAdd(&d[7], t_drain - t_end);
    atomicAdd(&d[0], t_pro - t_start);
    atomicAdd(&d[1], c_vm);
    atomicAdd(&d[2], c_mma);
    atomicAdd(&d[3], c_bar);
    atomicAdd(&d[4], t_end - t_loop);
    atomicAdd(&d[5], 1ull);
    atomicAdd(&d[6], t_loop - t_pro);
  }
#endif
}

template <typename T, typename TL, bool PRO, int EPI>
static int launch_halo_tile_(ConvK& k, hipStream_t st) {
  k.nbn = (k.a.Cout + TL::BN - 1) / TL::BN;
  const int patches = k.a.N * (k.a.H / TL::PH) * (k.a.W / TL::PW);
  k.nblk = patches * k.nbn;
  size_t lds = TL::NHBUF * (size_t)TL::HBUF + (size_t)TL::STAGES * TL::BSTAGE;
  if (PRO) lds += (size_t)k.a.Cin * sizeof(T);
  lds = std::max(lds, (size_t)TL::EROWS * TL::ES * 4);
  lds = std::max(lds, (size_t)TL::NW * TL::BN * 4);
  if (lds > 160 * 1024) return set_error("conv_halo: LDS budget exceeded");
  if (TL::NHBUF == 1 && k.a.Cin != ROWB / (int)sizeof(T))
    return set_error("conv_halo: single-buffer tile needs Cin = one channel block");
  auto fn = conv_halo_kernel<T, TL, PRO, EPI>;
  if (const int rc = ensure_dyn_lds((const void*)fn, 160 * 1024); rc != MIA_OK) return rc;
  k.prered = EPI >= 0 && (EPI & epi::CSUM);
  const int H = k.a.H, W = k.a.W;
  const int nslots = EPI >= 0    ? halo_red_slots(H, W, TL::FM, TL::WM, k.prered)
                     : EPI == -1 ? halo_red_slots(H, W, TL::FM, TL::WM, false)
                                 : (H / TL::PH) * (W / TL::PW);
  RedQ r;
  int rc = conv_red_begin(k, r, nslots, st);
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(k.nblk), dim3(TL::NT), lds, st, k);
  rc = check_launch("conv_halo");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

template <typename T, typename TL, bool PRO, bool SPEC>
static int launch_halo_tile(ConvK& k, hipStream_t st) {
  // T_HALO_EPI (tests / tuning): 0 LDS-staged shared epilogue, 2 register epilogue with runtime
  // features and the rolled tap loop; default 1 = specialised where one exists
  const int sel = tune(T_HALO_EPI);
  if (sel == 0) return launch_halo_tile_<T, TL, PRO, -2>(k, st);
  if constexpr (SPEC && sizeof(T) == 2) {  // fp32 (reference dtype) keeps the generic path
    if (sel == 1) {
      using namespace epi;
      const int f = epi_mask(k);
      if constexpr (PRO) {  // modulated input: the StyledConv forward
        if (f == (OSC | NOISE | BIAS | LRELU))
          return launch_halo_tile_<T, TL, PRO, OSC | NOISE | BIAS | LRELU>(k, st);
      } else switch (f) {  // the other launches of the attack step (vgg.py, stylegan2.py)
        case 0: return launch_halo_tile_<T, TL, PRO, 0>(k, st);
        // the StyledConv forward on per-image modulated + demodulated weights (mia_conv3x3_wmod)
        case NOISE | BIAS | LRELU: return launch_halo_tile_<T, TL, PRO, NOISE | BIAS | LRELU>(k, st);
        case BIAS | RELU: return launch_halo_tile_<T, TL, PRO, BIAS | RELU>(k, st);
        case MASK: return launch_halo_tile_<T, TL, PRO, MASK>(k, st);
        case TAP: return launch_halo_tile_<T, TL, PRO, TAP>(k, st);
        case OSC | SDOT: return launch_halo_tile_<T, TL, PRO, OSC | SDOT>(k, st);
        case OSC | SDOT | ACC: return launch_halo_tile_<T, TL, PRO, OSC | SDOT | ACC>(k, st);
        case OSC | SDOT | BAB: return launch_halo_tile_<T, TL, PRO, OSC | SDOT | BAB>(k, st);
        case OSC | SDOT | ACC | BAB:
          return launch_halo_tile_<T, TL, PRO, OSC | SDOT | ACC | BAB>(k, st);
        // e4e IR-SE50 body: conv1 fwd (PReLU), conv2 fwd (bias + SE pool), their input gradients
        case PRELU: return launch_halo_tile_<T, TL, PRO, PRELU>(k, st);
        case BIAS | CSUM: return launch_halo_tile_<T, TL, PRO, BIAS | CSUM>(k, st);
        case MASK | MSL: return launch_halo_tile_<T, TL, PRO, MASK | MSL>(k, st);
        case ACC: return launch_halo_tile_<T, TL, PRO, ACC>(k, st);
        default: break;
      }
    }
  }
  return launch_halo_tile_<T, TL, PRO, -1>(k, st);
}

// Eligible: one group, stride 1, 3×3 taps with pad 1, identity output placement, no pixel
// shuffle, 16-divisible spatial dims, whole channel blocks, and Cout > 64 or Cout ≤ 32 (at Cout = 64
// the generic 128×64 tile measured faster: the halo tile's fixed costs are paid for half the
// MFMAs; at Cout ≤ 32 — the VGG input gradient, 8 channels — the generic tile computes 64 columns
// and gathers every input row 9 times, the 32-column halo tile is memory-bound on one halo pass).
bool conv_halo_eligible(const ConvK& k, int dtype) {
  if (tune(T_CONV_HALO) == 0) return false;
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  const int bk = dtype == MIA_F32 ? 32 : 64;
  // Cout = 64 on the 64-channel halo tile (T_HALO_C64: 1 = the 2-byte types, default; 0 = never):
  // with its specialised epilogues and unrolled taps it beats the generic 64-column tile on every
  // attack shape (512² StyledConv forward bf16 2.69 → 1.39 ms, fp16 1.85 → 1.34, input gradient
  // + sdot 1.53 → 1.42, 128² 128 → 64 gradient 0.58 → 0.46; profiles/r03_halo_c64_ab.txt)
  const bool c64 = tune(T_HALO_C64) != 0 && dtype != MIA_F32;
  return k.ng == 1 && k.stride == 1 && G.kh == 3 && G.kw == 3 && G.pad_y == 1 && G.pad_x == 1 &&
         G.ho == a.H && G.wo == a.W && G.ay == 1 && G.ax == 1 && G.by == 0 && G.bx == 0 &&
         !a.shuffle_out && a.H % 16 == 0 && a.W % 16 == 0 && a.Cin % bk == 0 &&
         (a.Cout > 64 || a.Cout <= 32 || (a.Cout == 64 && c64)) &&
         k.HT == a.H && k.WT == a.W;
}

int launch_conv_halo(ConvK& k, int dtype, hipStream_t st) {
  const bool pro = k.a.in_scale != nullptr || k.a.act_in != MIA_ACT_NONE;
  // 8×16 patches (4 waves, 2 blocks per CU, 2-stage weight ring): measured 5–10 % faster than
  // 16×16 patches on 8 waves (1 block per CU, 4 stages) and 25–40 % faster than 16×16 patches on
  // 4 waves (FM = 8, one wave per SIMD) on every attack shape — two waves per SIMD keep the
  // matrix pipe fed through each other's LDS reads, DMA issue and barriers.
  // (round 3, fp16 / bf16 modulated forward at 256² / 128² / 64², bit-identical outputs:
  // 16×16 patches on 8 waves with a 3-stage ring −1.9 … +2.1 %, on 4 waves −9 … −18 %)
  typedef HaloTile<128, 8, 2> Small;
  typedef HaloTile<64, 8, 3> Small64;
  // Cout ≤ 32 (VGG input gradient): little MFMA work per K-step, so the weights of all nine taps
  // of a one-block Cin are DMA'd in the prologue (9 stages, 36 KB) and no step waits on L2.
  typedef HaloTile<32, 8, 2> Small32;
  typedef HaloTile<32, 8, 9, 1> Small32x9;
  MIA_DISPATCH_DTYPE(dtype, T, {
    if (k.a.Cout <= 32) {
      if (k.a.Cin == ROWB / (int)sizeof(T))
        return pro ? launch_halo_tile<T, Small32x9, true, false>(k, st)
                   : launch_halo_tile<T, Small32x9, false, true>(k, st);
      return pro ? launch_halo_tile<T, Small32, true, false>(k, st)
                 : launch_halo_tile<T, Small32, false, false>(k, st);
    }
    if (k.a.Cout <= 64)  // (specialised epilogues + unrolled taps, as the 128-channel tile)
      return pro ? launch_halo_tile<T, Small64, true, true>(k, st)
                 : launch_halo_tile<T, Small64, false, true>(k, st);
    return pro ? launch_halo_tile<T, Small, true, true>(k, st)
               : launch_halo_tile<T, Small, false, true>(k, st);
  });
  return MIA_OK;
}

// Per-image modulated + demodulated weights of a StyledConv (rosinality ModulatedConv2d's
// weight path, the form the reference's generator computes: w' = w·s[n][ci]·demod[n][co]), for
// the 2-byte halo kernel at high resolution: the activations enter the MFMAs unmodulated, so the
// kernel has no per-channel-block modulation pass over the halo in LDS and no demod in the
// epilogue. A block writes MW_ROWS rows [n][co0 .. co0+MW_ROWS) of the [N][Cout][Kpad] output, one
// 16-B vector per thread and pass, with the image's styles staged in LDS (the K index is tap-major,
// so a vector's 8 styles are 8 consecutive floats); no 64-bit index arithmetic.
constexpr int MW_ROWS = 16;
template <typename T>
__global__ __launch_bounds__(256) void modulate_weights_kernel(const T* __restrict__ w,
                                                               const float* __restrict__ s,
                                                               const float* __restrict__ d,
                                                               T* __restrict__ out, int Cout,
                                                               int Cin, int K, int Kpad) {
  typedef typename Vec<T>::type VT;
  constexpr int VEC = Vec<T>::N;
  __shared__ float sl[2048];
  const int n = blockIdx.y, co0 = blockIdx.x * MW_ROWS;
  for (int c = threadIdx.x; c < Cin; c += 256) sl[c] = s[(size_t)n * Cin + c];
  __syncthreads();
  const int vpr = Kpad / VEC, nv = MW_ROWS * vpr;
  for (int i = threadIdx.x; i < nv; i += 256) {
    const int r = i / vpr, kv = (i - r * vpr) * VEC, co = co0 + r;
    if (co >= Cout) break;
    const VT wv = *(const VT*)(w + (size_t)co * Kpad + kv);
    const float dm = d ? d[(size_t)n * Cout + co] : 1.f;
    const int c0 = kv & (Cin - 1);  // Cin ≥ 8 and a power of two: the vector stays in one tap
    VT o;
#pragma unroll
    for (int e = 0; e < VEC; ++e)
      o[e] = kv + e < K ? from_f<T>(to_f(wv[e]) * sl[c0 + e] * dm) : from_f<T>(0.f);
    *(VT*)(out + ((size_t)n * Cout + co) * Kpad + kv) = o;
  }
}

}  // namespace mia

using namespace mia;

extern "C" int mia_modulate_weights(const void* w, const float* in_scale, const float* out_scale,
                                    void* w_mod, int N, int Cout, int Cin, int Kpad, int dtype,
                                    void* stream) {
  MIA_CHECK_ARG(w && in_scale && w_mod && N > 0 && Cout > 0, "bad args");
  MIA_CHECK_ARG(dtype == MIA_F16 || dtype == MIA_BF16, "2-byte dtypes only");
  MIA_CHECK_ARG(Cin >= 8 && Cin <= 2048 && (Cin & (Cin - 1)) == 0,
                "Cin must be a power of two in [8, 2048]");
  MIA_CHECK_ARG(Kpad == mia_conv_kpad(Cin, dtype), "Kpad must be mia_conv_kpad()");
  MIA_CHECK_ARG(N <= 65535, "N > 65535");
  const dim3 grid((Cout + MW_ROWS - 1) / MW_ROWS, N);
  hipStream_t st = (hipStream_t)stream;
  MIA_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(modulate_weights_kernel<T>, grid, dim3(256), 0, st, (const T*)w,
                       in_scale, out_scale, (T*)w_mod, Cout, Cin, 9 * Cin, Kpad);
  });
  return check_launch("modulate_weights");
}

// mia_conv3x3 on per-image weights: args->w = [N][Cout][Kpad] (mia_modulate_weights), the images'
// matrices w_nstride elements apart; no in_scale (the modulation is in the weights).
extern "C" int mia_conv3x3_wmod(const mia_conv_args* args, int64_t w_nstride, int dtype,
                                void* stream) {
  MIA_CHECK_ARG(args != nullptr, "null args");
  const mia_conv_args& a = *args;
  MIA_CHECK_ARG(dtype == MIA_F16 || dtype == MIA_BF16, "2-byte dtypes only");
  MIA_CHECK_ARG(w_nstride >= (int64_t)a.Cout * a.Kpad, "w_nstride < Cout·Kpad");
  MIA_CHECK_ARG(a.in_scale == nullptr && a.act_in == MIA_ACT_NONE && !a.shuffle_out,
                "per-image weights: no in_scale / act_in / shuffle_out");
  MIA_CHECK_ARG(a.Cout > 64 && a.Cin <= 2048, "per-image weights: the 128-channel halo tile");
  ConvK k = {};
  k.a = a;
  k.stride = 1;
  k.ng = 1;
  ConvGroup& G = k.g[0];
  G.w = a.w;
  G.kpad = a.Kpad;
  G.kh = G.kw = 3;
  G.pad_y = G.pad_x = 1;
  G.ho = a.H;
  G.wo = a.W;
  G.ay = G.ax = 1;
  G.m = pixels_clamped(a.N, a.H, a.W);
  k.HT = a.H;
  k.WT = a.W;
  k.cout_mod = a.Cout;
  k.ystride = a.y_cstride > 0 ? a.y_cstride : a.Cout;
  k.wn = w_nstride;
  MIA_CHECK_ARG(k.ystride >= k.cout_mod, "y_cstride < Cout");
  MIA_CHECK_ARG(a.x && a.w && a.y && a.N > 0 && a.Cin % 64 == 0 && a.Cout % 8 == 0,
                "bad conv args");
  MIA_CHECK_ARG(a.Kpad == mia_conv_kpad(a.Cin, dtype), "Kpad must be mia_conv_kpad()");
  MIA_CHECK_ARG((int64_t)a.N * a.H * a.W * a.Cin < (1LL << 31), "input too large");
  if (conv_wres128_eligible(k, dtype)) return launch_conv_wres128(k, dtype, (hipStream_t)stream);
  MIA_CHECK_ARG(conv_halo_eligible(k, dtype), "per-image weights need the halo kernel's shapes "
                                              "(H, W multiples of 16)");
  return launch_conv_halo(k, dtype, (hipStream_t)stream);
}

#ifdef MIA_HALO_TIMING
extern "C" int mia_debug_halo_timing(unsigned long long* out, int reset) {
  static unsigned long long h[mia::HT_SLOTS][8];
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(mia::g_halo_dbg), sizeof(h));
  for (int c = 0; c < 8; ++c) {
    out[c] = 0;
    for (int r = 0; r < mia::HT_SLOTS; ++r) out[c] += h[r][c];
  }
  if (reset) {
    memset(h, 0, sizeof(h));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(mia::g_halo_dbg), h, sizeof(h));
  }
  return 0;
}
#endif
