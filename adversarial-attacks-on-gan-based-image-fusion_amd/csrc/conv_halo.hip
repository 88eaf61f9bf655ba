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
#if defined(MIA_HALO_EXP) && MIA_HALO_EXP >= 2
  static constexpr int STAGES = MIA_HALO_EXP;
  static constexpr int NHBUF = 1;  // tuning experiment: one halo buffer (wrong results)
#else
  static constexpr int STAGES = STAGES_;
  static constexpr int NHBUF = NHBUF_;
#endif
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

__device__ __forceinline__ void ld4f(const float* p, float (&v)[4]) {
  const f32x4 a = *(const f32x4*)p;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = a[e];
}

// Epilogue straight from the accumulators (REG kernels). Their MFMAs compute D = W·X̃ᵀ (output
// channels × patch pixels), so for every fragment a lane holds 4 consecutive output channels of
// one pixel: each per-element operation of conv_epilogue (same order, same semantics) runs in
// registers with 8-/16-byte aux loads and stores and no LDS staging. The sdot / q reductions sum
// a lane's pixels, then the 16 pixel lanes of a channel group by shuffles, then one atomic per
// channel per wave.
template <typename T, typename TL>
__device__ __forceinline__ void halo_epilogue(const ConvK& k, const f32x4 (&acc)[TL::FM][TL::FN],
                                              int n, int y0, int x0, int n0, int wm, int wn,
                                              int lane) {
  constexpr int FM = TL::FM, FN = TL::FN;
  const mia_conv_args& p = k.a;
  const int H = p.H, W = p.W, Cout = p.Cout;
  const int px = lane & 15;
  const int cl = n0 + wn * FN * 16 + ((lane >> 4) << 2);  // first channel of fragment 0
  const T* AX = (const T*)p.aux_x;
  const T* TA = (const T*)p.tap_a;
  const T* TT = (const T*)p.tap_t;
  const T* MA = (const T*)p.mask_a;
  T* __restrict__ Y = (T*)p.y;
  const bool bab = p.bab_demod != nullptr;
  float osc[FN][4], bia[FN][4], dmv[FN][4], bbv[FN][4], part[FN][4], partq[FN][4];
  float msl[FN][4], asl[FN][4], pcs[FN][4];
  const bool prelu = p.act_out == MIA_ACT_PRELU;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = cl + 16 * j;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      osc[j][e] = 1.f;
      bia[j][e] = dmv[j][e] = bbv[j][e] = part[j][e] = partq[j][e] = 0.f;
      msl[j][e] = asl[j][e] = pcs[j][e] = 0.f;
    }
    if (c < Cout) {  // c ≡ 0 mod 4 and Cout ≡ 0 mod 8: the whole quad is in range
      if (p.out_scale) ld4f(p.out_scale + (size_t)n * k.cout_mod + c, osc[j]);
      if (p.bias) ld4f(p.bias + c, bia[j]);
      if (p.mask_slope) ld4f(p.mask_slope + c, msl[j]);
      if (prelu) ld4f(p.act_slope + c, asl[j]);
      if (bab) {
        ld4f(p.bab_demod + (size_t)n * Cout + c, dmv[j]);
        if (p.bab_bias) ld4f(p.bab_bias + c, bbv[j]);
      }
    }
  }
  // 2-byte outputs: pairs of fragments are exchanged between lane rows (v_permlane16_swap) so
  // that every lane stores 8 consecutive channels with ONE 16-byte store — the store tail is
  // issue-bound per instruction (cdna_hip_programming.md T21), so half the instructions.
  constexpr bool WIDE = sizeof(T) == 2 && FN % 2 == 0;
  const int lrow = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int y = y0 + wm * FM + i, x = x0 + px;
    const int m = (n * H + y) * W + x;  // output pixel (identity placement, HT = H, WT = W)
    const float nz = p.noise ? p.noise_w * p.noise[y * W + x] : 0.f;
    const float bnz = (bab && p.bab_noise) ? p.bab_noise_w * p.bab_noise[y * W + x] : 0.f;
    float vo[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = cl + 16 * j;
#pragma unroll
      for (int e = 0; e < 4; ++e) vo[j][e] = 0.f;
      if (c >= Cout) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      const size_t aoff = (size_t)m * Cout + c;
      float xv[4];
      if (p.sdot || bab) load4<T>(AX + aoff, xv);
      if (p.sdot) {
#pragma unroll
        for (int e = 0; e < 4; ++e) part[j][e] += v[e] * apply_act(xv[e], p.act_aux);
      }
      if (Y) {
        const size_t off = (size_t)m * k.ystride + c;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] * osc[j][e] + nz + bia[j][e];
        float ma[4];
        if (TA) {
          float tt[4];
          load4<T>(TA + aoff, ma);  // the tap tensor doubles as the mask when they coincide
          load4<T>(TT + aoff, tt);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += p.tap_coef * (ma[e] - tt[e]);
        }
        if (MA) {
          if (MA != TA) load4<T>(MA + aoff, ma);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = ma[e] > 0.f ? v[e] : msl[j][e] * v[e];
        }
        if (prelu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : asl[j][e] * v[e];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act_out);
        }
        if (p.accumulate) {
          float yo[4];
          load4<T>(Y + off, yo);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += yo[e];
        }
        if (bab) {  // fused StyledConv backward front of the layer whose activation is aux_x
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gr = lrelu_s2_grad(xv[e]);
            const float gp = v[e] * gr;
            partq[j][e] += gp * (xv[e] / gr - bnz - bbv[j][e]);
            v[e] = gp * dmv[j][e];
          }
        }
        if (p.csum) {
#pragma unroll
          for (int e = 0; e < 4; ++e) pcs[j][e] += v[e];
        }
        if constexpr (WIDE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) vo[j][e] = v[e];
        } else {
          store4<T>(Y + off, v);
        }
      }
    }
    if constexpr (WIDE) {
      if (Y) {
        typedef T t2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int q = 0; q < FN / 2; ++q) {
          // A = fragment 2q (this lane's 4 channels), B = fragment 2q+1; after the swap lane
          // row r holds channels [8·(r>>1), +8) of fragment 2q + (r & 1)
          unsigned a[2], b[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const t2 ta = {(T)vo[2 * q][2 * h], (T)vo[2 * q][2 * h + 1]};
            const t2 tb = {(T)vo[2 * q + 1][2 * h], (T)vo[2 * q + 1][2 * h + 1]};
            a[h] = __builtin_bit_cast(unsigned, ta);
            b[h] = __builtin_bit_cast(unsigned, tb);
            const auto r = __builtin_amdgcn_permlane16_swap(a[h], b[h], false, false);
            a[h] = r[0];
            b[h] = r[1];
          }
          const int c = n0 + wn * FN * 16 + 16 * (2 * q + (lrow & 1)) + 8 * (lrow >> 1);
          if (c < Cout)
            *(uint4*)(Y + (size_t)m * k.ystride + c) = make_uint4(a[0], a[1], b[0], b[1]);
        }
      }
    }
  }
  if (p.sdot || bab || p.csum) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = cl + 16 * j;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = part[j][e], b = partq[j][e], cs = pcs[j][e];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a += __shfl_xor(a, o, 64);
          b += __shfl_xor(b, o, 64);
          cs += __shfl_xor(cs, o, 64);
        }
        if (px == 0 && c < Cout) {
          if (p.sdot) atomicAdd(&p.sdot[(size_t)n * Cout + c + e], a);
          if (bab) atomicAdd(&p.bab_q[(size_t)n * Cout + c + e], b);
          if (p.csum) atomicAdd(&p.csum[(size_t)n * Cout + c + e], cs);
        }
      }
    }
  }
}

// Epilogue feature mask (compile-time specialisations of halo_epilogue for the launches the
// attack makes; any other combination runs the runtime-generic halo_epilogue).
namespace epi {
constexpr int OSC = 1, NOISE = 2, BIAS = 4, TAP = 8, MASK = 16, ACC = 32, SDOT = 64, BAB = 128;
constexpr int RELU = MIA_ACT_RELU << 8, LRELU = MIA_ACT_LRELU_S2 << 8;
}  // namespace epi

template <typename T>
struct Raw4 {  // 4 consecutive elements of T, loaded raw (8 or 16 bytes)
  typedef T type __attribute__((ext_vector_type(4)));
};

// The same operations as halo_epilogue for one feature mask F, straight-line: every aux load of
// the tile is issued first (one wait instead of one per fragment — a wait also drains the stores
// issued before it), then the arithmetic and the 16-byte stores.
template <typename T, typename TL, int F>
__device__ __forceinline__ void halo_epilogue_f(const ConvK& k, const f32x4 (&acc)[TL::FM][TL::FN],
                                                int n, int y0, int x0, int n0, int wm, int wn,
                                                int lane) {
  constexpr int FM = TL::FM, FN = TL::FN;
  constexpr bool OSC = F & epi::OSC, NOISE = F & epi::NOISE, BIAS = F & epi::BIAS;
  constexpr bool TAP = F & epi::TAP, MASK = F & epi::MASK, ACC = F & epi::ACC;
  constexpr bool SDOT = F & epi::SDOT, BAB = F & epi::BAB;
  constexpr int ACT = (F >> 8) & 3;
  constexpr bool WIDE = sizeof(T) == 2 && FN % 2 == 0;
  typedef typename Raw4<T>::type R4;
  const mia_conv_args& p = k.a;
  const int H = p.H, W = p.W, Cout = p.Cout;
  const int px = lane & 15, lrow = lane >> 4;
  const int cl = n0 + wn * FN * 16 + (lrow << 2);
  T* __restrict__ Y = (T*)p.y;
  const T* AX = (const T*)p.aux_x;
  const T* TA = (const T*)p.tap_a;
  const T* TT = (const T*)p.tap_t;
  const T* MA = (const T*)p.mask_a;
  const bool ma_is_ta = MA == TA;

  float osc[FN][4], bia[FN][4], dmv[FN][4], bbv[FN][4];
  bool cok[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = cl + 16 * j;
    cok[j] = c < Cout;  // c ≡ 0 mod 4, Cout ≡ 0 mod 8: the whole quad is in range
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      osc[j][e] = 1.f;
      bia[j][e] = dmv[j][e] = bbv[j][e] = 0.f;
    }
    if (cok[j]) {
      if constexpr (OSC) ld4f(p.out_scale + (size_t)n * k.cout_mod + c, osc[j]);
      if constexpr (BIAS) ld4f(p.bias + c, bia[j]);
      if constexpr (BAB) {
        ld4f(p.bab_demod + (size_t)n * Cout + c, dmv[j]);
        if (p.bab_bias) ld4f(p.bab_bias + c, bbv[j]);
      }
    }
  }
  float part[FN][4], partq[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) part[j][e] = partq[j][e] = 0.f;
  // rows in chunks of FMC (the aux loads of a chunk are hoisted together; chunks bound the live
  // registers for tall wave tiles)
  constexpr int FMC = FM < 4 ? FM : 4;
#pragma unroll
  for (int i0 = 0; i0 < FM; i0 += FMC) {
  float nz[FMC], bnz[FMC];
  R4 rx[FMC][FN], rta[FMC][FN], rtt[FMC][FN], rma[FMC][FN], ryo[FMC][FN];
#pragma unroll
  for (int i = 0; i < FMC; ++i) {
    const int y = y0 + wm * FM + i0 + i, x = x0 + px;
    const int m = (n * H + y) * W + x;
    nz[i] = bnz[i] = 0.f;
    if constexpr (NOISE) nz[i] = p.noise_w * p.noise[y * W + x];
    if constexpr (BAB) {
      if (p.bab_noise) bnz[i] = p.bab_noise_w * p.bab_noise[y * W + x];
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if (!cok[j]) continue;
      const int c = cl + 16 * j;
      const size_t aoff = (size_t)m * Cout + c;
      if constexpr (SDOT || BAB) rx[i][j] = *(const R4*)(AX + aoff);
      if constexpr (TAP) {
        rta[i][j] = *(const R4*)(TA + aoff);
        rtt[i][j] = *(const R4*)(TT + aoff);
      }
      if constexpr (MASK) {
        if (!(TAP && ma_is_ta)) rma[i][j] = *(const R4*)(MA + aoff);
      }
      if constexpr (ACC) ryo[i][j] = *(const R4*)(Y + (size_t)m * k.ystride + c);
    }
  }

#pragma unroll
  for (int i = 0; i < FMC; ++i) {
    const int m = (n * H + y0 + wm * FM + i0 + i) * W + x0 + px;
    float vo[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) vo[j][e] = 0.f;
      if (!cok[j]) continue;
      float v[4] = {acc[i0 + i][j][0], acc[i0 + i][j][1], acc[i0 + i][j][2], acc[i0 + i][j][3]};
      float xv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) xv[e] = (SDOT || BAB) ? (float)rx[i][j][e] : 0.f;
      if constexpr (SDOT) {  // act_aux NONE (the host picks the generic epilogue otherwise)
#pragma unroll
        for (int e = 0; e < 4; ++e) part[j][e] += v[e] * xv[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (OSC) v[e] *= osc[j][e];
        if constexpr (NOISE) v[e] += nz[i];
        if constexpr (BIAS) v[e] += bia[j][e];
        if constexpr (TAP) v[e] += p.tap_coef * ((float)rta[i][j][e] - (float)rtt[i][j][e]);
        if constexpr (MASK) {
          const float ma = (TAP && ma_is_ta) ? (float)rta[i][j][e] : (float)rma[i][j][e];
          v[e] = ma > 0.f ? v[e] : 0.f;
        }
        if constexpr (ACT == MIA_ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
        if constexpr (ACT == MIA_ACT_LRELU_S2) v[e] = lrelu_s2(v[e]);
        if constexpr (ACC) v[e] += (float)ryo[i][j][e];
        if constexpr (BAB) {
          const float gr = lrelu_s2_grad(xv[e]);
          const float gp = v[e] * gr;
          partq[j][e] += gp * (xv[e] / gr - bnz[i] - bbv[j][e]);
          v[e] = gp * dmv[j][e];
        }
        vo[j][e] = v[e];
      }
      if constexpr (!WIDE) {
        if (Y) store4<T>(Y + (size_t)m * k.ystride + cl + 16 * j, v);
      }
    }
    if constexpr (WIDE) {
      if (Y) {
        typedef T t2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int q = 0; q < FN / 2; ++q) {
          unsigned a[2], b[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const t2 ta = {(T)vo[2 * q][2 * h], (T)vo[2 * q][2 * h + 1]};
            const t2 tb = {(T)vo[2 * q + 1][2 * h], (T)vo[2 * q + 1][2 * h + 1]};
            const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, ta),
                                                            __builtin_bit_cast(unsigned, tb),
                                                            false, false);
            a[h] = r[0];
            b[h] = r[1];
          }
          const int c = n0 + wn * FN * 16 + 16 * (2 * q + (lrow & 1)) + 8 * (lrow >> 1);
          if (c < Cout)
            *(uint4*)(Y + (size_t)m * k.ystride + c) = make_uint4(a[0], a[1], b[0], b[1]);
        }
      }
    }
  }
  }  // row chunks
  if constexpr (SDOT || BAB) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = cl + 16 * j;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = part[j][e], b = partq[j][e];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          if constexpr (SDOT) a += __shfl_xor(a, o, 64);
          if constexpr (BAB) b += __shfl_xor(b, o, 64);
        }
        if (px == 0 && c < Cout) {
          if constexpr (SDOT) atomicAdd(&p.sdot[(size_t)n * Cout + c + e], a);
          if constexpr (BAB) atomicAdd(&p.bab_q[(size_t)n * Cout + c + e], b);
        }
      }
    }
  }
}

// EPI: −2 = LDS-staged shared epilogue (conv_epilogue), −1 = register epilogue with runtime
// features (halo_epilogue), ≥ 0 = register epilogue specialised for feature mask EPI.
template <typename T, typename TL, bool PRO, int EPI>
__global__ __launch_bounds__(TL::NT, TL::WAVES_PER_SIMD) void conv_halo_kernel(const ConvK k) {
  // Blocks of equal work launched together stay in lockstep: every block loads its halo at the
  // same time and stores its tile at the same time, and HBM idles during the MFMA phase. Half of
  // the first dispatch wave starts late, so the memory phases of the two halves interleave with
  // each other's main loops for the rest of the launch (later blocks inherit their slot's phase).
  if (k.stagger_cycles && (int)blockIdx.x < k.stagger_blocks && ((blockIdx.x >> 3) & 1)) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < k.stagger_cycles) __builtin_amdgcn_s_sleep(16);
  }
  HT_STAMP(t_start);
  typedef typename Vec<T>::type VT;
  constexpr int VEC = Vec<T>::N;
  constexpr int BK = ROWB / (int)sizeof(T);
  constexpr int WN = TL::WN, FM = TL::FM, FN = TL::FN, NT = TL::NT, BN = TL::BN;
  constexpr int H_INS = TL::H_INS, B_INS = TL::B_INS, HBUF = TL::HBUF, BSTAGE = TL::BSTAGE;
  constexpr int STAGES = TL::STAGES, PH = TL::PH, PW = TL::PW, HSIDE = TL::HW, HROWS = TL::HROWS;
  constexpr int HPIECES = TL::HPIECES, BWAVES = TL::BWAVES, HWAVES = TL::HWAVES;
  constexpr int HPS = TL::H_PER_STEP;

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
  const T* __restrict__ Wt = (const T*)G.w;
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
#if defined(MIA_HALO_EXP) && MIA_HALO_EXP == 1
    return;  // tuning experiment: no halo traffic
#endif
    const T* a = src[j] ? src[j] + cb * BK : zero;
    __builtin_amdgcn_global_load_lds((gptr_t)a,
                                     (lptr_t)(hbuf + buf * HBUF + (hw + HWAVES * j) * 1024), 16,
                                     0, 0);
  };

  // ---- prologue: style row, halo of channel block 0, weights of steps 0 … STAGES−2 -----------
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;
  if constexpr (PRO) {
    const float mul = lrelu_in ? SQRT2 : 1.f;
    for (int i = tid; i < Cin; i += NT) {
      const float sv = p.in_scale ? p.in_scale[(size_t)n * Cin + i] : 1.f;
      stab[i] = from_f<T>(sv * mul);
    }
  }
  if (bwave) {
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) issue_b(s, s);  // nk ≥ 9
    wait_vmcnt((STAGES - 2) * B_INS);  // step 0 landed, steps 1, 2 may stay in flight
  } else {
#pragma unroll
    for (int j = 0; j < H_INS; ++j)
      if (j < my_pieces) issue_h(0, j, 0);
    wait_vmcnt(0);
  }
  __syncthreads();
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
      if constexpr (PRO) {
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
    st = st + 1 == STAGES ? 0 : st + 1;
    if (++t == 9) { t = 0; ++cb; }
  }
  HT_STAMP(t_loop);
  if constexpr (EPI >= 0) {
    halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, n0, wm, wn, lane);
  } else if constexpr (EPI == -1) {
#if defined(MIA_HALO_STOREONLY)  // tuning experiment: raw accumulator stores only (wrong results)
    if constexpr (sizeof(T) == 2 && FN % 2 == 0) {
      T* Yp = (T*)p.y;
      const int lrow = lane >> 4;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = (n * H + y0 + wm * FM + i) * W + x0 + (lane & 15);
#pragma unroll
        for (int q = 0; q < FN / 2; ++q) {
          typedef T t2 __attribute__((ext_vector_type(2)));
          unsigned a2[2], b2[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const t2 ta = {(T)acc[i][2 * q][2 * h], (T)acc[i][2 * q][2 * h + 1]};
            const t2 tb = {(T)acc[i][2 * q + 1][2 * h], (T)acc[i][2 * q + 1][2 * h + 1]};
            a2[h] = __builtin_bit_cast(unsigned, ta);
            b2[h] = __builtin_bit_cast(unsigned, tb);
            const auto r = __builtin_amdgcn_permlane16_swap(a2[h], b2[h], false, false);
            a2[h] = r[0];
            b2[h] = r[1];
          }
          const int c = n0 + wn * FN * 16 + 16 * (2 * q + (lrow & 1)) + 8 * (lrow >> 1);
          *(uint4*)(Yp + (size_t)m * p.Cout + c) = make_uint4(a2[0], a2[1], b2[0], b2[1]);
        }
      }
    }
#elif defined(MIA_HALO_NOEPI)  // tuning experiment: no epilogue (wrong results)
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) z += acc[i][j][0] + acc[i][j][3];
    if (z == 1234.5f) ((float*)p.y)[tid] = z;
#else
    halo_epilogue<T, TL>(k, acc, n, y0, x0, n0, wm, wn, lane);
#endif
  } else {
    __syncthreads();
    const int img_row = n * H + y0;
    conv_epilogue<T, TL>(k, G, acc, smem, n0, true, n, [=](int r) {
      return (img_row + (r >> 4)) * W + x0 + (r & 15);
    });
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
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    attr_set = true;
  }
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  const int per_cu = TL::WAVES_PER_SIMD == 2 ? 2 : 1;
  k.stagger_blocks = per_cu * ncu;
  const char* es = getenv("MIA_HALO_STAGGER");  // clocks; tuning / A-B switch
  k.stagger_cycles = es ? (unsigned)atoi(es) : 0u;
  if (k.nblk < 4 * k.stagger_blocks) k.stagger_cycles = 0;  // short launches: not worth a tail
  hipLaunchKernelGGL(fn, dim3(k.nblk), dim3(TL::NT), lds, st, k);
  return check_launch("conv_halo");
}

// Feature mask of a launch (−1: a combination without a specialisation, e.g. act_aux ≠ NONE).
static int epi_mask(const ConvK& k) {
  const mia_conv_args& a = k.a;
  if ((a.sdot || a.bab_demod) && a.act_aux != MIA_ACT_NONE) return -1;
  if (a.mask_slope || a.act_out == MIA_ACT_PRELU || a.csum) return -1;  // encoder features
  int f = 0;
  if (a.out_scale) f |= epi::OSC;
  if (a.noise) f |= epi::NOISE;
  if (a.bias) f |= epi::BIAS;
  if (a.tap_a) f |= epi::TAP;
  if (a.mask_a) f |= epi::MASK;
  if (a.accumulate) f |= epi::ACC;
  if (a.sdot) f |= epi::SDOT;
  if (a.bab_demod) f |= epi::BAB;
  return f | (a.act_out << 8);
}

template <typename T, typename TL, bool PRO, bool SPEC>
static int launch_halo_tile(ConvK& k, hipStream_t st) {
  // tuning / A-B switch, read per launch: MIA_HALO_EPI=0 LDS-staged shared epilogue, 2 register
  // epilogue with runtime features (no specialisation); default 1 = specialised where one exists
  const char* e = getenv("MIA_HALO_EPI");
  const int sel = e ? atoi(e) : 1;
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
        case BIAS | RELU: return launch_halo_tile_<T, TL, PRO, BIAS | RELU>(k, st);
        case MASK: return launch_halo_tile_<T, TL, PRO, MASK>(k, st);
        case TAP: return launch_halo_tile_<T, TL, PRO, TAP>(k, st);
        case OSC | SDOT: return launch_halo_tile_<T, TL, PRO, OSC | SDOT>(k, st);
        case OSC | SDOT | ACC: return launch_halo_tile_<T, TL, PRO, OSC | SDOT | ACC>(k, st);
        case OSC | SDOT | BAB: return launch_halo_tile_<T, TL, PRO, OSC | SDOT | BAB>(k, st);
        case OSC | SDOT | ACC | BAB:
          return launch_halo_tile_<T, TL, PRO, OSC | SDOT | ACC | BAB>(k, st);
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
  const char* e = getenv("MIA_CONV_HALO");  // tuning / A-B switch: 0 disables the halo path
  if (e && atoi(e) == 0) return false;
  const char* e64 = getenv("MIA_HALO_N64");  // tuning: 1 = halo path for Cout = 64 too
  const bool n64 = e64 && atoi(e64) == 1;
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  const int bk = dtype == MIA_F32 ? 32 : 64;
  return k.ng == 1 && k.stride == 1 && G.kh == 3 && G.kw == 3 && G.pad_y == 1 && G.pad_x == 1 &&
         G.ho == a.H && G.wo == a.W && G.ay == 1 && G.ax == 1 && G.by == 0 && G.bx == 0 &&
         !a.shuffle_out && a.H % 16 == 0 && a.W % 16 == 0 && a.Cin % bk == 0 &&
         (a.Cout > 64 || a.Cout <= 32 || (n64 && a.Cout == 64)) &&
         k.HT == a.H && k.WT == a.W;
}

int launch_conv_halo(ConvK& k, int dtype, hipStream_t st) {
  const bool pro = k.a.in_scale != nullptr || k.a.act_in != MIA_ACT_NONE;
  // 8×16 patches (4 waves, 2 blocks per CU, 2-stage weight ring): measured 5–10 % faster than
  // 16×16 patches on 8 waves (1 block per CU, 4 stages) and 25–40 % faster than 16×16 patches on
  // 4 waves (FM = 8, one wave per SIMD) on every attack shape — two waves per SIMD keep the
  // matrix pipe fed through each other's LDS reads, DMA issue and barriers.
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
    if (k.a.Cout <= 64)
      return pro ? launch_halo_tile<T, Small64, true, false>(k, st)
                 : launch_halo_tile<T, Small64, false, false>(k, st);
    return pro ? launch_halo_tile<T, Small, true, true>(k, st)
               : launch_halo_tile<T, Small, false, true>(k, st);
  });
  return MIA_OK;
}

}  // namespace mia

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
