// Register epilogue of the halo-tiled conv kernels (conv_halo.hip, conv_wres.hip): the MFMAs
// compute D = W·X̃ᵀ (output channels × patch pixels), so for every fragment a lane holds 4
// consecutive output channels of one pixel; every per-element operation of conv_epilogue
// (conv_common.h, same order and semantics) runs in registers with 8-/16-byte aux loads and
// 16-byte stores. halo_epilogue: runtime features; halo_epilogue_f<F>: specialised for feature
// mask F (epi::*), with every aux load of a row chunk hoisted.
#pragma once
#include "conv_common.h"

namespace mia {

__device__ __forceinline__ void ld4f(const float* p, float (&v)[4]) {
  const f32x4 a = *(const f32x4*)p;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = a[e];
}

// Epilogue straight from the accumulators (REG kernels). Their MFMAs compute D = W·X̃ᵀ (output
// channels × patch pixels), so for every fragment a lane holds 4 consecutive output channels of
// one pixel: each per-element operation of conv_epilogue (same order, same semantics) runs in
// registers with 8-/16-byte aux loads and stores and no LDS staging. The sdot / q reductions sum
// a lane's pixels, then the 16 pixel lanes of a channel group by shuffles, then one partial per
// channel per wave into the launch's reduction slots (red_put; added up in order after it).
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
  T* __restrict__ Y = y_base<T>(k, n0);
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
            partq[j][e] += gp * (xv[e] * lrelu_s2_inv_grad(xv[e]) - bnz - bbv[j][e]);
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
    // this wave's FM rows × 16 columns are one contributor slot (halo_red_slot)
    const int slot = halo_red_slot(y0 + wm * FM, x0, FM, W);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = cl + 16 * j;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = part[j][e], b = partq[j][e], cs = pcs[j][e];
        a = row16_sum(a);
        b = row16_sum(b);
        cs = row16_sum(cs);
        if (px == 0 && c < Cout) {
          const int i = n * Cout + c + e;
          if (p.sdot) red_put(k, 0, slot, i, a);
          if (bab) red_put(k, 1, slot, i, b);
          if (p.csum) red_put(k, 2, slot, i, cs);
        }
      }
    }
  }
}

// Epilogue feature mask (compile-time specialisations of halo_epilogue for the launches the
// attack makes; any other combination runs the runtime-generic halo_epilogue).
namespace epi {
constexpr int OSC = 1, NOISE = 2, BIAS = 4, TAP = 8, MASK = 16, ACC = 32, SDOT = 64, BAB = 128;
constexpr int RELU = MIA_ACT_RELU << 8, LRELU = MIA_ACT_LRELU_S2 << 8, PRELU = MIA_ACT_PRELU << 8;
// encoder features: the mask keeps slope·v (PReLU backward, mask_slope), channel sum (csum)
constexpr int MSL = 1024, CSUM = 2048;
}  // namespace epi

template <typename T>
struct Raw4 {  // 4 consecutive elements of T, loaded raw (8 or 16 bytes)
  typedef T type __attribute__((ext_vector_type(4)));
};

// The same operations as halo_epilogue for one feature mask F, straight-line: every aux load of
// the tile is issued first (one wait instead of one per fragment — a wait also drains the stores
// issued before it), then the arithmetic and the 16-byte stores.
// Per-pixel aux operands of FMC fragment rows (noise, stored activation, tap pair, mask, old y).
template <typename T, int FMC, int FN>
struct EpiRows {
  typedef typename Raw4<T>::type R4;
  float nz[FMC], bnz[FMC];
  R4 rx[FMC][FN], rta[FMC][FN], rtt[FMC][FN], rma[FMC][FN], ryo[FMC][FN];
};

template <typename TL>
struct EpiChunk {  // rows per aux-load chunk (bounds the live registers for tall wave tiles)
  static constexpr int FMC = TL::FM < 4 ? TL::FM : 4;
};

// Per-lane partial sums of the reductions (sdot, q, csum), kept across calls by a caller that
// flushes them itself (conv_thin.hip: one flush per image run instead of one per call).
template <int FN>
struct EpiSums {
  float part[FN][4], partq[FN][4], pcs[FN][4];
};

// Per-channel epilogue constants of one image (demod / out scale, bias, the bias-act backward's
// demod and bias, mask and PReLU slopes). A persistent caller that keeps a DMA in flight across
// its epilogue loads them BEFORE issuing the DMA (epi_chan_load) and passes them in: loaded inside
// the epilogue, their wait (vmcnt counts in issue order) would also wait for the DMA.
template <int FN>
struct EpiChan {
  f32x4 osc[FN], bia[FN], dmv[FN], bbv[FN], msl[FN], asl[FN];
};

template <int F, int FN>
__device__ __forceinline__ void epi_chan_load(const ConvK& k, EpiChan<FN>& E, int n, int cl) {
  const mia_conv_args& p = k.a;
  const int Cout = p.Cout;
  const f32x4 one = {1.f, 1.f, 1.f, 1.f}, zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = cl + 16 * j;
    E.osc[j] = one;
    E.bia[j] = E.dmv[j] = E.bbv[j] = E.msl[j] = E.asl[j] = zero;
    if (c < Cout) {  // c ≡ 0 mod 4, Cout ≡ 0 mod 8: the whole quad is in range
      if constexpr ((F & epi::OSC) != 0)
        E.osc[j] = *(const f32x4*)(p.out_scale + (size_t)n * k.cout_mod + c);
      if constexpr ((F & epi::BIAS) != 0) E.bia[j] = *(const f32x4*)(p.bias + c);
      if constexpr ((F & epi::MSL) != 0) E.msl[j] = *(const f32x4*)(p.mask_slope + c);
      if constexpr (((F >> 8) & 3) == MIA_ACT_PRELU) E.asl[j] = *(const f32x4*)(p.act_slope + c);
      if constexpr ((F & epi::BAB) != 0) {
        E.dmv[j] = *(const f32x4*)(p.bab_demod + (size_t)n * Cout + c);
        // no bias: four zeros from the zero page (a load either way: no branch around it)
        E.bbv[j] = *(const f32x4*)(p.bab_bias ? p.bab_bias + c : (const float*)g_zero16);
      }
    }
  }
}

// (Hg, Wg): the output grid the rows index; default (p.H, p.W). The generic tile passes a virtual
// grid of 16-pixel rows (HWo / 16, 16), so that its linear pixel rows use the same indexing.
// pre: the per-pixel operands of a single-chunk wave tile already gathered by the caller (the
// weights-resident kernel prefetches them into LDS during its MFMAs); nullptr: loaded here.
template <typename T, typename TL, int F>
__device__ __forceinline__ void halo_epilogue_f(
    const ConvK& k, const f32x4 (&acc)[TL::FM][TL::FN], int n, int y0, int x0, int n0, int wm,
    int wn, int lane, int Hg = -1, int Wg = -1,
    const EpiRows<T, EpiChunk<TL>::FMC, TL::FN>* pre = nullptr, float* red = nullptr, int nwm = 1,
    int cw = 0, EpiSums<TL::FN>* keep = nullptr, const EpiChan<TL::FN>* chan = nullptr) {
  constexpr int FM = TL::FM, FN = TL::FN;
  constexpr bool OSC = F & epi::OSC, NOISE = F & epi::NOISE, BIAS = F & epi::BIAS;
  constexpr bool TAP = F & epi::TAP, MASK = F & epi::MASK, ACC = F & epi::ACC;
  constexpr bool SDOT = F & epi::SDOT, BAB = F & epi::BAB;
  constexpr bool MSL = F & epi::MSL, CSUM = F & epi::CSUM;
  constexpr int ACT = (F >> 8) & 3;
  static_assert(!MSL || MASK, "MSL is a mask variant");
  constexpr bool WIDE = sizeof(T) == 2 && FN % 2 == 0;
  typedef typename Raw4<T>::type R4;
  const mia_conv_args& p = k.a;
  const int H = Hg < 0 ? p.H : Hg, W = Hg < 0 ? p.W : Wg, Cout = p.Cout;
  const int px = lane & 15, lrow = lane >> 4;
  const int cl = n0 + wn * FN * 16 + (lrow << 2);
  T* __restrict__ Y = y_base<T>(k, n0);
  const T* AX = (const T*)p.aux_x;
  const T* TA = (const T*)p.tap_a;
  const T* TT = (const T*)p.tap_t;
  const T* MA = (const T*)p.mask_a;
  const bool ma_is_ta = MA == TA;

  bool cok[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) cok[j] = cl + 16 * j < Cout;
  EpiChan<FN> El;
  EpiChan<FN>& E = chan != nullptr ? *const_cast<EpiChan<FN>*>(chan) : El;
  if (chan == nullptr) epi_chan_load<F, FN>(k, El, n, cl);
  const auto& osc = E.osc;
  const auto& bia = E.bia;
  const auto& dmv = E.dmv;
  const auto& bbv = E.bbv;
  const auto& msl = E.msl;
  const auto& asl = E.asl;
  float part[FN][4], partq[FN][4], pcs[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) part[j][e] = partq[j][e] = pcs[j][e] = 0.f;
  // rows in chunks of FMC (the aux loads of a chunk are hoisted together; chunks bound the live
  // registers for tall wave tiles)
  constexpr int FMC = EpiChunk<TL>::FMC;
#pragma unroll
  for (int i0 = 0; i0 < FM; i0 += FMC) {
  EpiRows<T, FMC, FN> Rl;
  const bool have = pre != nullptr && FMC == FM;
  // the caller's operands by reference (a copy would double their registers)
  EpiRows<T, FMC, FN>& R = have ? *const_cast<EpiRows<T, FMC, FN>*>(pre) : Rl;
  float(&nz)[FMC] = R.nz;
  float(&bnz)[FMC] = R.bnz;
  R4(&rx)[FMC][FN] = R.rx;
  R4(&rta)[FMC][FN] = R.rta;
  R4(&rtt)[FMC][FN] = R.rtt;
  R4(&rma)[FMC][FN] = R.rma;
  R4(&ryo)[FMC][FN] = R.ryo;
  if (!have) {
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

  }  // !have
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
          v[e] = ma > 0.f ? v[e] : (MSL ? msl[j][e] * v[e] : 0.f);
        }
        if constexpr (ACT == MIA_ACT_RELU) v[e] = v[e] > 0.f ? v[e] : 0.f;
        if constexpr (ACT == MIA_ACT_LRELU_S2) v[e] = lrelu_s2(v[e]);
        if constexpr (ACT == MIA_ACT_PRELU) v[e] = v[e] > 0.f ? v[e] : asl[j][e] * v[e];
        if constexpr (ACC) v[e] += (float)ryo[i][j][e];
        if constexpr (BAB) {
          const float gr = lrelu_s2_grad(xv[e]);
          const float gp = v[e] * gr;
          partq[j][e] += gp * (xv[e] * lrelu_s2_inv_grad(xv[e]) - bnz[i] - bbv[j][e]);
          v[e] = gp * dmv[j][e];
        }
        if constexpr (CSUM) pcs[j][e] += v[e];
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
  if constexpr (SDOT || BAB || CSUM) {
    if (keep != nullptr) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          keep->part[j][e] += part[j][e];
          keep->partq[j][e] += partq[j][e];
          keep->pcs[j][e] += pcs[j][e];
        }
      return;
    }
    const bool lds_red = red != nullptr && nwm > 1;
    const int rh = halo_red_h(FM, nwm, lds_red);  // contributor rows: the wave's or the block's
    const int slot = halo_red_slot(lds_red ? y0 : y0 + wm * FM, x0, rh, W);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = cl + 16 * j;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a = part[j][e], b = partq[j][e], cs = pcs[j][e];
        if constexpr (SDOT) a = row16_sum(a);
        if constexpr (BAB) b = row16_sum(b);
        if constexpr (CSUM) cs = row16_sum(cs);
        if (lds_red) {  // (quantity, wave row, block channel) in LDS
          if (px == 0) {
            const int lc = c - n0 + e;
            int qi = 0;
            if constexpr (SDOT) red[(qi++ * nwm + wm) * cw + lc] = a;
            if constexpr (BAB) red[(qi++ * nwm + wm) * cw + lc] = b;
            if constexpr (CSUM) red[(qi++ * nwm + wm) * cw + lc] = cs;
          }
        } else if (px == 0 && c < Cout) {
          const int i = n * Cout + c + e;
          if constexpr (SDOT) red_put(k, 0, slot, i, a);
          if constexpr (BAB) red_put(k, 1, slot, i, b);
          if constexpr (CSUM) red_put(k, 2, slot, i, cs);
        }
      }
    }
    if (lds_red) {
      // the waves of one channel range meet here; the first wave row sums them (in wave order)
      // and stores one partial per channel for the block (nwm× fewer partials). LDS-only
      // hand-off: lgkmcnt(0) + s_barrier + a compiler barrier, no memory fence (a fence would
      // also wait for a persistent caller's halo DMA in flight)
      lds_handoff();
      if (wm == 0 && px == 0) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c = cl + 16 * j;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (c >= Cout) continue;
            const int lc = c - n0 + e;
            int qi = 0;
            const bool has[3] = {SDOT, BAB, CSUM};
#pragma unroll
            for (int qq = 0; qq < 3; ++qq) {
              if (!has[qq]) continue;
              float t = 0.f;
              for (int w = 0; w < nwm; ++w) t += red[(qi * nwm + w) * cw + lc];
              red_put(k, qq, slot, n * Cout + c + e, t);
              ++qi;
            }
          }
        }
      }
    }
  }
}

// Feature mask of a launch (−1: a combination without a specialisation, e.g. act_aux ≠ NONE).
static inline int epi_mask(const ConvK& k) {
  const mia_conv_args& a = k.a;
  if ((a.sdot || a.bab_demod) && a.act_aux != MIA_ACT_NONE) return -1;
  if (a.mask_slope && !a.mask_a) return -1;
  int f = 0;
  if (a.mask_slope) f |= epi::MSL;
  if (a.csum) f |= epi::CSUM;
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

}  // namespace mia
