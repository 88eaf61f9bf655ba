// Shared pieces of the implicit-GEMM convolution kernels on CDNA4 MFMA (gfx950), NHWC:
// conv_mfma.hip (generic im2col tiles: any tap window / stride / output placement, multi-group)
// and conv_halo.hip (stride-1 3×3 layers on square output tiles with the input halo staged once
// per channel block). Operand tiles are rows of 128 B (one K-step slice of a pixel or of an
// output channel), filled by LDS-DMA with the bank swizzle applied through the source chunk.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "mia_common.h"

namespace mia {

struct ConvGroup {
  const void* w;
  int kpad, kh, kw, pad_y, pad_x, ho, wo, ay, by, ax, bx, blk0, nbm, m;
  const void* w_split;  // fp32 pre-split weights (mia_conv_args.w_split) or nullptr
  // batched independent convs (mia_conv2d_batched): this group reads images n_in … n_in + N − 1
  // of x, writes images n_out … of y (and the per-pixel aux operands), and reads the per-channel
  // operands (bias, act_slope, mask_slope) at channel offset c_off; 0 otherwise
  int n_in, n_out, c_off;
};
constexpr int MIA_MAX_GROUPS = 16;

// N·H·W as the int of ConvGroup::m, saturated: the product is formed before the argument checks
// (which reject anything ≥ 2^31), so it must not overflow on its way there (signed-overflow UB,
// found by the host sanitizer build, tools/asan/host_abi_check.cpp)
inline int pixels_clamped(int n, int h, int w) {
  const int64_t m = (int64_t)n * h * w;
  return m < 0 ? -1 : (m > 0x7fffffff ? 0x7fffffff : (int)m);
}

struct ConvK {
  mia_conv_args a;  // x, y, N, H/W = INPUT dims, Cin, Cout and the epilogue fields
  int stride, HT, WT, ystride, cout_mod, log2cin, n_first_max, ng, nblk, nbn;
  int prered;                    // register epilogues: pre-reduce the sums across the M waves in
                                 // LDS before the atomics; on for the channel sum (SE pool) only:
                                 // measured, the extra barrier costs more than it saves for the
                                 // sdot / q sums of the StyledConv dgrads
  int batched;                   // groups carry image / channel offsets: LDS-staged epilogue only
  int prio;                      // X6B tile: s_setprio(1) around the MFMA blocks
  // deterministic sums (mia_common.h RedQ): partial slots of sdot (q 0), bab_q (1), csum (2)
  float* red_part;
  int red_nslots, red_count;     // slots per output; outputs per quantity (N·Cout)
  int red_px;                    // LDS-staged epilogue: one slot per output pixel (small images)
  int ysplit;                    // > 0: output channel co goes to plane co / ysplit, channel
  int64_t yplane;                // co % ysplit; planes yplane elements apart (mia_conv2d_planes)
  int64_t wn;                    // elements between the images' weight matrices (0: one shared
                                 // [Cout][Kpad]; > 0: per-image modulated weights, mia_conv3x3_wmod,
                                 // the 2-byte halo kernel only)
  ConvGroup g[MIA_MAX_GROUPS];
};

// Output base of a block whose columns start at n0 (all inside one plane: ysplit is a multiple of
// every tile width): y + plane·yplane − plane·ysplit, so that y + m·ystride + co lands at
// (plane, m, co − plane·ysplit) with ystride = ysplit.
template <typename T>
__device__ __forceinline__ T* y_base(const ConvK& k, int n0) {
  T* y = (T*)k.a.y;
  if (k.ysplit > 0 && y) {
    const int pl = n0 / k.ysplit;
    y += pl * (k.yplane - k.ysplit);
  }
  return y;
}


// the partial of quantity q (0 sdot, 1 bab_q, 2 csum) of contributor `slot` to output i = n·Cout+c
__device__ __forceinline__ void red_put(const ConvK& k, int q, int slot, int i, float v) {
  red_store(k.red_part, k.red_nslots, k.red_count, q, slot, i, v);
}

// Slots of the register epilogues (halo_epilogue / halo_epilogue_f): a contributor is one wave's
// FM rows × 16 columns of the (Hg × Wg) output grid, or — with the LDS pre-reduction across the
// nwm wave rows — the block's FM·nwm rows × 16 columns.
__host__ __device__ __forceinline__ int halo_red_h(int FM, int nwm, bool lds_red) {
  return lds_red && nwm > 1 ? FM * nwm : FM;
}
__device__ __forceinline__ int halo_red_slot(int y_first, int x0, int h, int Wg) {
  return (y_first / h) * (Wg >> 4) + (x0 >> 4);
}
inline int halo_red_slots(int Hg, int Wg, int FM, int nwm, bool lds_red) {
  return (Hg / halo_red_h(FM, nwm, lds_red)) * (Wg / 16);
}
// open the launch's reductions (nslots contributors per output) / add them up after it
int conv_red_begin(ConvK& k, RedQ& r, int nslots, hipStream_t st, bool zero = false);

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

static __device__ __attribute__((aligned(16))) uint4 g_zero16[4];  // zero source for masked DMA lanes

__device__ __forceinline__ int xcd_remap(int b, int nblk) {
  // Blocks are dealt round-robin over the 8 XCDs; give each XCD a contiguous run of logical tiles
  // so tiles sharing A rows / B columns hit the same L2 (bijective for any nblk).
  if (nblk < 16) return b;
  const int xcd = b & 7, q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

// Bank swizzle of a 128-B tile row: stored chunk = chunk ^ fsw(row). ds_read_b128 serves a wave
// in 4 lane groups ({0–3,12–15,20–27}, {4–11,16–19,28–31}, +32), each one LDS cycle when its 16
// lanes hit 16 distinct 4-bank slots (MI355X_MICROARCH.md §LDS). A fragment read takes 16
// consecutive rows (lane & 15) and chunks q, q^1 (lane >> 4): with rows of 128 B the parity of a
// row picks the bank half, and 2·((row >> 1) & 3) makes every window of 16 consecutive rows —
// at ANY start row — conflict-free (found by exhaustive search; the classic (row >> 1) & 7 is
// conflict-free only for windows starting at row ≡ 0, 1 mod 4, which the halo kernel's
// tap-shifted reads do not respect).
__device__ __forceinline__ int fsw(int row) { return ((row >> 1) & 3) << 1; }


__device__ __forceinline__ int div_kw(int t, int kw) {
  return kw == 3 ? (t * 11) >> 5 : (kw == 2 ? t >> 1 : t);  // exact for t < 9
}

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
// fp32 operands on the bf16 matrix pipe (the default fp32 arithmetic of libmiattack).
// Each fp32 value splits EXACTLY into three bf16 terms, a = hi + mid + lo: hi = a with the low 16
// mantissa bits cleared (8 significant bits), r = a − hi is exact and has ≤ 16 significant bits,
// mid = r truncated the same way, lo = r − mid is exact with ≤ 8 significant bits, so it is a
// bf16 value as is. The product a·b keeps the six terms of order ≥ 2^-16 (hh, hm, mh, hl, lh, mm);
// the three dropped ones (ml, lm, ll) are below 2^-23·|ab| together, the size of one fp32
// rounding of the product (2^-24·|ab|) — the precision of the native v_mfma_f32_16x16x4_f32 — and
// every bf16×bf16 product is exact in the fp32 accumulator. Six products of 16 k on three
// v_mfma_f32_16x16x32_bf16 (16 cycles each) replace four v_mfma_f32_16x16x4_f32 (32 cycles each):
// 2.7× the fp32 matrix rate. Lane group q holds k = 4q..4q+3 of the chunk in both operands, so the
// 8 bf16 slots of a lane are two k-quads of terms, paired as (A | B):
//   (hi, mid | hi, hi) = hh + mh,  (hi, lo | mid, hi) = hm + lh,  (mid, hi | mid, lo) = mm + hl.
struct Split3 {
  bf16x8 hm, hl, mh;  // (hi, mid), (hi, lo), (mid, hi) packed 8-slot operands
};
__device__ __forceinline__ unsigned pack_hi16(float a0, float a1) {
  // high halves of two fp32 words → one packed bf16 pair (exact: the low halves are zero)
  return __builtin_amdgcn_perm(__builtin_bit_cast(unsigned, a1), __builtin_bit_cast(unsigned, a0),
                               0x07060302u);
}
__device__ __forceinline__ Split3 split3(const f32x4& a) {
  float h[4], m[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    // (a scalar copy first: clang's __builtin_bit_cast of a vector-element lvalue reads element 0)
    const float x = a[e];
    h[e] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, x) & 0xffff0000u);
    const float r = x - h[e];
    m[e] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, r) & 0xffff0000u);
    l[e] = r - m[e];
  }
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
  const u32x2 H = {pack_hi16(h[0], h[1]), pack_hi16(h[2], h[3])};
  const u32x2 M = {pack_hi16(m[0], m[1]), pack_hi16(m[2], m[3])};
  const u32x2 L = {pack_hi16(l[0], l[1]), pack_hi16(l[2], l[3])};
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  Split3 s;
  s.hm = __builtin_bit_cast(bf16x8, (u32x4){H[0], H[1], M[0], M[1]});
  s.hl = __builtin_bit_cast(bf16x8, (u32x4){H[0], H[1], L[0], L[1]});
  s.mh = __builtin_bit_cast(bf16x8, (u32x4){M[0], M[1], H[0], H[1]});
  return s;
}
__device__ __forceinline__ f32x4 mfma_split3(const Split3& A, const Split3& B, f32x4 c) {
  // B slots: (hi, hi), (mid, hi), (mid, lo) — built from the same three packed pairs
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  const u32x4 bhm = __builtin_bit_cast(u32x4, B.hm), bhl = __builtin_bit_cast(u32x4, B.hl);
  const bf16x8 bhh = __builtin_bit_cast(bf16x8, (u32x4){bhm[0], bhm[1], bhm[0], bhm[1]});
  const bf16x8 bml = __builtin_bit_cast(bf16x8, (u32x4){bhm[2], bhm[3], bhl[2], bhl[3]});
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.mh, bml, c, 0, 0, 0);         // mm + hl
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.hl, B.mh, c, 0, 0, 0);        // hm + lh
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(A.hm, bhh, c, 0, 0, 0);      // hh + mh
}
// ---- pre-split operands (conv_halo_x6.hip, conv_mfma.hip X6B) ---------------------------------
// A pre-split operand quad (4 consecutive k) is a 16-B [hi×4 | mid×4] record + an 8-B [lo×4]
// record (bf16). With a lane's registers laid out (lo, hi, mid), the tuples (hi, mid) and (lo, hi)
// are register windows and three MFMAs give the six products of split3:
//   (hi,mid)·(hi,mid) = hh + mm,  (lo,hi)·(hi,mid) = lh + hm,  (hi,mid)·(lo,hi) = hl + mh.
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// 8-byte lo slot of logical quad q in a 64-B lo row: 2·((row >> 2) & 3) XOR keeps every window of
// 16 consecutive rows × 2 adjacent quads on 32 distinct 8-byte bank slots (ds_read_b64), and moves
// 16-byte pairs of slots together (the weight planes are DMA'd in 16-byte lanes).
__device__ __forceinline__ int lsw(int row) { return ((row >> 2) & 3) << 1; }

// exact split of 4 fp32 values (see conv_common.h split3): [hi×4 | mid×4] and [lo×4] as bf16
__device__ __forceinline__ void split_quad(const f32x4& a, u32x4& hm, u32x2& lo) {
  float h[4], m[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = a[e];  // scalar copy (bit_cast of a vector element reads element 0)
    h[e] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, x) & 0xffff0000u);
    const float r = x - h[e];
    m[e] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, r) & 0xffff0000u);
    l[e] = r - m[e];
  }
  hm = u32x4{pack_hi16(h[0], h[1]), pack_hi16(h[2], h[3]), pack_hi16(m[0], m[1]),
             pack_hi16(m[2], m[3])};
  lo = u32x2{pack_hi16(l[0], l[1]), pack_hi16(l[2], l[3])};
}

// the six products of one 16-k quad group: (hi,mid)(hi,mid) + (lo,hi)(hi,mid) + (hi,mid)(lo,hi)
__device__ __forceinline__ f32x4 mfma_x6(const u32x4& ahm, const u32x2& al, const u32x4& bhm,
                                         const u32x2& bl, f32x4 c) {
  const bf16x8 AHM = __builtin_bit_cast(bf16x8, ahm), BHM = __builtin_bit_cast(bf16x8, bhm);
  const bf16x8 ALH = __builtin_bit_cast(bf16x8, u32x4{al[0], al[1], ahm[0], ahm[1]});
  const bf16x8 BLH = __builtin_bit_cast(bf16x8, u32x4{bl[0], bl[1], bhm[0], bhm[1]});
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(AHM, BLH, c, 0, 0, 0);  // hl + mh
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ALH, BHM, c, 0, 0, 0);  // lh + hm
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(AHM, BHM, c, 0, 0, 0);  // hh + mm
}

#ifdef MIA_F32_NATIVE
// A/B build (MIA_F32_ARITH=native): the fp32 convs on the native fp32 matrix instruction
template <>
__device__ __forceinline__ f32x4 mfma_chunk<float>(const f32x4& a, const f32x4& b, f32x4 c) {
  // fp32: lane group q holds k = 4q..4q+3 of the chunk; step s uses k = 4q+s for both operands
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}
#else
template <>
__device__ __forceinline__ f32x4 mfma_chunk<float>(const f32x4& a, const f32x4& b, f32x4 c) {
  return mfma_split3(split3(a), split3(b), c);
}
#endif

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

// 8 consecutive elements of T as fp32
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const typename Vec<T>::type t = *(const typename Vec<T>::type*)p;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)t[e];
  } else {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[e + 4] = b[e]; }
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    typename Vec<T>::type t;
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = (T)v[e];
    *(typename Vec<T>::type*)p = t;
  } else {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
}
__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[e + 4] = b[e]; }
}

// 4 consecutive elements of T as fp32 (8-byte or 16-byte access)
template <typename T>
__device__ __forceinline__ void load4(const T* p, float (&v)[4]) {
  if constexpr (sizeof(T) == 2) {
    typedef T t4 __attribute__((ext_vector_type(4)));
    const t4 t = *(const t4*)p;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (float)t[e];
  } else {
    const f32x4 a = *(const f32x4*)p;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = a[e];
  }
}
template <typename T>
__device__ __forceinline__ void store4(T* p, const float (&v)[4]) {
  if constexpr (sizeof(T) == 2) {
    typedef T t4 __attribute__((ext_vector_type(4)));
    t4 t;
#pragma unroll
    for (int e = 0; e < 4; ++e) t[e] = (T)v[e];
    *(t4*)p = t;
  } else {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  }
}

constexpr int ROWB = 128;  // bytes per tile row (one K-step slice)

// Tile configurations: WM×WN waves, each wave FM×FN 16×16 fragments; STAGES-deep DMA ring.
//   128×64  / 128×128 : 4 waves, 2 stages, 2 blocks per CU (small M, Cout ≤ 64)
//   256×128           : 8 waves, 3 stages, 1 block per CU (large M: 85 FLOP per staged byte,
//                       two K-steps of DMA in flight behind a counted vmcnt)
template <int WM_, int WN_, int FM_, int FN_, int STAGES_>
struct Tile {
  static constexpr int WM = WM_, WN = WN_, FM = FM_, FN = FN_, STAGES = STAGES_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  static constexpr int A_INS = BM / (8 * NW), B_INS = BN / (8 * NW);  // 1-KB DMA pieces/wave/step
  static constexpr int STAGE = (BM + BN) * ROWB;
  static constexpr int EROWS = BM < 128 ? BM : 128;  // rows staged per epilogue pass
  static constexpr int ES = BN + 4;                  // fp32 words per staged row (bank pad)
  static_assert(A_INS >= 1 && B_INS >= 1 && A_INS * 8 * NW == BM && B_INS * 8 * NW == BN, "");
};

// ---- shared epilogue --------------------------------------------------------------------------
// Stages the fp32 accumulator tile in LDS (EROWS rows per pass), then works on 8-channel vectors:
// sdot reduction, out_scale, noise, bias, tap-MSE term, ReLU mask, act_out, accumulate, store.
// rowm(local_row) gives the GEMM row (output pixel index m) of a tile row, or −1 past the end;
// `single` = every row of the tile belongs to image n_single. Waves with index ≥ TL::NW (a
// block's DMA-only waves) take part in the barriers only.
template <typename T, typename TL, typename RowM>
__device__ __forceinline__ void conv_epilogue(const ConvK& k, const ConvGroup& G,
                                              f32x4 (&acc)[TL::FM][TL::FN], char* smem, int n0,
                                              bool single, int n_single, RowM rowm,
                                              int slot = 0) {
  constexpr int WN = TL::WN, FM = TL::FM, FN = TL::FN, NT = TL::NT, NW = TL::NW;
  constexpr int BM = TL::BM, BN = TL::BN, ES = TL::ES, EROWS = TL::EROWS;
  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const bool worker = wid < NW;
  const int frow = lane & 15, fq = lane >> 4;
  const int HWo = G.ho * G.wo;
  float* tile = (float*)smem;
  const int Cout = p.Cout;
  constexpr int CPR = BN / 8;          // 8-channel chunks per row
  constexpr int RPP = NT / CPR;        // rows per pass
  const int cc = tid % CPR, r0 = tid / CPR;
  const int col = n0 + cc * 8;
  const bool col_ok = col < Cout;      // Cout % 8 == 0 (host check)
  const T* AX = (const T*)p.aux_x;
  const T* TA = (const T*)p.tap_a;
  const T* TT = (const T*)p.tap_t;
  const T* MA = (const T*)p.mask_a;
  T* __restrict__ Y = y_base<T>(k, n0);
  float part[8], partq[8], pcs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) part[e] = partq[e] = pcs[e] = 0.f;
  // encoder features: PReLU act / mask slopes per column
  float aslope8[8], mslope8[8];
  const bool prelu = p.act_out == MIA_ACT_PRELU;
#pragma unroll
  for (int e = 0; e < 8; ++e) aslope8[e] = mslope8[e] = 0.f;
  if (prelu && col_ok) load8f(p.act_slope + G.c_off + col, aslope8);
  if (p.mask_slope && col_ok) load8f(p.mask_slope + G.c_off + col, mslope8);
  const bool bab = p.bab_demod != nullptr;
  float bbias8[8];
  if (bab) {
    if (p.bab_bias && col_ok) {
      load8f(p.bab_bias + col, bbias8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bbias8[e] = 0.f;
    }
  }

  // per-column epilogue constants, loaded once (single-image tiles: out_scale too)
  float bias8[8], osc8[8];
  const int cm0 = p.shuffle_out ? col % k.cout_mod : col;
  n_single += G.n_out;  // batched groups: the group's first output image
  if (p.bias && col_ok) load8f(p.bias + G.c_off + cm0, bias8);
  if (p.out_scale && single && col_ok) load8f(p.out_scale + (size_t)n_single * k.cout_mod + cm0, osc8);
  constexpr int ITERS = EROWS / RPP;
  static_assert(ITERS * RPP == EROWS, "");

  for (int h = 0; h < BM / EROWS; ++h) {
    const int wrow0 = wm * FM * 16;
    if (worker && wrow0 >= h * EROWS && wrow0 < (h + 1) * EROWS) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            tile[(wrow0 - h * EROWS + 16 * i + fq * 4 + r) * ES + wn * FN * 16 + 16 * j + frow] =
                acc[i][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int rr = r0 + it * RPP;
      const int row = worker ? rowm(h * EROWS + rr) : -1;
      if (row >= 0 && col_ok) {
        float v[8];
        load8f(tile + rr * ES + cc * 8, v);
        const int ng = row / HWo;  // image within the group
        const int n = single ? n_single : ng + G.n_out;
        // output placement (aux operands share the output's pixel grid, channel stride Cout)
        const int pix = row - ng * HWo;
        const int y = pix / G.wo, x = pix - (pix / G.wo) * G.wo;
        int cm = col, yo, xo;
        if (p.shuffle_out) {
          const int ph = col / k.cout_mod;
          cm = col - ph * k.cout_mod;
          yo = 2 * y + (ph >> 1);
          xo = 2 * x + (ph & 1);
        } else {
          yo = G.ay * y + G.by;
          xo = G.ax * x + G.bx;
        }
        const size_t aoff = ((size_t)(n * k.HT + yo) * k.WT + xo) * Cout + col;
        float xv[8];
        if (p.sdot || bab) load8<T>(AX + aoff, xv);
        if (p.sdot) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float c = v[e] * apply_act(xv[e], p.act_aux);
            if (single) part[e] += c;
            else red_put(k, 0, pix, n * Cout + col + e, c);  // one slot per output pixel
          }
        }
        if (Y) {
          const size_t off = ((size_t)(n * k.HT + yo) * k.WT + xo) * k.ystride + cm;
          if (p.out_scale) {
            if (!single) load8f(p.out_scale + (size_t)n * k.cout_mod + cm, osc8);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= osc8[e];
          }
          if (p.noise) {
            const float nz = p.noise_w * p.noise[yo * k.WT + xo];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += nz;
          }
          if (p.bias) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bias8[e];
          }
          float ma[8];
          if (TA) {
            float tt[8];
            load8<T>(TA + aoff, ma);  // the tap tensor doubles as the mask when they coincide
            load8<T>(TT + aoff, tt);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += p.tap_coef * (ma[e] - tt[e]);
          }
          if (MA) {
            if (MA != TA) load8<T>(MA + aoff, ma);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = ma[e] > 0.f ? v[e] : mslope8[e] * v[e];
          }
          if (prelu) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : aslope8[e] * v[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], p.act_out);
          }
          if (p.accumulate) {
            float yo8[8];
            load8<T>(Y + off, yo8);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += yo8[e];
          }
          if (bab) {
            // fused StyledConv backward front of the layer whose activation is aux_x
            float dm8[8];
            load8f(p.bab_demod + (size_t)n * Cout + col, dm8);
            const float nz = p.bab_noise ? p.bab_noise_w * p.bab_noise[yo * k.WT + xo] : 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float gr = lrelu_s2_grad(xv[e]);
              const float gp = v[e] * gr;
              const float c = gp * (xv[e] * lrelu_s2_inv_grad(xv[e]) - nz - bbias8[e]);
              if (single) partq[e] += c;
              else red_put(k, 1, pix, n * Cout + col + e, c);
              v[e] = gp * dm8[e];
            }
          }
          if (p.csum) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              if (single) pcs[e] += v[e];
              else red_put(k, 2, pix, n * Cout + col + e, v[e]);
            }
          }
          store8<T>(Y + off, v);
        }
      }
    }
    __syncthreads();
  }

  if (bab && single) {
    // q partials: the same shuffle + LDS reduction as sdot below (before it reuses the LDS)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      for (int o = CPR; o < 64; o <<= 1) partq[e] += __shfl_xor(partq[e], o, 64);
    float* red = (float*)smem;
    if (worker && lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wid * BN + lane * 8 + e] = partq[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < Cout) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += red[w * BN + tid];
      red_put(k, 1, slot, n_single * Cout + n0 + tid, s);  // the block's slot
    }
    __syncthreads();
  }
  if (p.csum && single) {  // Σ_p y partials: the same reduction as sdot below
#pragma unroll
    for (int e = 0; e < 8; ++e)
      for (int o = CPR; o < 64; o <<= 1) pcs[e] += __shfl_xor(pcs[e], o, 64);
    float* red = (float*)smem;
    if (worker && lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wid * BN + lane * 8 + e] = pcs[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < Cout) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += red[w * BN + tid];
      red_put(k, 2, slot, n_single * Cout + n0 + tid, s);
    }
    __syncthreads();
  }
  if (p.sdot && single) {
    // reduce the per-thread partial sums of equal channel chunks: lanes cc, cc+CPR, … of a wave
    // by shuffles, then the waves through LDS, one partial per channel per block (its slot)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      for (int o = CPR; o < 64; o <<= 1) part[e] += __shfl_xor(part[e], o, 64);
    float* red = (float*)smem;  // [NW waves][BN]
    if (worker && lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wid * BN + lane * 8 + e] = part[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < Cout) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += red[w * BN + tid];
      red_put(k, 0, slot, n_single * Cout + n0 + tid, s);
    }
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform n ≤ 16 (the immediate must be a constant)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
  }
}

// fp32 stride-1 3×3 layers with pre-split weights, operands split once (conv_halo_x6.hip)
bool conv_halo_x6_eligible(const ConvK& k, int dtype);
int launch_conv_halo_x6(ConvK& k, hipStream_t st);
// halo-tiled stride-1 3×3 path (conv_halo.hip)
bool conv_halo_eligible(const ConvK& k, int dtype);
int launch_conv_halo(ConvK& k, int dtype, hipStream_t st);
// up-sampling StyledConv forward, halo-tiled interior (conv_upconv.hip)
bool upconv_halo_eligible(int dtype, int R, int Cin, int Cout);
int launch_upconv_halo(const void* x, const void* w_up, const void* w_up_split, void* t, int N,
                       int R, int Cin, int Cout, int act_in, const float* style, int dtype,
                       hipStream_t st);
// 64 → 64-channel stride-1 layers, weights resident in VGPRs, persistent (conv_wres.hip)
bool conv_wres_eligible(const ConvK& k, int dtype);
int launch_conv_wres(ConvK& k, int dtype, hipStream_t st);
bool conv_wres128_eligible(const ConvK& k, int dtype);
int launch_conv_wres128(ConvK& k, int dtype, hipStream_t st);
bool conv_wres32_eligible(const ConvK& k, int dtype);
int launch_conv_wres32(ConvK& k, int dtype, hipStream_t st);
// thin-channel layers: VGG conv1_1 forward and its input gradient (conv_thin.hip)
bool conv_thin_eligible(const ConvK& k, int dtype);
bool conv_thin32_eligible(const ConvK& k, int dtype);
int launch_conv_thin32(ConvK& k, int dtype, hipStream_t st);
int launch_conv_thin(ConvK& k, int dtype, hipStream_t st);

}  // namespace mia
