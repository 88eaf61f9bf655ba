// Thin-channel 3×3 convolutions (stride 1, pad 1, NHWC; MFMA for 2-byte types, fp32 VALU for
// fp32): the VGG input layer
// conv1_1 (code/vgg.py:45, 3 → 64 channels; the image is padded to 8 channels) and its input
// gradient (64 → 8 channels, 3 real). Both move far more bytes than they compute (forward: 16 B
// read and 128 B written per pixel for 27·64 MACs; gradient: 128 B read and 16 B written), so they
// are HBM/TA-bound, not MFMA-bound. The implicit-GEMM tiles (conv_mfma.hip, conv_halo.hip) pad K
// or N to a 128-B operand row and re-stage the whole weight tensor per tile, which made these two
// launches run at ≈1 TB/s. Here:
//   * the weights live in VGPRs for the whole kernel (each wave loads them once);
//   * a wave computes 16 consecutive pixels of one image row per step with MFMA 16×16×32,
//     D[channel][pixel]; the pixel operand is gathered straight from global memory into VGPRs
//     (one 16-B vector per lane per K-chunk, the neighbours' re-reads hit L1/L2), and no block
//     barrier;
//   * forward stores (round 5): the 16 pixels × 64 channels of a group go through the wave's own
//     LDS slice, so each non-temporal store instruction writes 8 whole pixels (1 KB contiguous);
//     the round-4 form (lane-row swaps, each instruction writing half of 16 pixel rows) wrote at
//     2.5 TB/s where a plain fill writes 6.6–6.9: 431 → 308 µs per 128 × 256² call
//     (profiles/r05_thin_store_ab.txt);
//   * the gradient kernel stages each input pixel once per wave work item in LDS (9 taps read it);
//   * waves stride over the pixel groups / work items.
#include <type_traits>

#include "conv_common.h"
#include "halo_epilogue.h"

namespace mia {

template <typename T>
__device__ __forceinline__ typename Vec<T>::type ld16_or_zero(const T* p, bool ok) {
  typedef typename Vec<T>::type VT;
  VT v;
  if (ok) {
    v = *(const VT*)p;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (T)0.f;
  }
  return v;
}

// ---- forward, Cin = 8 (image padded to 8 channels) → COUT channels, + bias, act ----------------
// K = 9 taps × 8 channels = 72 in three MFMA K-chunks of 32 (chunk m, lane group fq → tap 4m+fq,
// taps ≥ 9 are zero; the weight matrix [Cout][Kpad ≥ 96] is zero there too).
template <typename T, int COUT>
__global__ __launch_bounds__(256) void conv_thin_in_kernel(const T* __restrict__ x,
                                                           const T* __restrict__ w, int kpad,
                                                           const float* __restrict__ bias, int act,
                                                           const float* __restrict__ slope,
                                                           T* __restrict__ y, int N, int H, int W) {
  typedef typename Vec<T>::type VT;
  constexpr int FN = COUT / 16;
  __shared__ __attribute__((aligned(16))) char stage[4 * 16 * 144];  // per wave 16 pixels
  const int lane = threadIdx.x & 63, frow = lane & 15, fq = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  VT wr[FN][3];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int m = 0; m < 3; ++m) wr[j][m] = *(const VT*)(w + (size_t)(16 * j + frow) * kpad + 8 * (4 * m + fq));
  float bs[FN][4], sl[FN][4];  // bias; PReLU slope (act = MIA_ACT_PRELU: the e4e input layer)
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bs[j][r] = bias ? bias[16 * j + 4 * fq + r] : 0.f;
      sl[j][r] = act == MIA_ACT_PRELU ? slope[16 * j + 4 * fq + r] : 0.f;
    }

  const int gpr = W / 16, ngroups = N * H * gpr;
  for (int g = wave; g < ngroups; g += nwaves) {
    const int row = g / gpr, xg = (g - row * gpr) * 16;
    const int n = row / H, yy = row - n * H;
    const int px = xg + frow;
    VT af[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int t = 4 * m + fq;  // lane-dependent tap
      const int dy = t / 3 - 1, dx = t - (t / 3) * 3 - 1;
      const int sy = yy + dy, sx = px + dx;
      const bool ok = t < 9 && sy >= 0 && sy < H && sx >= 0 && sx < W;
      af[m] = ld16_or_zero<T>(x + ((size_t)(n * H + (ok ? sy : 0)) * W + (ok ? sx : 0)) * 8, ok);
    }
    f32x4 acc[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < 3; ++m) acc[j] = mfma_chunk<T>(wr[j][m], af[m], acc[j]);
    }
    // lane (frow = pixel, fq) holds channels 16j + 4fq … +3 of its pixel: staged through the
    // wave's LDS slice so each store instruction writes 8 whole pixels (1 KB contiguous)
    static_assert(COUT == 64, "the staged store covers 16 pixels x 128 B");
    constexpr int PITCH = 144;  // bytes per staged pixel (36 dwords: conflict-free b64 writes)
    char* const sw = stage + (threadIdx.x >> 6) * 16 * PITCH;
    typedef T t4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[j][r] + bs[j][r];
        if (act == MIA_ACT_PRELU) v[r] = v[r] > 0.f ? v[r] : sl[j][r] * v[r];
        else v[r] = apply_act(v[r], act);
      }
      *(t4*)(sw + frow * PITCH + (16 * j + 4 * fq) * 2) = t4{(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
    }
    asm volatile("" ::: "memory");  // a wave's LDS accesses execute in order: no barrier needed
    T* yg = y + ((size_t)row * W + xg) * COUT;
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = 8 * i + (lane >> 3), c = lane & 7;
      const u4v v = *(const u4v*)(sw + p * PITCH + 16 * c);
      __builtin_nontemporal_store(v, (u4v*)(yg + p * COUT + 8 * c));
    }
    asm volatile("" ::: "memory");
  }
}

// ---- input gradient, CIN = 64 channels → 8 output channels (store, or accumulate into y) -------
// On sliding-window row strips: a work item is a 16-pixel column strip × THIN_SR output rows; the
// wave keeps a ring of 4 input rows (18 pixels × 128 B, 3 LDS-DMA pieces each, bank-swizzled
// through the source chunk as in conv_halo.hip) and per output row DMAs only the next input row,
// so each input row comes from L2 / HBM about once (rocprof: 2.24 → 1.27 GB fetched per 1.07 GB
// gradient against round 3's 2-row items, which were removed in round 6). The 9 taps × 2 K-chunks
// read the rows as MFMA B fragments; D[channel][pixel] with channel rows 0 … 15 (rows ≥ COUT zero
// weights); K = 9 taps × 64 in chunks of 32: chunk s = (tap s / 2, channels 32·(s & 1) + 8·fq …).
constexpr int THIN_SR = 16, THIN_HW = 18, THIN_SLOT = 3 * 1024, THIN_RING = 4;

template <typename T, int COUT>
__global__ __launch_bounds__(256) void conv_thin_out_strip_kernel(const T* __restrict__ g,
                                                                  const T* __restrict__ w,
                                                                  int kpad, T* __restrict__ y,
                                                                  int accumulate, int N, int H,
                                                                  int W) {
  typedef typename Vec<T>::type VT;
  constexpr int CIN = 64, S = 18;
  static_assert(COUT == 8, "");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, frow = lane & 15, fq = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  char* const ring = smem + wid * THIN_RING * THIN_SLOT;
  const int wave = blockIdx.x * 4 + wid, nwaves = gridDim.x * 4;
  VT wr[S];
#pragma unroll
  for (int s = 0; s < S; ++s)
    wr[s] = ld16_or_zero<T>(w + (size_t)(frow < COUT ? frow : 0) * kpad + 32 * s + 8 * fq,
                            frow < COUT);
  const T* zero = (const T*)g_zero16;
  const int gpr = W / 16, rbi = (H + THIN_SR - 1) / THIN_SR, nitems = N * rbi * gpr;

  // input row sy (18 pixels from x0 − 1) of image n into ring slot `slot`: pixel px of the slot
  // is a 128-B row, its 16-B chunk c stored at c ^ fsw(px)
  auto issue_row = [&](int n, int sy, int x0, int slot) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int px = q * 8 + (lane >> 3);
      const int sx = x0 + px - 1;
      const bool ok = px < THIN_HW && sy >= 0 && sy < H && sx >= 0 && sx < W;
      const T* src = ok ? g + ((size_t)(n * H + sy) * W + sx) * CIN + ((lane & 7) ^ fsw(px)) * 8
                        : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src,
                                       (lptr_t)(ring + slot * THIN_SLOT + q * 1024), 16, 0, 0);
    }
  };

  for (int it = wave; it < nitems; it += nwaves) {
    const int row = it / gpr, x0 = (it - row * gpr) * 16;
    const int n = row / rbi, y0 = (row - n * rbi) * THIN_SR;
    const int nr = min(THIN_SR, H - y0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the previous item's ring reads are done
    issue_row(n, y0 - 1, x0, 0);
    issue_row(n, y0, x0, 1);
    issue_row(n, y0 + 1, x0, 2);
    for (int r = 0; r < nr; ++r) {
      // output row y0 + r reads input rows y0 + r − 1 … + 1 (slots r, r + 1, r + 2 mod 4)
      if (r + 1 < nr) {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // slot (r + 3) % 4 held row y0 + r − 2: reads done
        issue_row(n, y0 + r + 2, x0, (r + 3) & 3);
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // all but the row just issued
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const char* hb = ring + ((r + t / 3) & 3) * THIN_SLOT;
        const int px = frow + t % 3;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const VT bf = *(const VT*)(hb + px * ROWB + (((4 * c + fq) ^ fsw(px)) << 4));
          acc = mfma_chunk<T>(wr[2 * t + c], bf, acc);
        }
      }
      const int yy = y0 + r;
      if (fq < COUT / 4) {
        float v[4] = {acc[0], acc[1], acc[2], acc[3]};
        T* yp = y + ((size_t)(n * H + yy) * W + x0 + frow) * COUT + 4 * fq;
        if (accumulate) {
          float yo[4];
          load4<T>(yp, yo);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += yo[e];
        }
        store4<T>(yp, v);
      }
    }
  }
}

// ---- 32 → 32-channel stride-1 3×3 layers (StyleGAN2 1024² StyledConvs, cm = 2) ----------------
// K = 9 taps × 32 channels: ONE MFMA 16×16×32 K-chunk per tap. The wave holds all 9 × 2 weight
// fragments in VGPRs (72 registers) and walks a contiguous run of 16-pixel groups (one image row
// segment each): per tap one 16-byte A gather per lane straight from global memory (the
// neighbours' re-reads hit L1 / L2), the optional modulation x·s[n][ci] on the fragment (PRO, the
// StyledConv forward), 2 MFMAs → D[channel][pixel]; the epilogue is the specialised register
// epilogue (halo_epilogue_f, FM = 1, FN = 2). The sdot / q / csum partials stay in registers over
// the run and are flushed (shuffles + one atomic per channel) when the image changes.
struct Thin32Tile {
  static constexpr int FM = 1, FN = 2;
};

// the reductions of image n: the 16 pixel lanes by shuffles, then one partial per channel into the
// work item's slot of image n (its chunk index: fixed by the image shape, not by N or the grid)
template <int EPI>
__device__ __forceinline__ void thin32_flush(const ConvK& k, EpiSums<2>& sums, int n, int slot,
                                             int frow, int fq) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float a = sums.part[j][e], b = sums.partq[j][e], cs = sums.pcs[j][e];
      if constexpr ((EPI & epi::SDOT) != 0) a = row16_sum(a);
      if constexpr ((EPI & epi::BAB) != 0) b = row16_sum(b);
      if constexpr ((EPI & epi::CSUM) != 0) cs = row16_sum(cs);
      const int c = 16 * j + 4 * fq + e;
      if (frow == 0) {
        if constexpr ((EPI & epi::SDOT) != 0) red_put(k, 0, slot, n * 32 + c, a);
        if constexpr ((EPI & epi::BAB) != 0) red_put(k, 1, slot, n * 32 + c, b);
        if constexpr ((EPI & epi::CSUM) != 0) red_put(k, 2, slot, n * 32 + c, cs);
      }
      sums.part[j][e] = sums.partq[j][e] = sums.pcs[j][e] = 0.f;
    }
}

// 16-pixel groups per work item (= per reduction slot) of the 32-channel kernel
constexpr int THIN32_CHUNK = 64;

template <typename T, bool PRO, int EPI>
__global__ __launch_bounds__(256) void conv_thin32_kernel(const ConvK k) {
  typedef typename Vec<T>::type VT;
  typedef Thin32Tile TL;
  constexpr bool RED = (EPI & (epi::SDOT | epi::BAB | epi::CSUM)) != 0;
  const mia_conv_args& p = k.a;
  const int lane = threadIdx.x & 63, frow = lane & 15, fq = lane >> 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
  const int H = p.H, W = p.W;
  const T* __restrict__ X = (const T*)p.x;
  const T* __restrict__ Wt = (const T*)k.g[0].w;
  const int kpad = k.g[0].kpad;
  VT wr[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) wr[t][j] = *(const VT*)(Wt + (size_t)(16 * j + frow) * kpad + t * 32 + fq * 8);
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;
  const int gpr = W / 16, gpi = H * gpr;
  // work items: THIN32_CHUNK consecutive 16-pixel groups of ONE image; item (n, c) adds its sums
  // into slot c of image n. The partition depends on the image's shape only — not on N or on the
  // grid — so an image's sums do not depend on the other images of the call (mia_common.h RedQ)
  const int S = (gpi + THIN32_CHUNK - 1) / THIN32_CHUNK;
  const int64_t nitems = (int64_t)p.N * S;
  EpiSums<TL::FN> sums;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) sums.part[j][e] = sums.partq[j][e] = sums.pcs[j][e] = 0.f;
  VT sv;
  // the 9 A gathers of group g (issued one group ahead: they land during the previous group's
  // MFMAs and epilogue)
  auto gather = [&](int64_t g, VT (&a)[9]) __attribute__((always_inline)) {
    const int n = (int)(g / gpi);
    const int rem = (int)(g - (int64_t)n * gpi);
    const int y = rem / gpr, x0 = (rem - y * gpr) * 16;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int sy = y + t / 3 - 1, sx = x0 + frow + t % 3 - 1;
      const bool ok = sy >= 0 && sy < H && sx >= 0 && sx < W;
      a[t] = ld16_or_zero<T>(X + ((size_t)(n * H + (ok ? sy : 0)) * W + (ok ? sx : 0)) * 32 + fq * 8,
                             ok);
    }
  };
  VT a_cur[9], a_nxt[9];
  for (int64_t it = wave; it < nitems; it += nwaves) {
    const int n = (int)(it / S), c = (int)(it - (int64_t)n * S);
    const int64_t g0 = (int64_t)n * gpi + (int64_t)c * THIN32_CHUNK;
    const int64_t g1 = g0 + min(THIN32_CHUNK, gpi - c * THIN32_CHUNK);
    if constexpr (PRO) {
      const float mul = lrelu_in ? SQRT2 : 1.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sv[e] = from_f<T>(p.in_scale[(size_t)n * 32 + fq * 8 + e] * mul);
    }
    gather(g0, a_cur);
    for (int64_t g = g0; g < g1; ++g) {
      const int rem = (int)(g - (int64_t)n * gpi);
      const int y = rem / gpr, x0 = (rem - y * gpr) * 16;
      if (g + 1 < g1) gather(g + 1, a_nxt);
      f32x4 acc[1][2] = {{f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}}};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        VT a = a_cur[t];
        if constexpr (PRO) modulate<T>(a, sv, lrelu_in);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[0][j] = mfma_chunk<T>(wr[t][j], a, acc[0][j]);
      }
      halo_epilogue_f<T, TL, EPI>(k, acc, n, y, x0, 0, 0, 0, lane, -1, -1, nullptr, nullptr, 1, 0,
                                  RED ? &sums : nullptr);
#pragma unroll
      for (int t = 0; t < 9; ++t) a_cur[t] = a_nxt[t];
    }
    if constexpr (RED) thin32_flush<EPI>(k, sums, n, c, frow, fq);
  }
}

static int grid_for(int64_t groups, int waves_per_cu = 32) {
  const int ncu = device_cu_count();
  const int64_t waves = std::min<int64_t>(groups, (int64_t)ncu * waves_per_cu);
  return (int)std::max<int64_t>(1, (waves + 3) / 4);
}

// ---- fp32 thin layers on the fp32 VALU ------------------------------------------------------
// In fp32 the two input layers are HBM-bound with ≈ 1.7 k real MACs per pixel (3 real image
// channels): on the fp32 VALU (v_fma_f32, fp32 products, no operand split) the FMAs take
// ≈ 0.5 ms per 128 × 256² images against ≈ 0.5 ms of HBM traffic, where the split-MFMA tiles ran
// at 1.3 ms (forward) / 3.5 ms (gradient). The padded image channels have all-zero weights; each
// block finds them from the weights (a channel with a nonzero weight is "real") and skips them —
// exact, since the skipped terms are products with zero weights (and the padded input channels
// are zero). Both kernels give each 16-lane group of a wave one 4-pixel row segment, so every
// global access is a contiguous 256-B pixel record (lane = 4 channels) and the segment's
// 3 × 6 input pixels are loaded once for its 4 × 9 taps.
__device__ __forceinline__ int64_t thin_seg_origin(int64_t seg, int H, int W, int& n, int& yy,
                                                   int& x0) {
  const int spr = W / 4;  // 4-pixel segments per row
  const int64_t row = seg / spr;
  x0 = (int)(seg - row * spr) * 4;
  n = (int)(row / H);
  yy = (int)(row - (int64_t)n * H);
  return row * W + x0;  // first pixel index of the segment
}

// forward, Cin = 8 → 64, + bias, act. Lane q of a group owns output channels 4q … 4q+3; the
// weights are transposed into LDS as [k][64] (one 16-B read per (tap, channel) serves the
// segment's 4 pixels × 4 channels). CM: the real input channels as a compile-time mask (0x07, the
// RGB image), or 0xff with the runtime mask cmask.
// HOIST (the RGB-mask instance): the segment's 3 × 6 input pixels are all loaded before the first
// FMA (one exposed load latency per segment instead of one per tap row; round 3, 1.10 → 0.90 ms per
// 128 × 256² call); the runtime-mask instance loads per tap row.
template <int CM, bool HOIST>
__device__ __forceinline__ void thin_in_f32_body(const float* __restrict__ x,
                                                 const float* __restrict__ wl, int cmask,
                                                 const f32x4 bs, const f32x4 sl, int act,
                                                 float* __restrict__ y, int N, int H, int W) {
  constexpr int CIN = 8, COUT = 64;
  const int tid = threadIdx.x, c0 = 4 * (tid & 15);
  const bool hi4 = (cmask >> 4) != 0;  // a real channel among 4 … 7: load the second half too
  const int64_t nseg = (int64_t)N * H * (W / 4);
  for (int64_t seg = (int64_t)blockIdx.x * 16 + (tid >> 4); seg < nseg;
       seg += (int64_t)gridDim.x * 16) {
    int n, yy, x0;
    const int64_t pix0 = thin_seg_origin(seg, H, W, n, yy, x0);
    f32x4 acc[4] = {bs, bs, bs, bs};
    f32x4 xh[HOIST ? 3 : 1][6];
    if constexpr (HOIST) {
#pragma unroll
      for (int ty = 0; ty < 3; ++ty) {
        const int sy = yy + ty - 1;
        const bool oky = sy >= 0 && sy < H;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const int sx = x0 + c - 1;
          const bool ok = oky && sx >= 0 && sx < W;
          xh[ty][c] = ok ? *(const f32x4*)(x + ((size_t)(n * H + sy) * W + sx) * CIN)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
#pragma unroll
    for (int ty = 0; ty < 3; ++ty) {
      const int sy = yy + ty - 1;
      if (sy < 0 || sy >= H) continue;
      f32x4 xa[6], xb[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        if constexpr (HOIST) {
          xa[c] = xh[ty][c];
        } else {
          const int sx = x0 + c - 1;
          const bool ok = sx >= 0 && sx < W;
          const float* xp = x + ((size_t)(n * H + sy) * W + (ok ? sx : 0)) * CIN;
          xa[c] = ok ? *(const f32x4*)xp : f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr (CM >> 4) xb[c] = ok && hi4 ? *(const f32x4*)(xp + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int tx = 0; tx < 3; ++tx)
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          if (!((CM >> ci) & 1)) continue;
          if (CM == 0xff && !((cmask >> ci) & 1)) continue;
          const f32x4 wv = *(const f32x4*)(wl + ((3 * ty + tx) * CIN + ci) * COUT + c0);
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const float xv = ci < 4 ? xa[p + tx][ci & 3] : xb[p + tx][ci & 3];
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[p][e] = fmaf(xv, wv[e], acc[p][e]);
          }
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      f32x4 o = acc[p];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (act == MIA_ACT_PRELU) o[e] = o[e] > 0.f ? o[e] : sl[e] * o[e];
        else o[e] = apply_act(o[e], act);
      }
      // non-temporal: the 2.15 GB output streams past L2 / MALL (−9 % per call)
      __builtin_nontemporal_store(o, (f32x4*)(y + (size_t)(pix0 + p) * COUT + c0));
    }
  }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void conv_thin_in_f32_kernel(
    const float* __restrict__ x, const float* __restrict__ w, int kpad,
    const float* __restrict__ bias, int act, const float* __restrict__ slope,
    float* __restrict__ y, int N, int H, int W) {
  constexpr int CIN = 8, COUT = 64, K = 9 * CIN;
  __shared__ __attribute__((aligned(16))) float wl[K * COUT];
  __shared__ int cmask_s;
  const int tid = threadIdx.x;
  if (tid == 0) cmask_s = 0;
  __syncthreads();
  int cm = 0;
  for (int i = tid; i < K * COUT; i += 256) {
    const int co = i / K, kk = i - co * K;
    const float v = w[(size_t)co * kpad + kk];
    wl[kk * COUT + co] = v;
    if (v != 0.f) cm |= 1 << (kk % CIN);
  }
  if (cm) atomicOr(&cmask_s, cm);
  __syncthreads();
  const int cmask = __builtin_amdgcn_readfirstlane(cmask_s);
  const int c0 = 4 * (tid & 15);
  f32x4 bs = {0.f, 0.f, 0.f, 0.f}, sl = {0.f, 0.f, 0.f, 0.f};
  if (bias) bs = *(const f32x4*)(bias + c0);
  if (act == MIA_ACT_PRELU) sl = *(const f32x4*)(slope + c0);
  if (cmask == 0x07) {
    thin_in_f32_body<0x07, true>(x, wl, cmask, bs, sl, act, y, N, H, W);
  } else {
    thin_in_f32_body<0xff, false>(x, wl, cmask, bs, sl, act, y, N, H, W);
  }
}

// input gradient, Cin = 64 → 8 output channels (store or accumulate). Lane q of a group holds
// the input channels 4q … 4q+3 of every tap and the weights of output channels 0 … 3 for them
// in VGPRs; the segment's 4 pixels × 4 output channels are reduced over the 16 lanes by DPP.
// Real output channels ≥ 4 (never the case for an RGB image) take a slower path with the weights
// as wave-uniform scalar loads, one pixel per lane.
// The 144 weights a lane needs are read from LDS per tap (held in VGPRs they took 209 VGPRs and
// 2 waves per SIMD); LDS layout [tap][e][q][co], so the 16 lanes of a group read 256 contiguous
// bytes (no bank conflict). Sliding-window row strips (below): a grid-strided 4-pixel segment
// loop re-read each input row for 3 output rows from L2 / HBM (rocprof: 5.5 GB fetched per
// 2.15 GB gradient; 2.5 GB with the strips). Round 6: the round-2 / round-3 launch modes
// (MIA_THIN_F32 0–2, bit-identical and slower) were removed.
constexpr int THIN_STRIP = 16;
template <bool ACC>
__global__ __launch_bounds__(256) void conv_thin_out_f32_kernel(
    const float* __restrict__ g, const float* __restrict__ w, int kpad, float* __restrict__ y,
    int N, int H, int W, int gen_blocks) {
  constexpr int CIN = 64, COUT = 8, K = 9 * CIN;
  __shared__ __attribute__((aligned(16))) float wl[9 * 4 * 16 * 4];
  __shared__ int cmask_s;
  const int tid = threadIdx.x;
  if (tid == 0) cmask_s = 0;
  __syncthreads();
  int cm = 0;
  for (int i = tid; i < COUT * K; i += 256) {
    const int co = i / K;
    if (w[(size_t)co * kpad + (i - co * K)] != 0.f) cm |= 1 << co;
  }
  if (cm) atomicOr(&cmask_s, cm);
  __syncthreads();
  const int cmask = __builtin_amdgcn_readfirstlane(cmask_s);
  if (cmask >> 4) {  // general path
    const int64_t npix = (int64_t)N * H * W;
    // one pixel per thread, each reading whole 256-B records: past gen_blocks blocks the extra
    // waves only thrash L1 / TA (mode-1 grid: 3.5x slower), so the rest of the grid exits
    if ((int)blockIdx.x >= gen_blocks) return;
    for (int64_t pix = (int64_t)blockIdx.x * 256 + tid; pix < npix;
         pix += (int64_t)gen_blocks * 256) {
      const int n = (int)(pix / ((int64_t)H * W));
      const int rem = (int)(pix - (int64_t)n * H * W);
      const int yy = rem / W, xx = rem - (rem / W) * W;
      float acc[COUT];
#pragma unroll
      for (int co = 0; co < COUT; ++co) acc[co] = 0.f;
      for (int t = 0; t < 9; ++t) {
        const int sy = yy + t / 3 - 1, sx = xx + t % 3 - 1;
        if (sy < 0 || sy >= H || sx < 0 || sx >= W) continue;
        const float* gp = g + ((size_t)(n * H + sy) * W + sx) * CIN;
        for (int c4 = 0; c4 < CIN / 4; ++c4) {
          const f32x4 gv = *(const f32x4*)(gp + 4 * c4);
#pragma unroll
          for (int co = 0; co < COUT; ++co) {
            const float* wr = w + (size_t)co * kpad + t * CIN + 4 * c4;  // wave-uniform
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[co] = fmaf(gv[e], wr[e], acc[co]);
          }
        }
      }
      float* yp = y + (size_t)pix * COUT;
#pragma unroll
      for (int co = 0; co < COUT; ++co) yp[co] = ACC ? yp[co] + acc[co] : acc[co];
    }
    return;
  }
  const int q = tid & 15;
  for (int i = tid; i < 9 * 4 * 16 * 4; i += 256) {  // i = ((t·4 + e)·16 + q')·4 + co
    const int co = i & 3, qq = (i >> 2) & 15, te = i >> 6, t = te >> 2, e = te & 3;
    wl[i] = w[(size_t)co * kpad + t * CIN + 4 * qq + e];
  }
  __syncthreads();
  // a 16-lane group walks THIN_STRIP output rows of one 4-pixel column segment with a sliding
  // window of 3 input rows in VGPRs: one new input row (6 pixel records) per output row instead
  // of 3. The 16 groups of a block take 16 adjacent segments of the same strip. Per output
  // pixel the FMAs run in the same order as the segment loop below (bit-identical).
  const int spr = W / 4, nsy = (H + THIN_STRIP - 1) / THIN_STRIP;
  const int64_t nitems = (int64_t)N * nsy * spr;
  auto load_row = [&](int n, int sy, int x0, f32x4 (&dst)[6]) __attribute__((always_inline)) {
    const bool oky = sy >= 0 && sy < H;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const int sx = x0 + c - 1;
      const bool ok = oky && sx >= 0 && sx < W;
      dst[c] = ok ? *(const f32x4*)(g + ((size_t)(n * H + sy) * W + sx) * CIN + 4 * q)
                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // NCO = 3 when output channel 3 is padding too (cmask 0x07, an RGB image): its FMAs are
  // skipped and it stores +0, what the four-channel form computes from zero weights
  auto strip = [&](auto nco_c) __attribute__((always_inline)) {
  constexpr int NCO = decltype(nco_c)::value;
  for (int64_t it = (int64_t)blockIdx.x * 16 + (tid >> 4); it < nitems;
       it += (int64_t)gridDim.x * 16) {
    const int xs = (int)(it % spr);
    const int64_t r = it / spr;
    const int n = (int)(r / nsy), y0 = (int)(r - (int64_t)n * nsy) * THIN_STRIP;
    const int x0 = xs * 4, y1 = min(y0 + THIN_STRIP, H);
    f32x4 win[3][6];
    load_row(n, y0 - 1, x0, win[0]);
    load_row(n, y0, x0, win[1]);
    for (int yy = y0; yy < y1; ++yy) {
      load_row(n, yy + 1, x0, win[2]);
      float acc[4][4];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int co = 0; co < 4; ++co) acc[p][co] = 0.f;
#pragma unroll
      for (int ty = 0; ty < 3; ++ty) {
        const int sy = yy + ty - 1;
        if (sy < 0 || sy >= H) continue;
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) {
          f32x4 wt[4];
          int off = (((3 * ty + tx) * 4) * 16 + q) * 4;
          asm volatile("" : "+v"(off));
#pragma unroll
          for (int e = 0; e < 4; ++e) wt[e] = *(const f32x4*)(wl + off + e * 64);
#pragma unroll
          for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int co = 0; co < NCO; ++co)
                acc[p][co] = fmaf(win[ty][p + tx][e], wt[e][co], acc[p][co]);
        }
      }
      f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int co = 0; co < NCO; ++co) {
          const float sm = row16_sum(acc[p][co]);
          if (q == 2 * p) o[co] = sm;
        }
      if (q < 8) {
        float* yp = y + ((size_t)(n * H + yy) * W + x0 + (q >> 1)) * COUT + 4 * (q & 1);
        if constexpr (ACC) {
          const f32x4 a = *(const f32x4*)yp;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += a[e];
        }
        *(f32x4*)yp = o;
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        win[0][c] = win[1][c];
        win[1][c] = win[2][c];
      }
    }
  }
  };
  if (cmask == 0x07) strip(std::integral_constant<int, 3>{});
  else strip(std::integral_constant<int, 4>{});
}

// 32 → 32 layers: 2-byte type, one group, stride 1, 3×3 pad 1, identity placement, W % 16 == 0,
// an epilogue feature mask with a specialisation (the StyledConv forward and input gradient).
// T_CONV_THIN32 = 0 disables (tests / tuning).
static bool thin32_mask_ok(int f, bool pro) {
  using namespace epi;
  if (pro) return f == (OSC | NOISE | BIAS | LRELU);
  switch (f) {
    case OSC | SDOT: case OSC | SDOT | ACC: case OSC | SDOT | BAB: case OSC | SDOT | ACC | BAB:
    case 0: case ACC:
      return true;
    default:
      return false;
  }
}

bool conv_thin32_eligible(const ConvK& k, int dtype) {
  if (tune(T_CONV_THIN32) == 0) return false;
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  if (dtype == MIA_F32 || k.ng != 1 || k.stride != 1 || G.kh != 3 || G.kw != 3 || G.pad_y != 1 ||
      G.pad_x != 1 || G.ho != a.H || G.wo != a.W || G.ay != 1 || G.ax != 1 || G.by != 0 ||
      G.bx != 0 || a.shuffle_out || a.W % 16 != 0 || k.HT != a.H || k.WT != a.W ||
      k.ystride != a.Cout || a.Cin != 32 || a.Cout != 32 || G.kpad < 9 * 32 || !a.y)
    return false;
  const bool pro = a.in_scale != nullptr;
  if (!pro && a.act_in != MIA_ACT_NONE) return false;
  if (pro && k.cout_mod != a.Cout) return false;
  return thin32_mask_ok(epi_mask(k), pro);
}

template <typename T, bool PRO, int F>
static int launch_thin32_(ConvK& k, int grid, hipStream_t st) {
  // one slot per THIN32_CHUNK-group work item of an image (every slot has its contributor)
  const int64_t gpi = (int64_t)k.a.H * (k.a.W / 16);
  RedQ r;
  int rc = conv_red_begin(k, r, (int)((gpi + THIN32_CHUNK - 1) / THIN32_CHUNK), st, false);
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL((conv_thin32_kernel<T, PRO, F>), dim3(grid), dim3(256), 0, st, k);
  rc = check_launch("conv_thin32");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

int launch_conv_thin32(ConvK& k, int dtype, hipStream_t st) {
  using namespace epi;
  const int64_t groups = (int64_t)k.a.N * k.a.H * (k.a.W / 16);
  const int grid = grid_for(groups, 16);
  const bool pro = k.a.in_scale != nullptr;
  MIA_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      if (pro) return launch_thin32_<T, true, OSC | NOISE | BIAS | LRELU>(k, grid, st);
      switch (epi_mask(k)) {
        case OSC | SDOT: return launch_thin32_<T, false, OSC | SDOT>(k, grid, st);
        case OSC | SDOT | ACC: return launch_thin32_<T, false, OSC | SDOT | ACC>(k, grid, st);
        case OSC | SDOT | BAB: return launch_thin32_<T, false, OSC | SDOT | BAB>(k, grid, st);
        case OSC | SDOT | ACC | BAB:
          return launch_thin32_<T, false, OSC | SDOT | ACC | BAB>(k, grid, st);
        case 0: return launch_thin32_<T, false, 0>(k, grid, st);
        case ACC: return launch_thin32_<T, false, ACC>(k, grid, st);
        default: break;
      }
    }
  });
  return set_error("conv_thin32: no specialisation for this launch");
}

// Eligible launches (checked by run_conv): any dtype (fp32 on the VALU kernels above), one
// group, stride 1, 3×3 pad 1, identity output placement, W % 16 == 0, and either (Cin 8 → Cout
// 64, epilogue = bias + ReLU / PReLU: the VGG and e4e input layers) or (Cin 64 → Cout 8, plain or accumulating: their input gradients).
bool conv_thin_eligible(const ConvK& k, int dtype) {
  if (tune(T_CONV_THIN) == 0) return false;
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  if (k.ng != 1 || k.stride != 1 || G.kh != 3 || G.kw != 3 || G.pad_y != 1 ||
      G.pad_x != 1 || G.ho != a.H || G.wo != a.W || G.ay != 1 || G.ax != 1 || G.by != 0 ||
      G.bx != 0 || a.shuffle_out || a.W % 16 != 0 || k.HT != a.H || k.WT != a.W ||
      k.ystride != a.Cout || a.act_in != MIA_ACT_NONE || a.in_scale || a.out_scale || a.noise ||
      a.tap_a || a.mask_a || a.sdot || a.bab_demod || !a.y || a.csum)
    return false;
  if (a.Cin == 8 && a.Cout == 64 && G.kpad >= 96 && !a.accumulate) return true;
  if (a.Cin == 64 && a.Cout == 8 && !a.bias && a.act_out == MIA_ACT_NONE) return true;
  return false;
}

int launch_conv_thin(ConvK& k, int dtype, hipStream_t st) {
  const mia_conv_args& a = k.a;
  const int grid = grid_for((int64_t)a.N * a.H * (a.W / 16));  // ≤ 8 waves per SIMD
  if (dtype == MIA_F32) {  // the fp32 VALU kernels (one pixel per thread / per 16 threads)
    const int64_t npix = (int64_t)a.N * a.H * a.W;
    // the forward at 16 waves per CU (held to 128 VGPRs: 4 per SIMD), the gradient strips at
    // 12 (144 VGPRs); the gradient's general path (real output channels ≥ 4) runs on the first
    // gen_blocks blocks only
    const int grid_out = grid_for(npix / 16, 12);
    const int gen_blocks = std::min(grid_out, grid_for(npix / 16, 8));
    if (a.Cin == 8) {
      hipLaunchKernelGGL(conv_thin_in_f32_kernel, dim3(grid_for(npix / 16, 16)), dim3(256), 0, st,
                         (const float*)a.x, (const float*)k.g[0].w, k.g[0].kpad, a.bias,
                         a.act_out, a.act_slope, (float*)a.y, a.N, a.H, a.W);
    } else if (a.accumulate) {
      hipLaunchKernelGGL(conv_thin_out_f32_kernel<true>, dim3(grid_out), dim3(256), 0, st,
                         (const float*)a.x, (const float*)k.g[0].w, k.g[0].kpad, (float*)a.y,
                         a.N, a.H, a.W, gen_blocks);
    } else {
      hipLaunchKernelGGL(conv_thin_out_f32_kernel<false>, dim3(grid_out), dim3(256), 0, st,
                         (const float*)a.x, (const float*)k.g[0].w, k.g[0].kpad, (float*)a.y,
                         a.N, a.H, a.W, gen_blocks);
    }
    return check_launch("conv_thin_f32");
  }
  MIA_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      if (a.Cin == 8) {
        hipLaunchKernelGGL((conv_thin_in_kernel<T, 64>), dim3(grid), dim3(256), 0, st,
                           (const T*)a.x, (const T*)k.g[0].w, k.g[0].kpad, a.bias, a.act_out,
                           a.act_slope, (T*)a.y, a.N, a.H, a.W);
      } else {
        const int64_t items = (int64_t)a.N * ((a.H + THIN_SR - 1) / THIN_SR) * (a.W / 16);
        const int lds = 4 * THIN_RING * THIN_SLOT;  // 48 KB: 3 blocks per CU
        hipLaunchKernelGGL((conv_thin_out_strip_kernel<T, 8>), dim3(grid_for(items, 12)),
                           dim3(256), lds, st, (const T*)a.x, (const T*)k.g[0].w, k.g[0].kpad,
                           (T*)a.y, a.accumulate, a.N, a.H, a.W);
      }
      return check_launch("conv_thin");
    }
  });
  return set_error("conv_thin: unknown dtype");
}

}  // namespace mia
