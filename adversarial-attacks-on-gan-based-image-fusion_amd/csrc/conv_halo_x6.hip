// fp32 stride-1 3×3 convolution on the bf16 matrix pipe with the operands split ONCE, not per tap.
//
// The fp32 arithmetic of libmiattack (conv_common.h, mfma_chunk<float>) writes each fp32 operand
// as an exact three-term bf16 sum a = hi + mid + lo and keeps the six products of order ≥ 2^-16.
// Done on the fly, the split costs ≈ 22 VALU instructions per 4 values per fragment read, and a
// halo kernel reads every input value 9 × (taps) × 2 (column waves) times: measured 5–8 VALU
// instructions per MFMA, VALU-issue bound at ≈ 150 TFLOP/s. Here:
//   * the weights come pre-split from HBM (layouts.split_f32: per 4-k quad a 16-B [hi×4 | mid×4]
//     record in the fp32 row geometry + an 8-B lo record in a second [Cout][Kpad] bf16 plane);
//   * the input halo of each 32-channel block is split in LDS once, after its DMA lands (modulation
//     act(x)·s of a StyledConv applied before the split), [hi|mid] in place + lo into an L buffer;
//   * the main loop is ds_reads + 3 MFMAs per fragment pair, no split VALU: with a lane's registers
//     laid out (lo, hi, mid), the tuples (hi, mid) and (lo, hi) are register windows and
//       (hi,mid)·(hi,mid) = hh + mm,  (lo,hi)·(hi,mid) = lh + hm,  (hi,mid)·(lo,hi) = hl + mh.
// Tile: 16 × 16 output pixels × 128 channels, 8 waves (4 row waves × 2 column waves, each 4 × 4
// fragments), one block per CU: LDS = 2 raw/[hi|mid] halo buffers (2 × 41 KB) + one lo buffer
// (20 KB) + a 2-stage pre-split weight ring (2 × 24 KB) = 150 KB. DMA roles as conv_halo.hip:
// waves 0–3 stream the weights one K-step ahead, waves 4–7 the next channel block's halo during
// taps 0–3. Per channel block one extra barrier: the lo buffer is rewritten after the last tap of
// the previous block has read it.
// Measured dead end: each wave owning 16 channels × all 256 pixels with its weights loaded from
// L2 straight into VGPRs (no weight ring, no per-K-step barrier, 9 VALU per 96 MFMAs with
// padded [hi|mid] / [lo|hi] planes read as single ds_read_b128 tuples) ran 4–13 % SLOWER than
// this kernel. Phase stamps (csrc/Makefile `stamps`, tools/probe/x6_stamps.py) over the bench
// attack: the chip holds 2.2–2.3 GHz in this kernel; per block 3 % prologue, 3–6 % in-loop splits,
// 2–5 % epilogue, 88 % main loop, and the main loop runs at 72 % of its MFMA-only bound (16 cycles
// per MFMA, two waves per SIMD; 66 % before the taps were unrolled over offset tables): the loop is
// largely issue-bound. Wave 0 of a block spends a third of the loop at the step-end wait +
// barrier, wave 4 2–3 %, whichever DMA role either streams (the older wave wins the issue
// arbitration; the younger one is the long pole of each step).
// Measured neutral or slower for the loop (not kept): both halves' fragment reads up front, a
// fragment-level read/MFMA pipeline with (lo, hi) windows loaded in place (no register copies),
// every wave streaming a share of the weights and of the halo, a 4-stage weight ring (64-channel
// tile), a persistent form, and (round 3) per-stage LDS counters instead of the per-step block
// barrier (B-waves refill a stage once all 8 waves have read it, readers start once its 4 pieces
// landed, barriers only at channel-block ends): step 7564 → 7568 ms, ±3 % per layer.
#include "conv_common.h"
#include "halo_epilogue.h"

namespace mia {

#ifdef MIA_STAMPS
// Diagnostic build only (csrc/Makefile `stamps`, tools/probe/x6_stamps.py): wave 0 of every block
// adds its phase cycles here; nothing in the kernel reads them back and no output depends on them.
// [variant = (BN == 128) + 2·PRO][blocks, cycles, prologue, in-loop splits, epilogue, 100-MHz
// ticks, K-steps, wave 0 (weights) / wave 4 (halo) cycles in the end-of-step wait + barrier, -…]
__device__ unsigned long long g_x6_stamps[4][16];
#endif

// BN_ = 128: 4 row waves × 2 column waves of 4 × 4 fragments; BN_ = 64 (the 64-channel layers):
// 8 row waves of 2 × 4 fragments. TPS_ taps per K-step (round 4, the 64-column tile of the
// unrolled loop: 2): a stage holds the pre-split weights of TPS taps, so a K-step carries the
// 128-column tile's MFMA count (96 per wave) and weight DMA pieces (6 per B-wave) and the per-step
// barrier, wait and DMA issue are paid half as often (9 taps = 5 steps per channel block).
template <int BN_, int TPS_ = 1>
struct HaloX6 {
  static constexpr int PH = 16, PW = 16, NW = 8, NT = 64 * NW;
  static constexpr int WN = BN_ == 128 ? 2 : 1, WM = NW / WN, FM = 16 / WM, FN = 4;
  static constexpr int BM = PH * PW, BN = BN_, BK = 32;  // 32 fp32 channels per K-step
  static constexpr int HSIDE = PW + 2, HROWS = (PH + 2) * HSIDE;  // 324 halo pixels
  static constexpr int HPIECES = (HROWS + 7) / 8;                 // 1-KB pieces of 8 rows
  static constexpr int HBUF = HPIECES * 1024;
  static constexpr int LROWB = 64, LBUF = HROWS * LROWB;          // lo: 32 × bf16 per pixel
  static constexpr int TPS = TPS_, NG = (9 + TPS - 1) / TPS;  // taps per K-step, steps per block
  static constexpr int BHM = BN * ROWB, BL = BN * LROWB, BSTAGE1 = BHM + BL;  // one tap
  static constexpr int BSTAGE = TPS * BSTAGE1;
  static constexpr int BWAVES = 4, HWAVES = 4;
  static constexpr int B_HM_INS = BN / 8 / BWAVES;   // [hi|mid] pieces (8 rows) per B-wave
  static constexpr int B_L_INS = BN / 16 / BWAVES;   // lo pieces (16 rows of 64 B) per B-wave
  static constexpr int H_INS = (HPIECES + HWAVES - 1) / HWAVES;
  static constexpr int HSTEPS = (4 + TPS - 1) / TPS;    // next block's halo issued over taps 0–3
  static constexpr int H_PER_STEP = (H_INS + HSTEPS - 1) / HSTEPS;
  static constexpr int EROWS = 128, ES = BN + 4;      // shared LDS epilogue staging
  static constexpr int LDS = 2 * HBUF + LBUF + 2 * BSTAGE;
  static_assert(WM * FM * 16 == BM && WN * FN * 16 == BN, "");
  static_assert(B_HM_INS * 8 * BWAVES == BN && B_L_INS * 16 * BWAVES == BN, "");
  static_assert(LDS <= 160 * 1024, "");
};

template <int BN_, bool PRO, int EPI, bool EARLY, bool PRIO, bool UNR, int TPS = 1>
__global__ __launch_bounds__(HaloX6<BN_>::NT, 2) void conv_halo_x6_kernel(const ConvK k) {
  static_assert(!UNR || (EARLY && PRIO && EPI != -2), "UNR: the EARLY + PRIO schedule, D[ch][px]");
  static_assert(UNR || TPS == 1, "several taps per K-step: the unrolled loop only");
  typedef HaloX6<BN_, TPS> TL;
  constexpr int NG = TL::NG;
  constexpr int FM = TL::FM, FN = TL::FN, WN = TL::WN, NT = TL::NT, BN = TL::BN, BK = TL::BK;
  constexpr int HSIDE = TL::HSIDE, HROWS = TL::HROWS, HPIECES = TL::HPIECES, HBUF = TL::HBUF;
  constexpr int H_INS = TL::H_INS, HPS = TL::H_PER_STEP, HWAVES = TL::HWAVES;
  constexpr int B_HM_INS = TL::B_HM_INS, B_L_INS = TL::B_L_INS, BSTAGE = TL::BSTAGE;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                  // 2 halo buffers: raw fp32, then [hi|mid] in place
  char* const lbuf = smem + 2 * HBUF;       // lo of the current channel block
  char* const bring = lbuf + TL::LBUF;      // 2 stages of pre-split weights: [hi|mid] rows, lo rows

  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const ConvGroup G = k.g[0];
  const int H = p.H, W = p.W, Cin = p.Cin, Cout = p.Cout, Kpad = G.kpad;
  const int bl = xcd_remap(blockIdx.x, k.nblk);
  const int mt = bl / k.nbn, n0 = (bl % k.nbn) * BN;
  const int ptx = W / TL::PW, pty = H / TL::PH;
  const int x0 = (mt % ptx) * TL::PW;
  const int y0 = ((mt / ptx) % pty) * TL::PH;
  const int n = mt / (ptx * pty);

  const float* __restrict__ X = (const float*)p.x;
  const unsigned* __restrict__ Whm = (const unsigned*)G.w_split;                // [Cout][Kpad]
  const __bf16* __restrict__ Wl = (const __bf16*)(Whm + (size_t)Cout * Kpad);   // [Cout][Kpad]
  const char* zero = (const char*)g_zero16;
  const bool bwave = wid < TL::BWAVES;
  const int hw = wid - TL::BWAVES;
  const int my_pieces = bwave ? 0 : (HPIECES - hw + HWAVES - 1) / HWAVES;
#ifdef MIA_STAMPS
  const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long st_r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long st_pro = 0, st_cv = 0, st_wb = 0;
#endif

  // per-lane DMA sources (byte pointers; nullptr → the zero page)
  constexpr int NSRC = H_INS > B_HM_INS + B_L_INS ? H_INS : B_HM_INS + B_L_INS;
  const char* src[NSRC];
#pragma unroll
  for (int j = 0; j < NSRC; ++j) {
    src[j] = nullptr;
    if (bwave) {
      // register epilogues: weight rows past Cout read row Cout − 1 instead of the zero page (their
      // accumulator rows are never stored or summed), so the per-step DMA address needs no select
      if (j < B_HM_INS) {
        const int row = (wid * B_HM_INS + j) * 8 + (lane >> 3);
        const int c = EPI >= 0 ? min(n0 + row, Cout - 1) : n0 + row;
        if (c < Cout)
          src[j] = (const char*)(Whm + (size_t)c * Kpad + ((lane & 7) ^ fsw(row)) * 4);
      } else if (j < B_HM_INS + B_L_INS) {
        const int row = (wid * B_L_INS + j - B_HM_INS) * 16 + (lane >> 2);
        const int c = EPI >= 0 ? min(n0 + row, Cout - 1) : n0 + row;
        if (c < Cout)
          src[j] = (const char*)(Wl + (size_t)c * Kpad + ((lane & 3) ^ (lsw(row) >> 1)) * 8);
      }
    } else if (j < H_INS) {
      const int hr = (hw + HWAVES * j) * 8 + (lane >> 3);
      const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
      const int y = y0 + hy - 1, x = x0 + hx - 1;
      if (hr < HROWS && y >= 0 && y < H && x >= 0 && x < W)
        src[j] = (const char*)(X + ((size_t)(n * H + y) * W + x) * Cin + ((lane & 7) ^ fsw(hr)) * 4);
    }
  }
  const int ncb = Cin / BK, nk = NG * ncb;

  auto issue_b = [&](int s, int st) {  // B-wave: its weight pieces of K-step s = (cb, taps)
    const int cb = s / NG, tg = s - (s / NG) * NG;
#pragma unroll
    for (int tt = 0; tt < TPS; ++tt) {
      const int t = tg * TPS + tt;
      if (TPS > 1 && t >= 9) break;        // the block's last step holds 9 mod TPS taps
      const int koff = t * Cin + cb * BK;  // k offset (elements) of the tap in a weight row
      char* dst = bring + st * BSTAGE + tt * TL::BSTAGE1;
#pragma unroll
      for (int j = 0; j < B_HM_INS; ++j) {
        const char* a = EPI >= 0 ? src[j] + (size_t)koff * 4
                                 : src[j] ? src[j] + (size_t)koff * 4 : zero;
        __builtin_amdgcn_global_load_lds((gptr_t)a, (lptr_t)(dst + (wid * B_HM_INS + j) * 1024),
                                         16, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < B_L_INS; ++j) {
        const char* a = EPI >= 0                ? src[B_HM_INS + j] + (size_t)koff * 2
                        : src[B_HM_INS + j] ? src[B_HM_INS + j] + (size_t)koff * 2
                                            : zero;
        __builtin_amdgcn_global_load_lds((gptr_t)a,
                                         (lptr_t)(dst + TL::BHM + (wid * B_L_INS + j) * 1024), 16,
                                         0, 0);
      }
    }
  };
  auto issue_h = [&](int cb, int j, int buf) {  // H-wave: its halo piece j of channel block cb
    const char* a = src[j] ? src[j] + (size_t)cb * BK * 4 : zero;
    __builtin_amdgcn_global_load_lds((gptr_t)a,
                                     (lptr_t)(hbuf + buf * HBUF + (hw + HWAVES * j) * 1024), 16,
                                     0, 0);
  };
  // split the landed raw halo of channel block cb (buffer buf) in place + lo into lbuf
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;
  auto convert = [&](int cb, int buf) {
    char* hb = hbuf + buf * HBUF;
    for (int c = tid; c < HROWS * 8; c += NT) {
      const int hr = c >> 3, pc = c & 7, lc = pc ^ fsw(hr);
      f32x4 v = *(const f32x4*)(hb + hr * ROWB + pc * 16);
      if constexpr (PRO) {  // x̃ = act(x)·s, rounded as the on-the-fly path (conv_common.h)
        const float mul = lrelu_in ? SQRT2 : 1.f;
        f32x4 s4 = {1.f, 1.f, 1.f, 1.f};
        if (p.in_scale) s4 = *(const f32x4*)(p.in_scale + (size_t)n * Cin + cb * BK + lc * 4);
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

  // ---- prologue: weights of step 0, halo of channel block 0, its split -----------------------
  if (bwave) {
    issue_b(0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < H_INS; ++j)
      if (j < my_pieces) issue_h(0, j, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  convert(0, 0);
  __syncthreads();
#ifdef MIA_STAMPS
  st_pro = __builtin_amdgcn_s_memtime();
#endif

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fq = lane >> 4;
  if constexpr (UNR) {
    // The taps unrolled: every fragment address is a lane-constant LDS offset chosen at compile
    // time — for the A fragments one per (row shift q = i + dy, column shift dx), computed once
    // here (the swizzle is not linear in the row, so per step it cost ≈ 8 VALU per fragment); the
    // second MFMA half reads channel chunk ^ 4 (byte offset ^ 64, lo ^ 32). Same reads, same
    // MFMAs in the same order as the rolled loop below.
    int oh[FM + 2][3], ol[FM + 2][3];
#pragma unroll
    for (int q = 0; q < FM + 2; ++q)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int hr = (wm * FM + q) * HSIDE + frow + c;
        int vh = hr * ROWB + ((fq ^ fsw(hr)) << 4), vl = hr * TL::LROWB + ((fq ^ lsw(hr)) << 3);
        asm volatile("" : "+v"(vh), "+v"(vl));  // kept in registers, not recomputed per step
        oh[q][c] = vh;
        ol[q][c] = vl;
      }
    int st = 0;
    for (int cb = 0; cb < ncb; ++cb) {
#pragma unroll
      for (int tg = 0; tg < NG; ++tg) {
        const int s = cb * NG + tg;
        // opaque per step: keeps (table ^ half) and (buffer + table) from being hoisted out of
        // the unrolled taps as 54 more live registers
        int hoff = (cb & 1) * HBUF, x1 = 64, x2 = 32;
        asm volatile("" : "+s"(hoff), "+s"(x1), "+s"(x2));
        const char* ha = hbuf + hoff;
        const char* sb0 = bring + st * BSTAGE;
        if (bwave && s + 1 < nk) issue_b(s + 1, st ^ 1);
        if (!bwave && cb + 1 < ncb && tg < (H_INS + HPS - 1) / HPS) {
#pragma unroll
          for (int q = 0; q < HPS; ++q) {
            const int j = tg * HPS + q;
            if (j < H_INS && j < my_pieces) issue_h(cb + 1, j, (cb + 1) & 1);
          }
        }
#pragma unroll
        for (int tt = 0; tt < TPS; ++tt) {
          const int t = tg * TPS + tt;
          if (t >= 9) break;
          const int dy = t / 3, dx = t % 3;
          const char* sb = sb0 + tt * TL::BSTAGE1;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int ch = h * 4 + fq;
            u32x4 ahm[FM], bhm[FN];
            u32x2 al[FM], blo[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
              ahm[i] = *(const u32x4*)(ha + (h ? oh[i + dy][dx] ^ x1 : oh[i + dy][dx]));
              al[i] = *(const u32x2*)(lbuf + (h ? ol[i + dy][dx] ^ x2 : ol[i + dy][dx]));
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              const int row = wn * FN * 16 + 16 * j + frow;
              bhm[j] = *(const u32x4*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
              blo[j] = *(const u32x2*)(sb + TL::BHM + row * TL::LROWB + ((ch ^ lsw(row)) << 3));
            }
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
              for (int j = 0; j < FN; ++j)
                acc[i][j] = mfma_x6(bhm[j], blo[j], ahm[i], al[i], acc[i][j]);  // D[ch][px]
            __builtin_amdgcn_s_setprio(0);
          }
        }
#ifdef MIA_STAMPS
        const unsigned long long w0 = __builtin_amdgcn_s_memtime();
#endif
        if (bwave || tg == NG - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
#ifdef MIA_STAMPS
        st_wb += __builtin_amdgcn_s_memtime() - w0;
#endif
        if (tg == NG - 1 && cb + 1 < ncb) {
#ifdef MIA_STAMPS
          const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
          convert(cb + 1, (cb + 1) & 1);
          __syncthreads();
#ifdef MIA_STAMPS
          st_cv += __builtin_amdgcn_s_memtime() - c0;
#endif
        }
        st ^= 1;
      }
    }
  } else {
  int st = 0, cb = 0, t = 0;
  for (int s = 0; s < nk; ++s) {
    const char* ha = hbuf + (cb & 1) * HBUF;
    const char* sb = bring + st * BSTAGE;
    const int dy = t >= 6 ? 2 : (t >= 3 ? 1 : 0), dx = t - 3 * dy;
    if (bwave && s + 1 < nk) issue_b(s + 1, st ^ 1);
    if constexpr (EARLY) {
      // H-waves: the next block's halo pieces of this tap before the step's LDS reads, so both
      // MFMA halves and their fragment reads form one scheduling region
      if (!bwave && cb + 1 < ncb) {
#pragma unroll
        for (int tt = 0; tt < (H_INS + HPS - 1) / HPS; ++tt) {
          if (t == tt) {
#pragma unroll
            for (int q = 0; q < HPS; ++q) {
              const int j = tt * HPS + q;
              if (j < H_INS && j < my_pieces) issue_h(cb + 1, j, (cb + 1) & 1);
            }
          }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = h * 4 + fq;  // this lane's logical 16-B quad of the K-step (k = 4·ch …)
      u32x4 ahm[FM], bhm[FN];
      u32x2 al[FM], blo[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int hr = (wm * FM + i + dy) * HSIDE + frow + dx;
        ahm[i] = *(const u32x4*)(ha + hr * ROWB + ((ch ^ fsw(hr)) << 4));
        al[i] = *(const u32x2*)(lbuf + hr * TL::LROWB + ((ch ^ lsw(hr)) << 3));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * FN * 16 + 16 * j + frow;
        bhm[j] = *(const u32x4*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
        blo[j] = *(const u32x2*)(sb + TL::BHM + row * TL::LROWB + ((ch ^ lsw(row)) << 3));
      }
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = EPI != -2 ? mfma_x6(bhm[j], blo[j], ahm[i], al[i], acc[i][j])  // D[ch][px]
                                : mfma_x6(ahm[i], al[i], bhm[j], blo[j], acc[i][j]);  // D[px][ch]
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      if (!EARLY && h == 0 && !bwave && cb + 1 < ncb) {
        // H-waves: the next block's halo between the two MFMA halves, HPS pieces per tap 0–3
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tt = 0; tt < (H_INS + HPS - 1) / HPS; ++tt) {
          if (t == tt) {
#pragma unroll
            for (int q = 0; q < HPS; ++q) {
              const int j = tt * HPS + q;
              if (j < H_INS && j < my_pieces) issue_h(cb + 1, j, (cb + 1) & 1);
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // B-wave: step s+1's weights must have landed. H-wave: the next block's halo by the last tap.
#ifdef MIA_STAMPS
    const unsigned long long w0 = __builtin_amdgcn_s_memtime();
#endif
    if (bwave || t == 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS reads of the step are done
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#ifdef MIA_STAMPS
    st_wb += __builtin_amdgcn_s_memtime() - w0;
#endif
    if (t == 8 && cb + 1 < ncb) {  // every wave is past the last read of lbuf: split block cb+1
#ifdef MIA_STAMPS
      const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
      convert(cb + 1, (cb + 1) & 1);
      __syncthreads();
#ifdef MIA_STAMPS
      st_cv += __builtin_amdgcn_s_memtime() - c0;
#endif
    }
    st ^= 1;
    if (++t == 9) { t = 0; ++cb; }
  }
  }  // !UNR
#ifdef MIA_STAMPS
  const unsigned long long st_loop = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (EPI >= 0) {
    halo_epilogue_f<float, TL, EPI>(k, acc, n, y0, x0, n0, wm, wn, lane, -1, -1, nullptr,
                                    k.prered ? (float*)smem : nullptr, TL::WM, TL::BN);
  } else if constexpr (EPI == -1) {
    halo_epilogue<float, TL>(k, acc, n, y0, x0, n0, wm, wn, lane);
  } else {
    __syncthreads();
    const int img_row = n * H + y0;
    conv_epilogue<float, TL>(k, G, acc, smem, n0, true, n, [=](int r) {
      return (img_row + (r >> 4)) * W + x0 + (r & 15);
    }, (y0 / TL::PH) * (W / TL::PW) + x0 / TL::PW);  // the patch's reduction slot
  }
#ifdef MIA_STAMPS
  if (wid == 0 && lane == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* g = g_x6_stamps[(BN_ == 128 ? 1 : 0) + (PRO ? 2 : 0)];
    atomicAdd(g + 0, 1ull);
    atomicAdd(g + 1, t1 - st_t0);
    atomicAdd(g + 2, st_pro - st_t0);
    atomicAdd(g + 3, st_cv);
    atomicAdd(g + 4, t1 - st_loop);
    atomicAdd(g + 5, r1 - st_r0);
    atomicAdd(g + 6, (unsigned long long)nk);
    atomicAdd(g + 7, st_wb);
  }
  if (wid == 4 && lane == 0) atomicAdd(&g_x6_stamps[(BN_ == 128 ? 1 : 0) + (PRO ? 2 : 0)][8], st_wb);
#endif
}

template <int BN_, bool PRO, int EPI, bool EARLY, bool PRIO = false, bool UNR = false,
          int TPS = 1>
static int launch_x6_e(ConvK& k, hipStream_t st) {
  typedef HaloX6<BN_, TPS> TL;
  k.nbn = (k.a.Cout + TL::BN - 1) / TL::BN;
  k.nblk = k.a.N * (k.a.H / TL::PH) * (k.a.W / TL::PW) * k.nbn;
  size_t lds = TL::LDS;
  lds = std::max(lds, (size_t)TL::EROWS * TL::ES * 4);
  lds = std::max(lds, (size_t)TL::NW * TL::BN * 4);
  auto fn = conv_halo_x6_kernel<BN_, PRO, EPI, EARLY, PRIO, UNR, TPS>;
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
  rc = check_launch("conv_halo_x6");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

template <int BN_, bool PRO, int EPI>
static int launch_x6_(ConvK& k, hipStream_t st) {
  // the next block's halo DMA at the step start (measured +2-3 % on the stride-1 layers over
  // issuing it between the two MFMA halves) + s_setprio(1) around each MFMA block (+1-4 %): the
  // wave in its MFMA phase keeps issue priority over the co-resident wave's LDS reads
  if constexpr (EPI >= 0) {  // + the taps unrolled with lane-constant fragment offsets
    // T_X6_UNR = 2 (default): the 64-column tile takes two taps per K-step (HaloX6 TPS)
    const int u = tune(T_X6_UNR);
    if constexpr (BN_ == 64) {
      if (u == 2) return launch_x6_e<BN_, PRO, EPI, true, true, true, 2>(k, st);
    }
    if (u != 0) return launch_x6_e<BN_, PRO, EPI, true, true, true>(k, st);
  }
  return launch_x6_e<BN_, PRO, EPI, true, true>(k, st);  // the rolled loop (T_X6_UNR = 0)
}

// ---- the 64-channel layers, two blocks per CU (round 4) ---------------------------------------
// The 64-column tile above runs one 8-wave block per CU: its 18-step K loop (Cin = 64) leaves the
// prologue (first halo from HBM + split, 15 % of a block), the epilogue (7 %) and every per-step
// barrier exposed — the two waves of a SIMD belong to the same block and stall together (stamps:
// loop at 64 % of its MFMA-only bound). Here a block is an 8 × 16 patch × 64 channels on 4 waves
// (4 row waves of 2 × 4 fragments, the same wave tile), LDS = ONE halo buffer (raw, split in place)
// + lo + a 2-stage pre-split weight ring = 58 KB, so two blocks share a CU and each one's halo
// waits, splits, barriers and epilogue run under the other's MFMAs (the 2-byte halo kernel's
// 8 × 16 / 2-blocks-per-CU arrangement). Every wave streams a share of the weights (3 pieces per
// K-step); the next channel block's halo is fetched by all waves after the last tap of the current
// one (single buffer). Same MFMAs in the same order per output as the 8-wave tile (bit-identical).
struct HaloX6S {
  static constexpr int PH = 8, PW = 16, NW = 4, NT = 64 * NW;
  static constexpr int WN = 1, WM = 4, FM = 2, FN = 4;
  static constexpr int BM = PH * PW, BN = 64, BK = 32;
  static constexpr int HSIDE = PW + 2, HROWS = (PH + 2) * HSIDE;  // 180 halo pixels
  static constexpr int HPIECES = (HROWS + 7) / 8;                 // 23 pieces of 8 rows
  static constexpr int HBUF = HPIECES * 1024;
  static constexpr int LROWB = 64, LBUF = HROWS * LROWB;
  static constexpr int BHM = BN * ROWB, BL = BN * LROWB, BSTAGE = BHM + BL;  // 12 KB
  static constexpr int B_HM_INS = BN / 8 / NW, B_L_INS = BN / 16 / NW;      // 2 + 1 per wave
  static constexpr int H_INS = (HPIECES + NW - 1) / NW;                      // 6
  static constexpr int EROWS = 128, ES = BN + 4;
  static constexpr int LDS = HBUF + LBUF + 2 * BSTAGE;
  static_assert(WM * FM * 16 == BM && WN * FN * 16 == BN, "");
  static_assert(B_HM_INS * 8 * NW == BN && B_L_INS * 16 * NW == BN, "");
  static_assert(LDS <= 80 * 1024, "two blocks per CU");
};

template <bool PRO, int EPI>
__global__ __launch_bounds__(HaloX6S::NT, 2) void conv_halo_x6s_kernel(const ConvK k) {
  static_assert(EPI >= 0, "the specialised register epilogues only");
  typedef HaloX6S TL;
  constexpr int FM = TL::FM, FN = TL::FN, NT = TL::NT, BN = TL::BN, BK = TL::BK;
  constexpr int HSIDE = TL::HSIDE, HROWS = TL::HROWS, HPIECES = TL::HPIECES;
  constexpr int H_INS = TL::H_INS, B_HM_INS = TL::B_HM_INS, B_L_INS = TL::B_L_INS;
  constexpr int BSTAGE = TL::BSTAGE;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const hbuf = smem;                 // the halo: raw fp32, then [hi|mid] in place
  char* const lbuf = smem + TL::HBUF;      // lo of the current channel block
  char* const bring = lbuf + TL::LBUF;     // 2 stages of pre-split weights

  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid, wn = 0;
  const ConvGroup G = k.g[0];
  const int H = p.H, W = p.W, Cin = p.Cin, Cout = p.Cout, Kpad = G.kpad;
  const int bl = xcd_remap(blockIdx.x, k.nblk);
  const int mt = bl / k.nbn, n0 = (bl % k.nbn) * BN;
  const int ptx = W / TL::PW, pty = H / TL::PH;
  const int x0 = (mt % ptx) * TL::PW;
  const int y0 = ((mt / ptx) % pty) * TL::PH;
  const int n = mt / (ptx * pty);

  const float* __restrict__ X = (const float*)p.x;
  const unsigned* __restrict__ Whm = (const unsigned*)G.w_split;               // [Cout][Kpad]
  const __bf16* __restrict__ Wl = (const __bf16*)(Whm + (size_t)Cout * Kpad);  // [Cout][Kpad]
  const char* zero = (const char*)g_zero16;

  // per-lane DMA sources: weight pieces (every wave) and halo pieces (every wave), byte pointers
  const char* wsrc[B_HM_INS + B_L_INS];
#pragma unroll
  for (int j = 0; j < B_HM_INS + B_L_INS; ++j) {
    // weight rows past Cout read row Cout − 1 (never stored or summed: register epilogues)
    if (j < B_HM_INS) {
      const int row = (wid * B_HM_INS + j) * 8 + (lane >> 3);
      const int c = min(n0 + row, Cout - 1);
      wsrc[j] = (const char*)(Whm + (size_t)c * Kpad + ((lane & 7) ^ fsw(row)) * 4);
    } else {
      const int row = (wid * B_L_INS + j - B_HM_INS) * 16 + (lane >> 2);
      const int c = min(n0 + row, Cout - 1);
      wsrc[j] = (const char*)(Wl + (size_t)c * Kpad + ((lane & 3) ^ (lsw(row) >> 1)) * 8);
    }
  }
  const char* hsrc[H_INS];
#pragma unroll
  for (int j = 0; j < H_INS; ++j) {
    hsrc[j] = nullptr;
    const int hr = (wid + TL::NW * j) * 8 + (lane >> 3);
    const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
    const int y = y0 + hy - 1, x = x0 + hx - 1;
    if (hr < HROWS && y >= 0 && y < H && x >= 0 && x < W)
      hsrc[j] = (const char*)(X + ((size_t)(n * H + y) * W + x) * Cin + ((lane & 7) ^ fsw(hr)) * 4);
  }
  const int ncb = Cin / BK, nk = 9 * ncb;

  auto issue_b = [&](int s, int st) {  // this wave's weight pieces of K-step s = (cb, tap)
    const int cb = s / 9, t = s - (s / 9) * 9;
    const size_t koff = (size_t)t * Cin + cb * BK;
    char* dst = bring + st * BSTAGE;
#pragma unroll
    for (int j = 0; j < B_HM_INS; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(wsrc[j] + koff * 4),
                                       (lptr_t)(dst + (wid * B_HM_INS + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < B_L_INS; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(wsrc[B_HM_INS + j] + koff * 2),
                                       (lptr_t)(dst + TL::BHM + (wid * B_L_INS + j) * 1024), 16,
                                       0, 0);
  };
  auto issue_halo = [&](int cb) {  // this wave's halo pieces of channel block cb
#pragma unroll
    for (int j = 0; j < H_INS; ++j) {
      if (wid + TL::NW * j >= HPIECES) break;
      const char* a = hsrc[j] ? hsrc[j] + (size_t)cb * BK * 4 : zero;
      __builtin_amdgcn_global_load_lds((gptr_t)a, (lptr_t)(hbuf + (wid + TL::NW * j) * 1024), 16,
                                       0, 0);
    }
  };
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;
  auto convert = [&](int cb) {  // split the landed raw halo in place + lo into lbuf
    for (int c = tid; c < HROWS * 8; c += NT) {
      const int hr = c >> 3, pc = c & 7, lc = pc ^ fsw(hr);
      f32x4 v = *(const f32x4*)(hbuf + hr * ROWB + pc * 16);
      if constexpr (PRO) {  // x̃ = act(x)·s, rounded as the on-the-fly path (conv_common.h)
        const float mul = lrelu_in ? SQRT2 : 1.f;
        f32x4 s4 = {1.f, 1.f, 1.f, 1.f};
        if (p.in_scale) s4 = *(const f32x4*)(p.in_scale + (size_t)n * Cin + cb * BK + lc * 4);
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

  // prologue: halo of channel block 0 and the weights of step 0, then the split
  issue_halo(0);
  issue_b(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  convert(0);
  __syncthreads();

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the taps unrolled over lane-constant fragment offsets (as the 8-wave kernel's UNR loop)
  const int frow = lane & 15, fq = lane >> 4;
  int oh[FM + 2][3], ol[FM + 2][3];
#pragma unroll
  for (int q = 0; q < FM + 2; ++q)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int hr = (wm * FM + q) * HSIDE + frow + c;
      int vh = hr * ROWB + ((fq ^ fsw(hr)) << 4), vl = hr * TL::LROWB + ((fq ^ lsw(hr)) << 3);
      asm volatile("" : "+v"(vh), "+v"(vl));
      oh[q][c] = vh;
      ol[q][c] = vl;
    }
  int st = 0;
  for (int cb = 0; cb < ncb; ++cb) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int s = cb * 9 + t;
      int x1 = 64, x2 = 32;
      asm volatile("" : "+s"(x1), "+s"(x2));
      const int dy = t / 3, dx = t % 3;
      const char* sb = bring + st * BSTAGE;
      if (s + 1 < nk) issue_b(s + 1, st ^ 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = h * 4 + fq;
        u32x4 ahm[FM], bhm[FN];
        u32x2 al[FM], blo[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          ahm[i] = *(const u32x4*)(hbuf + (h ? oh[i + dy][dx] ^ x1 : oh[i + dy][dx]));
          al[i] = *(const u32x2*)(lbuf + (h ? ol[i + dy][dx] ^ x2 : ol[i + dy][dx]));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = 16 * j + frow;
          bhm[j] = *(const u32x4*)(sb + row * ROWB + ((ch ^ fsw(row)) << 4));
          blo[j] = *(const u32x2*)(sb + TL::BHM + row * TL::LROWB + ((ch ^ lsw(row)) << 3));
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = mfma_x6(bhm[j], blo[j], ahm[i], al[i], acc[i][j]);  // D[ch][px]
        __builtin_amdgcn_s_setprio(0);
      }
      // the next step's weights landed (this wave's pieces; the barrier covers the others')
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_handoff();
      __builtin_amdgcn_sched_barrier(0);
      st ^= 1;
    }
    if (cb + 1 < ncb) {  // every wave is past its last read of the halo and lo: next block
      issue_halo(cb + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      convert(cb + 1);
      __syncthreads();
    }
  }
  halo_epilogue_f<float, TL, EPI>(k, acc, n, y0, x0, n0, wm, wn, lane, -1, -1, nullptr,
                                  k.prered ? (float*)smem : nullptr, TL::WM, TL::BN);
}

template <bool PRO, int EPI>
static int launch_x6s_(ConvK& k, hipStream_t st) {
  typedef HaloX6S TL;
  k.nbn = (k.a.Cout + TL::BN - 1) / TL::BN;
  k.nblk = k.a.N * (k.a.H / TL::PH) * (k.a.W / TL::PW) * k.nbn;
  size_t lds = TL::LDS;
  lds = std::max(lds, (size_t)TL::EROWS * TL::ES * 4);
  lds = std::max(lds, (size_t)TL::NW * TL::BN * 4);
  auto fn = conv_halo_x6s_kernel<PRO, EPI>;
  if (const int rc = ensure_dyn_lds((const void*)fn, 80 * 1024); rc != MIA_OK) return rc;
  k.prered = (EPI & epi::CSUM);
  const int nslots = halo_red_slots(k.a.H, k.a.W, TL::FM, TL::WM, k.prered);
  RedQ r;
  int rc = conv_red_begin(k, r, nslots, st);
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(k.nblk), dim3(TL::NT), lds, st, k);
  rc = check_launch("conv_halo_x6s");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

// T_X6_64S = 1 (default): the Cout = 64 launches with a specialised epilogue on the two-blocks-
// per-CU tile; returns X6S_NONE (not handled) for any other feature mask
constexpr int X6S_NONE = 1;  // not an MIA_* status (those are ≤ 0)
static int launch_x6s(ConvK& k, hipStream_t st, bool pro) {
  using namespace epi;
  const int f = epi_mask(k);
  if (pro) {
    if (f == (OSC | NOISE | BIAS | LRELU)) return launch_x6s_<true, OSC | NOISE | BIAS | LRELU>(k, st);
    return X6S_NONE;
  }
  switch (f) {
    case 0: return launch_x6s_<false, 0>(k, st);
    case BIAS: return launch_x6s_<false, BIAS>(k, st);
    case BIAS | RELU: return launch_x6s_<false, BIAS | RELU>(k, st);
    case PRELU: return launch_x6s_<false, PRELU>(k, st);
    case MASK: return launch_x6s_<false, MASK>(k, st);
    case TAP: return launch_x6s_<false, TAP>(k, st);
    case TAP | MASK: return launch_x6s_<false, TAP | MASK>(k, st);
    case ACC: return launch_x6s_<false, ACC>(k, st);
    case MASK | MSL: return launch_x6s_<false, MASK | MSL>(k, st);
    default: return X6S_NONE;
  }
}

// The register epilogue specialised for the feature masks of the attack's fp32 launches (every aux
// load of a row chunk hoisted, compile-time features; halo_epilogue.h): the runtime-generic one
// issues its per-row loads one dependent round trip at a time, ≈ 10 % of a block's cycles
// (tools/probe/x6_stamps.py). Any other mask runs the generic epilogue.
template <int BN_, bool PRO>
static int launch_x6_spec(ConvK& k, hipStream_t st) {
  using namespace epi;
  const int f = epi_mask(k);
  if constexpr (PRO) {  // modulated input: the StyledConv forward
    if (f == (OSC | NOISE | BIAS | LRELU))
      return launch_x6_<BN_, PRO, OSC | NOISE | BIAS | LRELU>(k, st);
  } else if constexpr (BN_ == 64) {  // the 64-column tile: launches without per-pixel aux operands
    switch (f) {
      case 0: return launch_x6_<BN_, PRO, 0>(k, st);
      case BIAS: return launch_x6_<BN_, PRO, BIAS>(k, st);            // e4e conv2 (SE body)
      case BIAS | RELU: return launch_x6_<BN_, PRO, BIAS | RELU>(k, st);  // VGG forward
      case PRELU: return launch_x6_<BN_, PRO, PRELU>(k, st);          // e4e conv1
      // per-pixel aux operands (the tap pair: MIA_X6_64S=0, A/B and bitwise tests only)
      case MASK: return launch_x6_<BN_, PRO, MASK>(k, st);
      case TAP: return launch_x6_<BN_, PRO, TAP>(k, st);
      case ACC: return launch_x6_<BN_, PRO, ACC>(k, st);
      case MASK | MSL: return launch_x6_<BN_, PRO, MASK | MSL>(k, st);
      default: break;
    }
  } else {
    switch (f) {
      case 0: return launch_x6_<BN_, PRO, 0>(k, st);
      case BIAS: return launch_x6_<BN_, PRO, BIAS>(k, st);
      case BIAS | RELU: return launch_x6_<BN_, PRO, BIAS | RELU>(k, st);
      case PRELU: return launch_x6_<BN_, PRO, PRELU>(k, st);
      case MASK: return launch_x6_<BN_, PRO, MASK>(k, st);            // VGG input gradient
      case TAP: return launch_x6_<BN_, PRO, TAP>(k, st);              // VGG gradient at a tap
      case ACC: return launch_x6_<BN_, PRO, ACC>(k, st);              // e4e residual gradient
      case MASK | MSL: return launch_x6_<BN_, PRO, MASK | MSL>(k, st);  // e4e PReLU gradient
      case OSC | SDOT: return launch_x6_<BN_, PRO, OSC | SDOT>(k, st);  // StyledConv dgrad
      case OSC | SDOT | BAB: return launch_x6_<BN_, PRO, OSC | SDOT | BAB>(k, st);
      default: break;
    }
  }
  return launch_x6_<BN_, PRO, -1>(k, st);
}

// Eligible: fp32 with pre-split weights (mia_conv_args.w_split / mia_conv_group.w_split), one
// group, stride 1, 3×3 pad 1, identity placement, 16-divisible maps, Cin % 32 == 0, Cout ≥ 64.
bool conv_halo_x6_eligible(const ConvK& k, int dtype) {
#ifdef MIA_F32_NATIVE
  (void)k;
  (void)dtype;
  return false;  // the native-fp32 A/B build keeps every fp32 conv on v_mfma_f32_16x16x4_f32
#endif
  if (tune(T_CONV_X6) == 0) return false;  // the on-the-fly split kernels
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  return dtype == MIA_F32 && G.w_split != nullptr && k.ng == 1 && k.stride == 1 && G.kh == 3 &&
         G.kw == 3 && G.pad_y == 1 && G.pad_x == 1 && G.ho == a.H && G.wo == a.W && G.ay == 1 &&
         G.ax == 1 && G.by == 0 && G.bx == 0 && !a.shuffle_out && a.H % 16 == 0 &&
         a.W % 16 == 0 && a.Cin % 32 == 0 && k.HT == a.H && k.WT == a.W &&
         // 64 channels: the two-blocks-per-CU x6s tile (T_X6_64S = 1, default; with the tap pair
         // too), or the 8-wave 64-column tile (0, A/B)
         a.Cout >= 64;
}

#ifdef MIA_STAMPS
extern "C" int mia_debug_x6_stamps(unsigned long long* host, int reset) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_x6_stamps), sizeof(g_x6_stamps)) != hipSuccess)
    return 1;
  if (reset) {
    static const unsigned long long zero[4][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_x6_stamps), zero, sizeof(zero)) != hipSuccess) return 1;
  }
  return 0;
}
#endif

int launch_conv_halo_x6(ConvK& k, hipStream_t st) {
  const bool pro = k.a.in_scale != nullptr || k.a.act_in != MIA_ACT_NONE;
#ifdef MIA_STAMPS
  {  // each distinct (Cout tile, prologue, epilogue feature mask) once
    static int seen[64];
    static int nseen = 0;
    const int key = (epi_mask(k) << 2) | (pro ? 2 : 0) | (k.a.Cout == 64 ? 1 : 0);
    bool found = false;
    for (int i = 0; i < nseen; ++i) found |= seen[i] == key;
    if (!found && nseen < 64) {
      seen[nseen++] = key;
      fprintf(stderr, "x6 launch: Cout %d pro %d epi_mask %d (%dx%d Cin %d)\n", k.a.Cout, pro,
              epi_mask(k), k.a.H, k.a.W, k.a.Cin);
    }
  }
#endif
  const int sel = tune(T_HALO_EPI);  // 0 LDS-staged epilogue, 2 runtime; default 1 specialised
  if (k.a.Cout == 64 && sel == 1 && tune(T_X6_64S) != 0 && k.a.H % HaloX6S::PH == 0) {
    const int rc = launch_x6s(k, st, pro);
    if (rc != X6S_NONE) return rc;
  }
  if (k.a.Cout == 64) {
    if (sel == 0) return pro ? launch_x6_<64, true, -2>(k, st) : launch_x6_<64, false, -2>(k, st);
    if (sel == 1) return pro ? launch_x6_spec<64, true>(k, st) : launch_x6_spec<64, false>(k, st);
    return pro ? launch_x6_<64, true, -1>(k, st) : launch_x6_<64, false, -1>(k, st);
  }
  if (sel == 0) return pro ? launch_x6_<128, true, -2>(k, st) : launch_x6_<128, false, -2>(k, st);
  if (sel == 1) return pro ? launch_x6_spec<128, true>(k, st) : launch_x6_spec<128, false>(k, st);
  return pro ? launch_x6_<128, true, -1>(k, st) : launch_x6_<128, false, -1>(k, st);
}

}  // namespace mia
