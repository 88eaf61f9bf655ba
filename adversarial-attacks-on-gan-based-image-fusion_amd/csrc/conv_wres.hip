// Weights-resident persistent 3×3 conv for the 64 → 64-channel layers (NHWC, fp16/bf16, CDNA4).
//
// Serves VGG conv1_2 forward and input gradient (code/vgg.py:45-62, 256²) and the e4e encoder's
// first IR-SE50 stage (Encoder4Editing body units 0-2 conv1/conv2 and their input gradients,
// 256² / 128²; un-vendored, code/utils/model_utils.py:24). At Cout = 64 the tiled kernels pay the
// per-K-step weight staging and barrier for half the MFMAs of a 128-channel tile (measured 375-
// 440 TFLOP/s); here the weights (K = 9·64 = 576) are loaded ONCE per wave into VGPRs as MFMA B
// fragments and the block is persistent over a contiguous run of 16×16-pixel output patches:
//   * 8 waves, two per SIMD: wave (wm, wn) owns patch rows 4·wm … 4·wm+3 (one 16-pixel MFMA
//     fragment per row) × output channels 32·wn … 32·wn+31, and holds only those channels'
//     weights (144 VGPRs). One wave's epilogue, DMA issue and LDS waits run under its partner's
//     MFMAs (round 5: the first form, 4 waves × all 64 channels with 288 weight VGPRs and one
//     wave per SIMD, ran 13–18 % slower per layer and is gone);
//   * per patch the (16+2)×(16+2) input halo (one 64-channel block, 41 KB) is DMA'd into one of
//     two LDS buffers a full patch ahead (global_load_lds, bank swizzle fsw() through the source
//     chunk, zero page for the padding);
//   * the main loop is 9 taps × 2 K-chunks of ds_read_b128 A fragments and 8 MFMAs each, with
//     no barrier and no weight traffic;
//   * one barrier per patch (all waves finished the previous patch and waited for their DMA
//     pieces) before the next halo is issued into the buffer just released; each wave drains its
//     DMA (vmcnt(0)) AFTER its MFMAs and BEFORE its epilogue stores, so the wait never covers
//     stores and the DMA had a whole patch to land;
//   * the epilogue is halo_epilogue_f (registers, 16-byte stores); a single per-pixel operand
//     (mask or old y) of the wave's pixels and channels is DMA'd into LDS at the start of the
//     patch (WresAux) and lands during the MFMAs instead of stalling the epilogue.
#include "conv_common.h"
#include "halo_epilogue.h"

namespace mia {

template <int NW_, int WN_>
struct WresTileT {
  // NW waves; WN channel halves: wave (wm, wn) owns patch rows wm·FM … +FM−1 × output channels
  // 16·FN·wn … +16·FN−1, and holds only those channels' weights (FN = 4 / WN fragments)
  static constexpr int NW = NW_, WN = WN_, WM = NW / WN, FM = 16 / WM, FN = 4 / WN, NT = 64 * NW;
  static constexpr int PH = 16, PW = 16, HSIDE = PW + 2, HROWS = (PH + 2) * HSIDE;  // 324
  static constexpr int HPIECES = (HROWS + 7) / 8;                                    // 41
  static constexpr int HBUF = HPIECES * 8 * ROWB;
  static constexpr int H_INS = (HPIECES + NW - 1) / NW;
  static constexpr int CPP = 2 * FN;            // 16-B chunks per pixel of a wave's channels
  static constexpr int AUXW = FM * 16 * CPP * 16;  // one per-pixel epilogue operand of a wave
  static_assert(WM * FM == PH && WN * FN == 4, "");
};
// two waves per SIMD, each 32 channels (144 weight VGPRs)
typedef WresTileT<8, 2> WresTile;

// Per-pixel epilogue operands prefetched into LDS (a wave's 64 pixels × its 32 channels): MASK →
// mask_a, ACC → old y, TAP | MASK → the tap pair (tap_a, also the ReLU mask, and tap_t). LDS-DMA
// costs no registers (a register prefetch spilled next to the resident weights).
template <int EPI>
struct WresAux {
  static constexpr bool TAP = EPI & epi::TAP, MASK = (EPI & epi::MASK) && !TAP;
  static constexpr bool ACC = EPI & epi::ACC;
  // TAP: the tap pair (tap_a, which is also the mask: conv_wres_eligible, and tap_t)
  static constexpr int N = TAP ? 2 : (MASK ? 1 : 0) + (ACC ? 1 : 0);
  static_assert(N <= 2 && (TAP || N <= 1), "prefetched operands per wave");
  static_assert(!(EPI & (epi::SDOT | epi::BAB | epi::NOISE)), "not a weights-resident epilogue");
};

// bank swizzle of the prefetched operand rows (16-B chunk c of pixel q stored at c ^ asw(q)): a
// ds_read_b64 of 16 pixels × one channel quad pair hits 16 distinct (pixel parity, chunk) slots.
// FN = 2 (64-B rows): chunk c ^ ((q >> 2) & 3), 16 pixels × 2 halves on 64 distinct dwords.
template <int FN>
__device__ __forceinline__ int asw(int q) { return FN == 4 ? (q >> 1) & 7 : (q >> 2) & 3; }

// EPI: the epilogue feature mask (halo_epilogue.h, specialised only; see wres_mask_ok); wave wm
// owns rows wm·FM …, wn = 0, n0 = 0
template <typename T, typename TL, int EPI>
__global__ __launch_bounds__(TL::NT, 1) void conv_wres_kernel(const ConvK k) {
  typedef typename Vec<T>::type VT;
  constexpr int FM = TL::FM, FN = TL::FN, HSIDE = TL::HSIDE, HROWS = TL::HROWS;
  constexpr int HPIECES = TL::HPIECES, HBUF = TL::HBUF, H_INS = TL::H_INS, NW = TL::NW;
  constexpr int WM = TL::WM, CPP = TL::CPP;
  constexpr int VEC = 8;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef WresAux<EPI> AUX;
  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid % WM, wn = wid / WM;
  const int frow = lane & 15, fq = lane >> 4;
  const int H = p.H, W = p.W;
  const int ptx = W / TL::PW, pty = H / TL::PH;
  const int ntiles = p.N * ptx * pty;
  const T* __restrict__ X = (const T*)p.x;
  const T* __restrict__ Wt = (const T*)k.g[0].w;
  const int kpad = k.g[0].kpad;
  const T* zero = (const T*)g_zero16;

  // weights → VGPRs: B fragment (tap t, K-chunk h, channel fragment j) = 8 input channels
  // (h·4 + fq)·8 … of output channel 16·(FN·wn + j) + frow
  VT wreg[9][2][FN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        wreg[t][h][j] = *(const VT*)(Wt + (size_t)(16 * (FN * wn + j) + frow) * kpad + t * 64 +
                                     (h * 4 + fq) * VEC);

  auto tile_pos = [&](int tile, int& n, int& y0, int& x0) {
    x0 = (tile % ptx) * TL::PW;
    y0 = ((tile / ptx) % pty) * TL::PH;
    n = tile / (ptx * pty);
  };
  // wave wid DMAs halo pieces wid + NW·j (8 halo pixels = 1 KB each)
  auto issue_halo = [&](int tile, int buf) {
    int n, y0, x0;
    tile_pos(tile, n, y0, x0);
    // opaque copy of the lane id: the per-piece halo coordinates are recomputed per patch
    // instead of being hoisted out of the patch loop (they would spill next to the resident
    // weights, and every spill reload waits vmcnt(0) on the DMA just issued)
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int j = 0; j < H_INS; ++j) {
      const int piece = wid + NW * j;
      if (piece < HPIECES) {
        const int hr = piece * 8 + (ln >> 3);
        const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
        const int y = y0 + hy - 1, x = x0 + hx - 1;
        const T* src = zero;
        if (hr < HROWS && y >= 0 && y < H && x >= 0 && x < W)
          src = X + ((size_t)(n * H + y) * W + x) * 64 + ((ln & 7) ^ fsw(hr)) * VEC;
        __builtin_amdgcn_global_load_lds((gptr_t)src,
                                         (lptr_t)(smem + buf * HBUF + piece * 1024), 16, 0, 0);
      }
    }
  };

  // wave wid DMAs the epilogue operands of its FM output rows × its channels (1 KB pieces of
  // 64 / CPP pixels)
  char* const auxw = smem + 2 * HBUF + wid * (AUX::N * TL::AUXW);  // this wave's operand slots
  // sdot / q / csum pre-reduction of the WM wave rows (each covers its channels of its rows)
  float* const red = k.prered ? (float*)(smem + 2 * HBUF + NW * AUX::N * TL::AUXW) : nullptr;
  auto issue_aux = [&](int n, int y0, int x0) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const T* srcs[2] = {AUX::TAP ? (const T*)p.tap_a : (AUX::MASK ? (const T*)p.mask_a : (const T*)p.y),
                        (const T*)p.tap_t};
#pragma unroll
    for (int t = 0; t < AUX::N; ++t)
#pragma unroll
      for (int j = 0; j < FM * CPP / 4; ++j) {
        const int q = j * (64 / CPP) + ln / CPP;  // wave-local pixel: row q / 16, column q % 16
        const int y = y0 + wm * FM + (q >> 4), x = x0 + (q & 15);
        const T* src = srcs[t] + ((size_t)(n * H + y) * W + x) * 64 + 16 * FN * wn +
                       ((ln % CPP) ^ asw<FN>(q)) * VEC;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(auxw + t * TL::AUXW + j * 1024),
                                         16, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // one address live at a time (weights fill the VGPRs)
      }
  };

  // a contiguous run of patches per block (neighbouring halos overlap: L2 hits on its XCD)
  const int per = (ntiles + gridDim.x - 1) / gridDim.x;
  const int t_end = min((int)blockIdx.x * per + per, ntiles);
  const int t_step = 1;
  int tile = blockIdx.x * per;
  if (tile < t_end) issue_halo(tile, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int buf = 0;
  for (; tile < t_end; tile += t_step) {
    // every wave finished the previous patch (buffer buf^1 is free) and drained its DMA pieces
    // of this patch (buffer buf is complete)
    __syncthreads();
    const int next = tile + t_step;
    int n, y0, x0;
    tile_pos(tile, n, y0, x0);
    if constexpr (AUX::N > 0) issue_aux(n, y0, x0);  // land during this patch's MFMAs
    if (next < t_end) issue_halo(next, buf ^ 1);
    const char* ha = smem + buf * HBUF;
    // opaque pixel-row lane index: the 36 swizzled A-fragment addresses (lane-dependent XOR, no
    // immediate-offset form) are recomputed inside the patch, not held across it
    int fr = frow;
    asm volatile("" : "+v"(fr));
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3, dx = t - 3 * (t / 3);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = h * 4 + fq;
        VT af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int hr = (wm * FM + i + dy) * HSIDE + fr + dx;
          af[i] = *(const VT*)(ha + hr * ROWB + ((ch ^ fsw(hr)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = mfma_chunk<T>(wreg[t][h][j], af[i], acc[i][j]);  // D[channel][pixel]
      }
    }
    // the next patch's halo (and this patch's epilogue operands) were issued a whole patch ago:
    // drain them now, before any store
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (AUX::N > 0) {
      {
        typedef typename Raw4<T>::type R4;
        EpiRows<T, FM, FN> R;
        const int px = lane & 15, lrow = lane >> 4;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int q = i * 16 + px;
          R.nz[i] = R.bnz[i] = 0.f;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            // channels 16j + 4·lrow … +3: chunk 2j + lrow/2, byte 8·(lrow & 1) within it
            const int off =
                q * (CPP * 16) + (((2 * j + (lrow >> 1)) ^ asw<FN>(q)) << 4) + ((lrow & 1) << 3);
            if constexpr (AUX::MASK) R.rma[i][j] = *(const R4*)(auxw + off);
            if constexpr (AUX::ACC) R.ryo[i][j] = *(const R4*)(auxw + off);
            if constexpr (AUX::TAP) {
              R.rta[i][j] = *(const R4*)(auxw + off);
              R.rtt[i][j] = *(const R4*)(auxw + TL::AUXW + off);
            }
          }
        }
        halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, 0, wm, wn, lane, -1, -1, &R, red, WM, 64);
      }
    } else {
      halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, 0, wm, wn, lane, -1, -1, nullptr, red, WM,
                                  64);
    }
    buf ^= 1;
  }
}

template <typename T, typename TL, int EPI>
static int launch_wres_(ConvK& k, int grid, size_t lds, hipStream_t st) {
  auto fn = conv_wres_kernel<T, TL, EPI>;
  if (const int rc = ensure_dyn_lds((const void*)fn, 160 * 1024); rc != MIA_OK) return rc;
  RedQ r;
  int rc = conv_red_begin(k, r,
                          halo_red_slots(k.a.H, k.a.W, TL::FM, TL::WM, k.prered), st);
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(TL::NT), lds, st, k);
  rc = check_launch("conv_wres");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

// the epilogue feature masks with a specialisation (the runtime-feature epilogue would spill next
// to the 288 resident weight registers): the launches of the attack step, vgg.py forward /
// input gradient and e4e IR-SE50 stage 1 (forward conv1 / conv2, input gradients of conv2 / conv1)
static bool wres_mask_ok(int f) {
  using namespace epi;
  switch (f) {
    case BIAS | RELU: case TAP | MASK: case 0: case PRELU: case BIAS | CSUM: case MASK | MSL:
    case ACC: case BIAS:
      return true;
    default:
      return false;
  }
}

bool conv_wres_eligible(const ConvK& k, int dtype) {
  if (tune(T_CONV_WRES) == 0) return false;
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  return dtype != MIA_F32 && k.ng == 1 && k.stride == 1 && G.kh == 3 && G.kw == 3 &&
         G.pad_y == 1 && G.pad_x == 1 && G.ho == a.H && G.wo == a.W && G.ay == 1 && G.ax == 1 &&
         G.by == 0 && G.bx == 0 && !a.shuffle_out && a.H % 16 == 0 && a.W % 16 == 0 &&
         a.Cin == 64 && a.Cout == 64 && k.HT == a.H && k.WT == a.W && !a.in_scale &&
         a.act_in == MIA_ACT_NONE && G.kpad >= 9 * 64 && wres_mask_ok(epi_mask(k)) &&
         (!a.tap_a || a.mask_a == a.tap_a);
}

template <typename TL>
static int launch_conv_wres_t(ConvK& k, int dtype, hipStream_t st) {
  const int ncu = device_cu_count();
  const int ntiles = k.a.N * (k.a.H / TL::PH) * (k.a.W / TL::PW);
  const int per = (ntiles + ncu - 1) / ncu;
  const int grid = (ntiles + per - 1) / per;  // contiguous runs: every block gets a non-empty one
  k.nbn = 1;
  k.nblk = ntiles;
  using namespace epi;
  const int f = epi_mask(k);
  const int naux = (f & TAP) ? 2 : ((f & MASK) ? 1 : 0) + ((f & ACC) ? 1 : 0);
  const size_t lds = 2 * (size_t)TL::HBUF + (size_t)TL::NW * naux * TL::AUXW + 3 * TL::WM * 64 * 4;
  k.prered = (f & CSUM);
  MIA_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      switch (f) {
        case BIAS | RELU: return launch_wres_<T, TL, BIAS | RELU>(k, grid, lds, st);
        case TAP | MASK: return launch_wres_<T, TL, TAP | MASK>(k, grid, lds, st);
        case 0: return launch_wres_<T, TL, 0>(k, grid, lds, st);
        case PRELU: return launch_wres_<T, TL, PRELU>(k, grid, lds, st);
        case BIAS | CSUM: return launch_wres_<T, TL, BIAS | CSUM>(k, grid, lds, st);
        case MASK | MSL: return launch_wres_<T, TL, MASK | MSL>(k, grid, lds, st);
        case ACC: return launch_wres_<T, TL, ACC>(k, grid, lds, st);
        case BIAS: return launch_wres_<T, TL, BIAS>(k, grid, lds, st);  // e4e conv2 (SE body)
        default: break;
      }
    }
  });
  return set_error("conv_wres: no specialisation for this launch (see conv_wres_eligible)");
}

int launch_conv_wres(ConvK& k, int dtype, hipStream_t st) {
  return launch_conv_wres_t<WresTile>(k, dtype, st);
}


// ---- 32 → 32-channel layers on an LDS halo (StyleGAN2 1024² StyledConvs, cm = 2) --------------
// The forward (x̃ = act(x)·s, + demod, noise, bias, leaky ReLU) and the input gradient (+ the
// style-gradient dot, the fused bias-act backward sums) of the 1024² StyledConvs
// (code/model.py ModulatedConv2d / StyledConv, channel_multiplier 2). K = 9 taps × 32 channels:
// ONE MFMA 16×16×32 K-chunk per tap, so the whole weight matrix is 9 × 2 B fragments = 72 VGPRs
// per wave, loaded once. Persistent blocks of 4 waves walk a contiguous run of 16×16-pixel patches
// (a patch's halo rows are mostly this block's own neighbouring patches: L2 hits on one XCD).
// Per patch t:
//   * the epilogue's per-pixel operands of t (noise, the stored activation of the sdot / bab
//     sums, the old y) are loaded into registers, THEN the (16+2)² × 64-B halo of patch t+1 (21
//     × 1 KB pieces, 16-B chunk c of halo pixel r for swizzled slot c ^ sw32(r)) — plain loads
//     only, so the epilogue's waits are counted (vmcnt(#halo loads)) and never wait for the next
//     halo (an LDS-DMA in flight makes every compiler-derived wait vmcnt(0));
//   * 9 taps × 4 ds_read_b128 A fragments and 8 MFMAs per wave, D[channel][pixel], then the
//     specialised register epilogue (halo_epilogue_f, FM = 4, FN = 2; the sdot / q / csum sums of
//     the 4 waves pre-reduced in LDS to one ordered slot per patch);
//   * the halo of t+1 lands under all that; it is written to the other LDS buffer (PRO: modulated
//     on the way, modulate<T> exactly as conv_thin32 rounds it per fragment read), and one
//     barrier per patch hands it over.
// Per-channel epilogue constants (demod / bias / bab) are loaded once per image of the run into
// LDS and read back per epilogue.
// Replaces conv_thin32 (16-B global gathers per tap, latency-bound at 100–210 TFLOP/s) where
// H % 16 == 0.
struct Wres32Tile {
  static constexpr int FM = 4, FN = 2, NW = 4, NT = 256;
  static constexpr int PH = 16, PW = 16, HSIDE = PW + 2, HROWS = (PH + 2) * HSIDE;  // 324
  static constexpr int RB = 64;                                // bytes per halo pixel
  static constexpr int HPIECES = (HROWS + 15) / 16;            // 21 pieces of 16 pixels (1 KB)
  static constexpr int H_INS = (HPIECES + NW - 1) / NW;        // ≤ 6 per wave
  static constexpr int HBUF = HPIECES * 1024;
  static constexpr int RED = 3 * NW * 32 * 4;                  // LDS pre-reduction
  static constexpr int STAB = 64;                              // s[n][·] as T (PRO)
  static constexpr int CTAB = 6 * 32 * 4;                      // per-channel epilogue constants
  static constexpr int LDS = 2 * HBUF + RED + STAB + CTAB;     // 45.4 KB: 3 blocks per CU
};

// 16-B chunk swizzle of a 64-B halo pixel row: every ds_read_b128 lane group (16 lanes: 8 pixels
// × 2 chunks, MI355X_MICROARCH.md §LDS) lands on 16 distinct 16-B bank slots for any base pixel
__device__ __forceinline__ int sw32(int r) { return (r >> 1) & 3; }

template <typename T, bool PRO, int EPI>
__global__ __launch_bounds__(256, 2) void conv_wres32_kernel(const ConvK k) {
  typedef Wres32Tile TL;
  typedef typename Vec<T>::type VT;
  typedef typename Raw4<T>::type R4;
  constexpr int FM = TL::FM, FN = TL::FN, HSIDE = TL::HSIDE, HROWS = TL::HROWS;
  constexpr int HPIECES = TL::HPIECES, HBUF = TL::HBUF, H_INS = TL::H_INS, NW = TL::NW;
  using namespace epi;
  constexpr bool NZ = EPI & NOISE, XS = EPI & (SDOT | BAB), YO = EPI & ACC, BB = EPI & BAB;
  constexpr bool PRE = NZ || XS || YO || BB;
  static_assert(!(EPI & (TAP | MASK)), "no tap / mask launches at 32 channels");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int H = p.H, W = p.W;
  const int ptx = W / TL::PW, pty = H / TL::PH;
  const int ntiles = p.N * ptx * pty;
  const T* __restrict__ X = (const T*)p.x;
  const T* __restrict__ Wt = (const T*)k.g[0].w;
  const int kpad = k.g[0].kpad;
  const T* zero = (const T*)g_zero16;
  float* const red = k.prered ? (float*)(smem + 2 * HBUF) : nullptr;
  T* const stab = (T*)(smem + 2 * HBUF + TL::RED);
  float* const ctab = (float*)(smem + 2 * HBUF + TL::RED + TL::STAB);  // [6][32]: EpiChan rows
  const bool lrelu_in = p.act_in == MIA_ACT_LRELU_S2;

  const int per = (ntiles + gridDim.x - 1) / gridDim.x;
  const int t0 = blockIdx.x * per, t1 = min(t0 + per, ntiles);
  if (t0 >= t1) return;

  // weights → VGPRs: B fragment (tap t, channel fragment j) = input channels 8·fq … of output
  // channel 16·j + frow
  VT wreg[9][FN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      wreg[t][j] = *(const VT*)(Wt + (size_t)(16 * j + frow) * kpad + t * 32 + fq * 8);

  auto tile_pos = [&](int tile, int& n, int& y0, int& x0) {
    x0 = (tile % ptx) * TL::PW;
    y0 = ((tile / ptx) % pty) * TL::PH;
    n = tile / (ptx * pty);
  };
  // wave wid holds halo pieces wid + NW·j: lane L = pixel piece·16 + L/4, slot L % 4 (logical
  // chunk (L % 4) ^ sw32(pixel)); padding reads the zero page
  VT hreg[H_INS];
  auto load_halo = [&](int tile) {
    int n, y0, x0;
    tile_pos(tile, n, y0, x0);
#pragma unroll
    for (int j = 0; j < H_INS; ++j) {
      const int piece = wid + NW * j;
      if (piece < HPIECES) {  // wave-uniform
        const int hr = piece * 16 + (lane >> 2);
        const int hy = hr / HSIDE, hx = hr - (hr / HSIDE) * HSIDE;
        const int y = y0 + hy - 1, x = x0 + hx - 1;
        const bool in = hr < HROWS && y >= 0 && y < H && x >= 0 && x < W;
        const T* a = X + ((size_t)(n * H + (in ? y : 0)) * W + (in ? x : 0)) * 32 +
                     ((lane & 3) ^ sw32(hr)) * 8;
        hreg[j] = *(const VT*)(in ? a : zero);
      }
    }
  };
  auto store_halo = [&](int buf) {
#pragma unroll
    for (int j = 0; j < H_INS; ++j) {
      const int piece = wid + NW * j;
      if (piece < HPIECES) {
        VT v = hreg[j];
        if constexpr (PRO) {  // act(x)·s rounded as conv_thin32 (zero padding stays zero)
          const int hr = piece * 16 + (lane >> 2);
          const VT sv = *(const VT*)(stab + ((lane & 3) ^ sw32(hr)) * 8);
          modulate<T>(v, sv, lrelu_in);
        }
        *(VT*)(smem + buf * HBUF + piece * 1024 + lane * 16) = v;
      }
    }
  };
  // PRO: s[n][·]·(√2) as T into stab (block-uniform call: the run reaches a new image)
  auto set_style = [&](int n) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of the old row are done
    __builtin_amdgcn_s_barrier();
    if (tid < 32) stab[tid] = from_f<T>(p.in_scale[(size_t)n * 32 + tid] * (lrelu_in ? SQRT2 : 1.f));
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
  };

  // prologue: the first patch's halo
  int n_first, yy, xx;
  tile_pos(t0, n_first, yy, xx);
  int sn = -1, en = -1;  // image of stab / of the epilogue constants
  load_halo(t0);
  if constexpr (PRO) {
    set_style(n_first);
    sn = n_first;
  }
  store_halo(0);
  // the per-channel epilogue constants of image n into ctab (block-uniform call, rare): one
  // wave loads them (EpiChan layout: lane group g = lane / 16 holds channels 4g … of each
  // 16-channel fragment) and stores its copy; the epilogue reads them back from LDS, so they
  // hold no registers across the MFMAs
  auto set_chan = [&](int n) {
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    if (wid == 0) {
      EpiChan<FN> E;
      epi_chan_load<EPI, FN>(k, E, n, (lane >> 4) << 2);
      if ((lane & 15) == 0) {
        const int cl = (lane >> 4) << 2;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          f32x4* r = (f32x4*)(ctab + cl + 16 * j);
          r[0] = E.osc[j];
          r[8] = E.bia[j];
          r[16] = E.dmv[j];
          r[24] = E.bbv[j];
          r[32] = E.msl[j];
          r[40] = E.asl[j];
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
  };
  int buf = 0;
  for (int tile = t0; tile < t1; ++tile) {
    // patch tile's halo is in buf (every wave stored its pieces), every wave finished the
    // previous patch (buf ^ 1 is free)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    int n, y0, x0;
    tile_pos(tile, n, y0, x0);
    if (n != en) {  // per-channel constants of a new image (block-uniform, rare)
      set_chan(n);
      en = n;
    }
    // the epilogue's per-pixel operands: raw loads, issued before the next halo
    EpiRows<T, FM, FN> R;
    if constexpr (PRE) {
      const int px = lane & 15, cl = (lane >> 4) << 2;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int y = y0 + wid * FM + i, x = x0 + px;
        const size_t m = (size_t)(n * H + y) * W + x;
        R.nz[i] = R.bnz[i] = 0.f;
        if constexpr (NZ) R.nz[i] = p.noise[y * W + x];
        if constexpr (BB)
          R.bnz[i] = *(p.bab_noise ? p.bab_noise + y * W + x : (const float*)g_zero16);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int c = cl + 16 * j;
          if constexpr (XS) R.rx[i][j] = *(const R4*)((const T*)p.aux_x + m * 32 + c);
          if constexpr (YO) R.ryo[i][j] = *(const R4*)((const T*)p.y + m * k.ystride + c);
        }
      }
    }
    const bool more = tile + 1 < t1;
    if (more) load_halo(tile + 1);

    const char* ha = smem + buf * HBUF;
    int fr = frow;
    asm volatile("" : "+v"(fr));
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3, dx = t - 3 * (t / 3);
      VT af[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int hr = (wid * FM + i + dy) * HSIDE + fr + dx;
        af[i] = *(const VT*)(ha + hr * TL::RB + ((fq ^ sw32(hr)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma_chunk<T>(wreg[t][j], af[i], acc[i][j]);  // D[channel][pixel]
    }
    if constexpr (NZ || BB) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (NZ) R.nz[i] = p.noise_w * R.nz[i];
        if constexpr (BB) R.bnz[i] = p.bab_noise_w * R.bnz[i];
      }
    }
    EpiChan<FN> E;
    {
      const int cl = (lane >> 4) << 2;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const f32x4* r = (const f32x4*)(ctab + cl + 16 * j);
        E.osc[j] = r[0];
        E.bia[j] = r[8];
        E.dmv[j] = r[16];
        E.bbv[j] = r[24];
        E.msl[j] = r[32];
        E.asl[j] = r[40];
      }
    }
    halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, 0, wid, 0, lane, -1, -1, PRE ? &R : nullptr,
                                red, NW, 32, nullptr, &E);
    if (more) {  // block-uniform
      if constexpr (PRO) {
        const int n1 = (tile + 1) / (ptx * pty);
        if (n1 != sn) {
          set_style(n1);
          sn = n1;
        }
      }
      store_halo(buf ^ 1);
    }
    buf ^= 1;
  }
}

static bool wres32_mask_ok(int f, bool pro) {
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

// Eligible: 2-byte type, 32 → 32 channels, one group, stride 1, 3×3 pad 1, identity placement,
// 16-divisible maps, dense output rows, a feature mask with a specialisation (the StyledConv
// forward / input gradient). T_CONV_WRES32 = 0 disables (tests / tuning).
bool conv_wres32_eligible(const ConvK& k, int dtype) {
  if (tune(T_CONV_WRES32) == 0) return false;
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  if (dtype == MIA_F32 || k.ng != 1 || k.stride != 1 || G.kh != 3 || G.kw != 3 || G.pad_y != 1 ||
      G.pad_x != 1 || G.ho != a.H || G.wo != a.W || G.ay != 1 || G.ax != 1 || G.by != 0 ||
      G.bx != 0 || a.shuffle_out || a.H % 16 != 0 || a.W % 16 != 0 || k.HT != a.H ||
      k.WT != a.W || k.ystride != a.Cout || a.Cin != 32 || a.Cout != 32 || G.kpad < 9 * 32 ||
      !a.y)
    return false;
  const bool pro = a.in_scale != nullptr;
  if (!pro && a.act_in != MIA_ACT_NONE) return false;
  if (pro && k.cout_mod != a.Cout) return false;
  return wres32_mask_ok(epi_mask(k), pro);
}

template <typename T, bool PRO, int EPI>
static int launch_wres32_(ConvK& k, hipStream_t st) {
  typedef Wres32Tile TL;
  auto fn = conv_wres32_kernel<T, PRO, EPI>;
  // blocks per CU of this instantiation (a thread-safe function-local static), × the device's CUs
  static const int occ = [&] {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (const void*)fn, TL::NT, TL::LDS) !=
            hipSuccess || o < 1)
      o = 1;
    return o;
  }();
  const int per_cu = device_cu_count() * occ;
  const int ntiles = k.a.N * (k.a.H / TL::PH) * (k.a.W / TL::PW);
  const int grid = std::min(ntiles, per_cu);
  k.nbn = 1;
  k.nblk = ntiles;
  constexpr bool RED = (EPI & (epi::SDOT | epi::BAB | epi::CSUM)) != 0;
  k.prered = RED;
  RedQ r;
  int rc = conv_red_begin(k, r, halo_red_slots(k.a.H, k.a.W, TL::FM, TL::NW, k.prered), st);
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(TL::NT), TL::LDS, st, k);
  rc = check_launch("conv_wres32");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

int launch_conv_wres32(ConvK& k, int dtype, hipStream_t st) {
  using namespace epi;
  const bool pro = k.a.in_scale != nullptr;
  MIA_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      if (pro) return launch_wres32_<T, true, OSC | NOISE | BIAS | LRELU>(k, st);
      switch (epi_mask(k)) {
        case OSC | SDOT: return launch_wres32_<T, false, OSC | SDOT>(k, st);
        case OSC | SDOT | ACC: return launch_wres32_<T, false, OSC | SDOT | ACC>(k, st);
        case OSC | SDOT | BAB: return launch_wres32_<T, false, OSC | SDOT | BAB>(k, st);
        case OSC | SDOT | ACC | BAB:
          return launch_wres32_<T, false, OSC | SDOT | ACC | BAB>(k, st);
        case 0: return launch_wres32_<T, false, 0>(k, st);
        case ACC: return launch_wres32_<T, false, ACC>(k, st);
        default: break;
      }
    }
  });
  return set_error("conv_wres32: no specialisation for this launch");
}

}  // namespace mia
