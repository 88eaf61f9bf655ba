// Weights-resident persistent 3×3 conv for the 64 → 64-channel layers (NHWC, fp16/bf16, CDNA4).
//
// Serves VGG conv1_2 forward and input gradient (code/vgg.py:45-62, 256²) and the e4e encoder's
// first IR-SE50 stage (Encoder4Editing body units 0-2 conv1/conv2 and their input gradients,
// 256² / 128²; un-vendored, code/utils/model_utils.py:24). At Cout = 64 the tiled kernels pay the
// per-K-step weight staging and barrier for half the MFMAs of a 128-channel tile (measured 375-
// 440 TFLOP/s); here the whole weight matrix (K = 9·64 = 576 × 64 channels = 72 KB) is loaded
// ONCE per wave into VGPRs as MFMA B fragments (288 registers, one wave per SIMD) and the block
// is persistent over 16×16-pixel output patches:
//   * per patch the (16+2)×(16+2) input halo (one 64-channel block, 41 KB) is DMA'd into one of
//     two LDS buffers a full patch ahead (global_load_lds, bank swizzle fsw() through the source
//     chunk, zero page for the padding);
//   * the main loop is 9 taps × 2 K-chunks of ds_read_b128 A fragments and 16 MFMAs each, with
//     no barrier and no weight traffic;
//   * one barrier per patch (all waves finished the previous patch and waited for their DMA
//     pieces) before the next halo is issued into the buffer just released; each wave drains its
//     DMA (vmcnt(0)) AFTER its MFMAs and BEFORE its epilogue stores, so the wait never covers
//     stores and the DMA had a whole patch to land;
//   * the epilogue is halo_epilogue_f (registers, 16-byte stores); a single per-pixel operand
//     (mask or old y) is DMA'd into LDS at the start of the patch (WresAux) and lands during the
//     MFMAs instead of stalling the epilogue.
// Wave w owns patch rows 4w … 4w+3 (one 16-pixel MFMA fragment per row) × all 64 channels.
#include "conv_common.h"
#include "halo_epilogue.h"

namespace mia {

struct WresTile {
  static constexpr int FM = 4, FN = 4, NW = 4, NT = 256;
  static constexpr int PH = 16, PW = 16, HSIDE = PW + 2, HROWS = (PH + 2) * HSIDE;  // 324
  static constexpr int HPIECES = (HROWS + 7) / 8;                                    // 41
  static constexpr int HBUF = HPIECES * 8 * ROWB;
  static constexpr int H_INS = (HPIECES + NW - 1) / NW;                              // 11
  static constexpr int AUXW = FM * 16 * ROWB;  // one per-pixel epilogue operand of a wave: 8 KB
};

// Per-pixel epilogue operand prefetched into LDS (a wave's 64 pixels × 64 channels): MASK →
// mask_a, ACC → old y. Register prefetch spills next to the 288 resident weight VGPRs; LDS-DMA
// costs no registers. The tap pair (TAP | MASK, VGG dgrad) still loads in the epilogue: with two
// operands the epilogue's extra live registers spill the weights (measured in the ISA: reloads
// with vmcnt(0) inside the MFMA loop).
template <int EPI>
struct WresAux {
  static constexpr bool TAP = EPI & epi::TAP, MASK = (EPI & epi::MASK) && !TAP;
  static constexpr bool ACC = EPI & epi::ACC;
  static constexpr int N = TAP ? 0 : (MASK ? 1 : 0) + (ACC ? 1 : 0);
  static_assert(N <= 1, "one prefetched operand per wave");
  static_assert(!(EPI & (epi::SDOT | epi::BAB | epi::NOISE)), "not a weights-resident epilogue");
};

// bank swizzle of the prefetched operand rows (16-B chunk c of pixel q stored at c ^ asw(q)): a
// ds_read_b64 of 16 pixels × one channel quad pair hits 16 distinct (pixel parity, chunk) slots
__device__ __forceinline__ int asw(int q) { return (q >> 1) & 7; }

// EPI: the epilogue feature mask (halo_epilogue.h, specialised only; see wres_mask_ok); wave wm
// owns rows wm·FM …, wn = 0, n0 = 0
template <typename T, int EPI>
__global__ __launch_bounds__(256, 1) void conv_wres_kernel(const ConvK k) {
  typedef WresTile TL;
  typedef typename Vec<T>::type VT;
  constexpr int FM = TL::FM, FN = TL::FN, HSIDE = TL::HSIDE, HROWS = TL::HROWS;
  constexpr int HPIECES = TL::HPIECES, HBUF = TL::HBUF, H_INS = TL::H_INS, NW = TL::NW;
  constexpr int VEC = 8;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef WresAux<EPI> AUX;
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

  // weights → VGPRs: B fragment (tap t, K-chunk h, channel fragment j) = 8 input channels
  // (h·4 + fq)·8 … of output channel 16·j + frow
  VT wreg[9][2][FN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        wreg[t][h][j] = *(const VT*)(Wt + (size_t)(16 * j + frow) * kpad + t * 64 +
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

  // wave wid DMAs the epilogue operands of its 4 output rows (pieces of 8 pixels = 1 KB)
  char* const auxw = smem + 2 * HBUF + wid * (AUX::N * TL::AUXW);  // this wave's operand slots
  // sdot / q / csum pre-reduction of the 4 waves (each covers all 64 channels of its rows)
  float* const red = k.prered ? (float*)(smem + 2 * HBUF + NW * AUX::N * TL::AUXW) : nullptr;
  auto issue_aux = [&](int n, int y0, int x0) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const T* srcs[1] = {AUX::MASK ? (const T*)p.mask_a : (const T*)p.y};
#pragma unroll
    for (int t = 0; t < AUX::N; ++t)
#pragma unroll
      for (int j = 0; j < FM * 2; ++j) {
        const int q = j * 8 + (ln >> 3);  // wave-local pixel: row q / 16, column q % 16
        const int y = y0 + wid * FM + (q >> 4), x = x0 + (q & 15);
        const T* src = srcs[t] + ((size_t)(n * H + y) * W + x) * 64 + ((ln & 7) ^ asw(q)) * VEC;
        __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(auxw + t * TL::AUXW + j * 1024),
                                         16, 0, 0);
        __builtin_amdgcn_sched_barrier(0);  // one address live at a time (weights fill the VGPRs)
      }
  };

  int tile = blockIdx.x;
  if (tile < ntiles) issue_halo(tile, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int buf = 0;
  for (; tile < ntiles; tile += gridDim.x) {
    // every wave finished the previous patch (buffer buf^1 is free) and drained its DMA pieces
    // of this patch (buffer buf is complete)
    __syncthreads();
    const int next = tile + gridDim.x;
    int n, y0, x0;
    tile_pos(tile, n, y0, x0);
    if constexpr (AUX::N > 0) issue_aux(n, y0, x0);  // land during this patch's MFMAs
    if (next < ntiles) issue_halo(next, buf ^ 1);
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
          const int hr = (wid * FM + i + dy) * HSIDE + fr + dx;
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
            const int off = q * ROWB + (((2 * j + (lrow >> 1)) ^ asw(q)) << 4) + ((lrow & 1) << 3);
            if constexpr (AUX::MASK) R.rma[i][j] = *(const R4*)(auxw + off);
            if constexpr (AUX::ACC) R.ryo[i][j] = *(const R4*)(auxw + off);
          }
        }
        halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, 0, wid, 0, lane, -1, -1, &R, red, NW, 64);
      }
    } else {
      halo_epilogue_f<T, TL, EPI>(k, acc, n, y0, x0, 0, wid, 0, lane, -1, -1, nullptr, red, NW,
                                  64);
    }
    buf ^= 1;
  }
}

template <typename T, int EPI>
static int launch_wres_(ConvK& k, int grid, size_t lds, hipStream_t st) {
  auto fn = conv_wres_kernel<T, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    attr_set = true;
  }
  RedQ r;
  int rc = conv_red_begin(k, r,
                          halo_red_slots(k.a.H, k.a.W, WresTile::FM, WresTile::NW, k.prered), st);
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(WresTile::NT), lds, st, k);
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
    case ACC:
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
         a.act_in == MIA_ACT_NONE && G.kpad >= 9 * 64 && wres_mask_ok(epi_mask(k));
}

int launch_conv_wres(ConvK& k, int dtype, hipStream_t st) {
  typedef WresTile TL;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  const int ntiles = k.a.N * (k.a.H / TL::PH) * (k.a.W / TL::PW);
  const int grid = std::min(ntiles, ncu);
  k.nbn = 1;
  k.nblk = ntiles;
  using namespace epi;
  const int f = epi_mask(k);
  const int naux = (f & TAP) ? 0 : ((f & MASK) ? 1 : 0) + ((f & ACC) ? 1 : 0);
  const size_t lds = 2 * (size_t)TL::HBUF + (size_t)TL::NW * naux * TL::AUXW + 3 * TL::NW * 64 * 4;
  k.prered = prered_enabled() && (f & CSUM);
  MIA_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      switch (f) {
        case BIAS | RELU: return launch_wres_<T, BIAS | RELU>(k, grid, lds, st);
        case TAP | MASK: return launch_wres_<T, TAP | MASK>(k, grid, lds, st);
        case 0: return launch_wres_<T, 0>(k, grid, lds, st);
        case PRELU: return launch_wres_<T, PRELU>(k, grid, lds, st);
        case BIAS | CSUM: return launch_wres_<T, BIAS | CSUM>(k, grid, lds, st);
        case MASK | MSL: return launch_wres_<T, MASK | MSL>(k, grid, lds, st);
        case ACC: return launch_wres_<T, ACC>(k, grid, lds, st);
        default: break;
      }
    }
  });
  return set_error("conv_wres: no specialisation for this launch (see conv_wres_eligible)");
}

}  // namespace mia
