// Weights-resident persistent 3×3 conv with 128 output channels (NHWC, fp16 / bf16, CDNA4):
// the StyledConv forward of the 256² generator block on per-image modulated + demodulated weights
// (rosinality ModulatedConv2d's weight path, code/attack/attack_main2.py:619-621 decoder call;
// channel_multiplier 2: 128 → 128 channels at 256², K = 9·128 = 1 152).
//
// Why: the halo tile (conv_halo.hip, 8×16 patch × 128 channels, one block per patch) spends a
// fifth of every block in its prologue (the first halo from HBM) and its epilogue, and streams
// every K-step's weights through an LDS ring with a block barrier per step; at K = 1 152 those
// fixed costs are not amortised (profiles/r04_fp16_halo_phases_wmod.txt: prologue 8.4 k +
// epilogue 4.9 k of ≈ 41 k cycles per block, 837–866 TFLOP/s). Here:
//   * each of the 8 waves (two per SIMD) holds the B fragment of ITS 16 output channels over the
//     whole K in VGPRs: 9 taps × (Cin/32) K-chunks × 4 VGPRs = 144 at Cin = 128, loaded once per
//     image (per-image weights: a block's run covers about half an image, so one reload per run)
//     — no weight ring, no per-step barrier. Two waves per SIMD: one wave's epilogue, DMA issue
//     and LDS waits run under its partner's MFMAs (the first form, 4 waves × 32 channels with 288
//     weight VGPRs and one wave per SIMD, measured 831 TFLOP/s against the halo tile's 868);
//   * the block is persistent over a contiguous run of 8×16-pixel patches; the (8+2)×(16+2)
//     halo of the next patch is DMA'd into the other LDS buffer a whole patch ahead (one barrier
//     per patch), so no patch waits for HBM;
//   * every wave computes all 128 patch pixels × its 16 channels (acc 8 fragments). The A
//     fragment of halo row q, column shift dx and K-chunk s feeds the three taps (dy = 0, 1, 2)
//     of output rows q − dy: 120 ds_read_b128 per wave per patch for 288 MFMAs, read three ahead
//     (MIA_WRES128_PF) as inline-asm ds_read_b128 with counted lgkmcnt waits;
//   * the epilogue (noise, bias, leaky ReLU · √2) runs in registers; the patch's noise rows are
//     DMA'd into LDS with the halo and the bias sits in VGPRs, so it waits on nothing.
// Halo LDS image (2-byte types, PB = 2·Cin bytes per pixel): halo rows padded to HS = 20 pixels
// (columns 18, 19 never read), pixels in groups of 4 (GB = 4·PB bytes): pixel hr, 32-channel
// sub-plane s, 16-B chunk c at (hr / 4)·GB + s·256 + (hr % 4)·64 + (c ^ sw(hr % 20))·16. Row q
// starts at group 5q, so a fragment address is a lane constant per column shift dx plus the
// immediate q·5·GB + s·256; sw(v) = (v >> 1) & 3 keeps every ds_read_b128 lane group on 16
// distinct 16-B bank slots for any dx (checked exhaustively, tests/test_host.py).
#include "conv_common.h"
#include "halo_epilogue.h"

// fragment reads issued this many fragments ahead of their MFMAs, as inline asm with counted
// waits (tuning build flags; round 5: PF 3 asm vs 1 compiler-scheduled: 256² forward 2135 -> 2072,
// input gradient 2404 -> 2366, VGG 128² 464 -> 455 µs, profiles/r05_layers_fp16_wres128_pf.txt)
#ifndef MIA_WRES128_PF
#define MIA_WRES128_PF 3
#endif
#ifndef MIA_WRES128_ASMREAD
#define MIA_WRES128_ASMREAD 1
#endif

namespace mia {

template <int CIN, int COUT = 128>
struct Wres128Tile {
  // wave (row group wid / WNC, channel group wid % WNC): FM patch rows × 16 output channels
  static constexpr int NW = 8, NT = 512, PH = 8, PW = 16, BN = COUT;
  static constexpr int WNC = COUT / 16, WMR = NW / WNC, FM = PH / WMR;
  static_assert((COUT == 128 || COUT == 64) && WMR * WNC == NW, "8 waves of 16 channels");
  static constexpr int HS = 20, HROWS = (PH + 2) * HS;  // 200 halo pixels
  static constexpr int PB = 2 * CIN, GB = 4 * PB;       // bytes per pixel / per 4-pixel group
  static constexpr int NS = CIN / 32;                   // K-chunks (32-channel sub-planes) per tap
  static constexpr int HBUF = HROWS * PB;               // 51 200 B at Cin = 128
  static constexpr int NPIECE = HBUF / 1024;            // 1-KB DMA pieces per halo (50)
  static constexpr int P_INS = (NPIECE + NW - 1) / NW;  // pieces per wave (≤ 7)
  static constexpr int NZB = 1024;                      // per wave: the patch's noise rows
  static constexpr int AXB = FM * 16 * 32;              // per wave: 16 channels of aux_x (4 KB)
  static constexpr int CHB = 256;                       // per wave: 3 × 16 per-channel constants
  // a 1-KB DMA piece = 1024 / GB 4-pixel groups (Cin 128: one, Cin 64: two)
  static_assert((CIN == 128 || CIN == 64) && HBUF % 1024 == 0, "halo layout");
};

__device__ __forceinline__ int sw128(int v) { return (v >> 1) & 3; }

// EPI (halo_epilogue.h feature masks, the same per-element operations in the same order):
//   NOISE | BIAS | LRELU — the StyledConv forward on per-image modulated + demodulated weights
//     (k.wn > 0: the images' matrices wn elements apart);
//   OSC | SDOT | BAB — the StyledConv input gradient of the 256² block with the style-gradient dot
//     (sdot) and the fused backward front of the layer below (bab: its lrelu', demod scale and the
//     q sum), on the shared dgrad matrix (k.wn = 0).
template <typename T, int CIN, int EPI, int COUT = 128>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_wres128_kernel(const ConvK k) {
  typedef Wres128Tile<CIN, COUT> TL;
  typedef typename Vec<T>::type VT;
  using namespace epi;
  constexpr int FM = TL::FM, NW = TL::NW, NS = TL::NS, HBUF = TL::HBUF, NPIECE = TL::NPIECE;
  constexpr int GB = TL::GB, P_INS = TL::P_INS;
  constexpr bool FWD = EPI == (NOISE | BIAS | LRELU);  // StyledConv forward, per-image weights
  constexpr bool DG = EPI == (OSC | SDOT | BAB);
  // shared-weight launches with a plain per-element epilogue (halo_epilogue_f's operations in
  // its order): VGG forward BIAS | RELU and input gradient MASK; e4e IR-SE body (128 channels)
  // conv1 PRELU, conv2 BIAS, the input gradients MASK | MSL (PReLU') and ACC (identity shortcut)
  constexpr bool GEN = EPI == 0 || EPI == (BIAS | RELU) || EPI == MASK || EPI == PRELU ||
                       EPI == BIAS || EPI == (MASK | MSL) || EPI == ACC;
  static_assert(COUT == 128 || GEN, "Cout 64: the shared-weight plain epilogues");
  static_assert(FWD || DG || GEN, "the StyledConv / VGG / e4e epilogues");
  constexpr bool G_BIAS = GEN && (EPI & BIAS), G_MASK = GEN && (EPI & MASK);
  constexpr bool G_MSL = GEN && (EPI & MSL), G_ACC = GEN && (EPI & ACC);
  constexpr bool G_RELU = GEN && ((EPI >> 8) & 3) == MIA_ACT_RELU;
  constexpr bool G_PRELU = GEN && ((EPI >> 8) & 3) == MIA_ACT_PRELU;
  constexpr bool NZ = FWD || DG;              // noise rows DMA'd per patch
  constexpr bool AUXX = DG || G_MASK || G_ACC;  // a 16-channel per-pixel operand DMA'd per patch
  constexpr int SLOTB = TL::CHB + TL::NZB + (AUXX ? TL::AXB : 0);  // per-wave epilogue operands
  // DG: the next halo's DMA pieces are issued one per (dx, s) fragment group inside the MFMA loop
  // (868 → 906 TFLOP/s); the forward keeps them at the patch start (1207 vs 1182 spread;
  // profiles/r05_layers_fp16_{spread,nospread}.txt)
  constexpr bool SPREAD = DG;
  static_assert(!SPREAD || 3 * NS >= P_INS, "one piece per fragment group");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const mia_conv_args& p = k.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const int H = p.H, W = p.W, Cout = p.Cout;
  const int ptx = W / TL::PW, pty = H / TL::PH;
  const int ntiles = p.N * ptx * pty;
  // Cout = nct · BN: blocks [ct·runs, (ct+1)·runs) take output channels ct·BN … of every patch
  const int nct = Cout / TL::BN, runs = gridDim.x / nct;
  const int ct = blockIdx.x / runs, rb = blockIdx.x - ct * runs;
  const int per = (ntiles + runs - 1) / runs;
  const int t0 = rb * per, t1 = min(t0 + per, ntiles);
  if (t0 >= t1) return;
  const T* __restrict__ X = (const T*)p.x;
  const T* __restrict__ W0 = (const T*)k.g[0].w;
  const int kpad = k.g[0].kpad;
  T* __restrict__ Y = (T*)p.y;
  const int cw0 = TL::BN * ct + 16 * (wid % TL::WNC);  // this wave's first output channel
  const int row0 = FM * (wid / TL::WNC);  // and its first patch row
  const int cl = cw0 + ((lane >> 4) << 2);  // this lane's 4 channels (lane row r: cw0 + 4r …)
  // the zero page for padding lanes, loaded once (not rematerialised per DMA piece)
  const T* zero = (const T*)g_zero16;
  asm volatile("" : "+s"(zero));

  auto tile_pos = [&](int tile, int& n, int& y0, int& x0) {
    x0 = (tile % ptx) * TL::PW;
    y0 = ((tile / ptx) % pty) * TL::PH;
    n = tile / (ptx * pty);
  };

  // B fragments of this wave's 16 channels: (tap t, K-chunk s) = input channels s·32 + fq·8 …
  // +7 of tap t for output channel cw0 + frow
  VT wreg[9][NS];
  auto load_w = [&](int n) {
    const T* Wn = W0 + (size_t)n * k.wn + (size_t)(cw0 + frow) * kpad + fq * 8;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int s = 0; s < NS; ++s) wreg[t][s] = *(const VT*)(Wn + t * CIN + s * 32);
  };
  // per-channel epilogue constants of image n (FWD: the bias; DG: style s, the layer below's
  // demod and bias), kept in this wave's LDS slot [3][16] (not in registers across the MFMAs)
  char* const slot = smem + 2 * HBUF + wid * SLOTB;
  float* const chl = (float*)slot;
  auto load_chan = [&](int n) {
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f}, c2 = {0.f, 0.f, 0.f, 0.f};
    if constexpr (FWD || G_BIAS) {
      c0 = *(const f32x4*)(p.bias + cl);
    } else if constexpr (G_PRELU) {
      c0 = *(const f32x4*)(p.act_slope + cl);
    } else if constexpr (G_MSL) {
      c0 = *(const f32x4*)(p.mask_slope + cl);
    } else if constexpr (DG) {
      c0 = *(const f32x4*)(p.out_scale + (size_t)n * k.cout_mod + cl);
      c1 = *(const f32x4*)(p.bab_demod + (size_t)n * Cout + cl);
      c2 = *(const f32x4*)(p.bab_bias ? p.bab_bias + cl : (const float*)zero);
    }
    if ((lane & 15) == 0) {  // (a wave's LDS accesses execute in order: no wait before reads)
      *(f32x4*)(chl + cl - cw0) = c0;
      *(f32x4*)(chl + 16 + cl - cw0) = c1;
      *(f32x4*)(chl + 32 + cl - cw0) = c2;
    }
  };

  // wave wid DMAs halo pieces wid + NW·j; piece pc = halo row pc / 5, pixels 4·(pc % 5) …
  auto issue_piece = [&](int j, int n, int y0, int x0, int buf) {
    const int pc = wid + NW * j;  // wave-uniform
    if (pc >= NPIECE) return;
    // the lane's part of a DMA piece (one 4-pixel group of a halo row): sub-plane s, pixel pp of
    // the group, stored chunk cs (LDS byte 16·lane of the piece); from an opaque copy of the lane
    // id, so the per-piece lane terms are recomputed per patch instead of hoisted (they spilled)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    // LDS byte 16·lane of the piece: group gi, sub-plane ls, pixel lpp of the group, chunk lcs
    constexpr int GPP = 1024 / GB;  // groups per piece
    const int gi = (ln * 16) / GB, lb = (ln * 16) % GB;
    const int ls = lb >> 8, lpp = (lb >> 6) & 3, lcs = (lb >> 4) & 3;
    const int hp = (pc * GPP + gi) * 4 + lpp;  // padded halo pixel (rows of HS)
    const int hy = hp / TL::HS, hx = hp - TL::HS * hy;
    const int y = y0 + hy - 1;
    const int x = x0 + hx - 1;
    const bool ok = y >= 0 && y < H && hx < TL::PW + 2 && x >= 0 && x < W;
    const int yc = ok ? y : 0, xc = ok ? x : 0;
    const T* a = X + ((size_t)(n * H + yc) * W + xc) * CIN + ls * 32 + ((lcs ^ sw128(hx)) << 3);
    __builtin_amdgcn_global_load_lds((gptr_t)(ok ? a : zero),
                                     (lptr_t)(smem + buf * HBUF + pc * 1024), 16, 0, 0);
  };
  auto issue_halo = [&](int tile, int buf) {
    int n, y0, x0;
    tile_pos(tile, n, y0, x0);
#pragma unroll
    for (int j = 0; j < P_INS; ++j) issue_piece(j, n, y0, x0, buf);
  };
  // this wave's epilogue operands of the patch, DMA'd at its start (they land during the MFMAs):
  // the noise rows (FWD: the layer's noise; DG: the layer below's) as 8 rows × 16 floats (lanes
  // ≥ 32 read zeros), and (DG) its 16 channels of aux_x for the 128 pixels: pixel q's two 16-B
  // chunks at q·32 + ((c ^ (q >> 3)) & 1)·16 (ds_read_b64 of the epilogue conflict-free)
  char* const aux = slot + TL::CHB;
  auto issue_aux = [&](int n, int y0, int x0) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    if constexpr (NZ) {
      const float* nzp = FWD ? p.noise : p.bab_noise;
      const float* src = ln < 32 && nzp ? nzp + (size_t)(y0 + (ln >> 2)) * W + x0 + 4 * (ln & 3)
                                        : (const float*)zero;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)aux, 16, 0, 0);
    }
    if constexpr (AUXX) {  // DG: the stored activation aux_x; MASK: the mask operand; ACC: old y
      const T* AX = (const T*)(DG ? p.aux_x : (G_MASK ? p.mask_a : p.y));
#pragma unroll
      for (int j = 0; j < FM / 2; ++j) {
        const int q = j * 32 + (ln >> 1), c = (ln & 1) ^ ((q >> 3) & 1);
        const T* a =
            AX + ((size_t)(n * H + y0 + row0 + (q >> 4)) * W + x0 + (q & 15)) * Cout + cw0 + 8 * c;
        __builtin_amdgcn_global_load_lds((gptr_t)a, (lptr_t)(aux + TL::NZB + j * 1024), 16, 0,
                                         0);
      }
    }
  };

  int wimg = -1;
  {
    int n, y0, x0;
    tile_pos(t0, n, y0, x0);
    load_w(n);
    load_chan(n);
    wimg = n;
  }
  issue_halo(t0, 0);
  // vmcnt(0) as the builtin (the compiler's wait insertion sees it and adds none later for the
  // weight registers; an inline-asm wait is opaque to it)
  __builtin_amdgcn_s_waitcnt(0x0f70);
  int buf = 0;
  for (int tile = t0; tile < t1; ++tile) {
    // every wave finished the previous patch (buffer buf^1 and its operand slot are free) and
    // drained its DMA pieces of this patch (buffer buf is complete). LDS-only hand-off: no
    // vector-memory wait, so the previous epilogue's stores stay in flight
    lds_handoff();
    int n, y0, x0;
    tile_pos(tile, n, y0, x0);
    issue_aux(n, y0, x0);
    // SPREAD: the next patch's halo pieces go out inside the MFMA loop, each wave's DMA issue
    // overlapping its own MFMAs
    const bool more = tile + 1 < t1;
    int n1 = 0, y1 = 0, x1 = 0;
    if (more) tile_pos(tile + 1, n1, y1, x1);
    if (more && !SPREAD) issue_halo(tile + 1, buf ^ 1);
    const char* hb = smem + buf * HBUF;
    // lane-constant A-fragment offsets per column shift dx (pixel column v = frow + dx),
    // recomputed per patch from an opaque lane id (held across the whole run they were spilled,
    // and the reload's vmcnt wait then also waited for the next halo's DMA)
    int offa[3];
    {
      int ln = lane;
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int v = (ln & 15) + dx, f = ln >> 4;
        offa[dx] = (v >> 2) * GB + (v & 3) * 64 + ((f ^ sw128(v)) << 4);
      }
    }
    f32x4 acc[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the 120 fragment reads in (dx, s, q) order, each feeding the taps dy = 0, 1, 2 of output
    // row q − dy; the next read is issued before the current fragment's MFMAs
    const char* hd[3] = {hb + offa[0] + row0 * 5 * GB, hb + offa[1] + row0 * 5 * GB,
                         hb + offa[2] + row0 * 5 * GB};
    // fragment f = (dx·NS + s)·(FM + 2) + q, read PF fragments ahead into a ring of PF + 1
    constexpr int NQ = FM + 2, NF = 3 * NS * NQ, PF = MIA_WRES128_PF;
#if MIA_WRES128_ASMREAD
    // the reads as inline asm with explicit counted waits (the compiler's own waits were
    // lgkmcnt(0) right after the next read's issue, exposing the LDS latency every few MFMAs).
    // Safe beside the compiler's own LDS waits: an unknown younger read only makes them stricter;
    // the MFMA loop issues no other LDS operation between a read and its wait.
    unsigned hl[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) hl[d] = (unsigned)(size_t)(lptr_t)(hd[d]);
    auto frag = [&](int f) {
      const int dxf = f / (NS * NQ), rf = f % (NS * NQ);
      VT v;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(hl[dxf] + (rf % NQ) * 5 * GB + (rf / NQ) * 256));
      return v;
    };
#else
    auto frag = [&](int f) {
      const int dxf = f / (NS * NQ), rf = f % (NS * NQ);
      return *(const VT*)(hd[dxf] + (rf % NQ) * 5 * GB + (rf / NQ) * 256);
    };
#endif
    VT ring[PF + 1];
#pragma unroll
    for (int f = 0; f < PF; ++f) ring[f] = frag(f);
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int f = (dx * NS + s) * NQ + q;
          if (f + PF < NF) ring[(f + PF) % (PF + 1)] = frag(f + PF);
          VT cur = ring[f % (PF + 1)];
#if MIA_WRES128_ASMREAD
          {  // fragment f landed: at most the reads issued after it (f+1 … f+PF) outstanding
            const int younger = NF - 1 - f < PF ? NF - 1 - f : PF;
            if (younger >= 3) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(cur));
            else if (younger == 2) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(cur));
            else if (younger == 1) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(cur));
            else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur));
          }
#endif
#pragma unroll
          for (int dy = 0; dy < 3; ++dy) {
            const int i = q - dy;
            if (i < 0 || i >= FM) continue;
            acc[i] = mfma_chunk<T>(wreg[dy * 3 + dx][s], cur, acc[i]);  // D[channel][pixel]
          }
          if constexpr (SPREAD) {
            const int g = dx * NS + s;
            if (q == 1 && g < P_INS && more) {
              __builtin_amdgcn_sched_barrier(0);
              issue_piece(g, n1, y1, x1, buf ^ 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
    // the next patch's halo and this patch's operands were issued during its MFMAs: drain them
    // before the epilogue's stores (vmcnt retires in order); the empty asm keeps the epilogue's
    // LDS reads of the DMA'd operands below the wait
    __builtin_amdgcn_s_waitcnt(0x0f70);
    asm volatile("" ::: "memory");
    // lane terms of the epilogue from an opaque copy of the lane id: held across the patch loop
    // (8 aux row offsets + the channel slot) they were spilled, and each scratch reload's
    // vmcnt(0) then waited for the epilogue's own stores (DG 2849 µs vs 2069 without its math)
    int ln_e = lane;
    asm volatile("" : "+v"(ln_e));
    const int px = ln_e & 15, lrow = ln_e >> 4;
    const int cle = (lrow << 2);  // this lane's channel quad within the wave's 16
    const float* nz = (const float*)aux;
    const float nzw = FWD ? p.noise_w : (DG ? p.bab_noise_w : 0.f);
    // (DG: the per-channel constants are re-read from LDS per row pair below — held across the
    // epilogue they pushed the kernel past 256 VGPRs)
    const f32x4 c0 = FWD || GEN ? *(const f32x4*)(chl + cle) : f32x4{0.f, 0.f, 0.f, 0.f};
    float part[4] = {0.f, 0.f, 0.f, 0.f}, partq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < FM; i += 2) {
      // rows i, i+1: after the swap lane row r holds channels 8·(r >> 1) … +7 of row i + (r & 1)
      float vo[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float z = NZ ? nzw * nz[(row0 + i + u) * 16 + px] : 0.f;
        typedef T t4 __attribute__((ext_vector_type(4)));
        const int q = (i + u) * 16 + px;
        if constexpr (GEN) {
          t4 ar = {};
          if constexpr (AUXX)
            ar = *(const t4*)(aux + TL::NZB + q * 32 + ((((lrow >> 1) ^ (q >> 3)) & 1) << 4) +
                              ((lrow & 1) << 3));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[i + u][e];
            if constexpr (G_BIAS) v += c0[e];
            if constexpr (G_MASK) v = (float)ar[e] > 0.f ? v : (G_MSL ? c0[e] * v : 0.f);
            if constexpr (G_RELU) v = v > 0.f ? v : 0.f;
            if constexpr (G_PRELU) v = v > 0.f ? v : c0[e] * v;
            if constexpr (G_ACC) v += (float)ar[e];
            vo[u][e] = v;
          }
        } else if constexpr (FWD) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[i + u][e];
            v += z;
            v += c0[e];
            vo[u][e] = lrelu_s2(v);
          }
        } else {
          const f32x4 c0 = *(const f32x4*)(chl + cle);
          const f32x4 c1 = *(const f32x4*)(chl + 16 + cle);
          const f32x4 c2 = *(const f32x4*)(chl + 32 + cle);
          const t4 xr = *(const t4*)(aux + TL::NZB + q * 32 +
                                     ((((lrow >> 1) ^ (q >> 3)) & 1) << 4) + ((lrow & 1) << 3));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[i + u][e];
            const float xv = (float)xr[e];
            part[e] += v * xv;
            v *= c0[e];
            const float gr = lrelu_s2_grad(xv);
            const float gp = v * gr;
            partq[e] += gp * (xv * lrelu_s2_inv_grad(xv) - z - c2[e]);
            vo[u][e] = gp * c1[e];
          }
        }
      }
      typedef T t2 __attribute__((ext_vector_type(2)));
      unsigned a[2], b[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const t2 ta = {(T)vo[0][2 * h], (T)vo[0][2 * h + 1]};
        const t2 tb = {(T)vo[1][2 * h], (T)vo[1][2 * h + 1]};
        const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, ta),
                                                        __builtin_bit_cast(unsigned, tb), false,
                                                        false);
        a[h] = r[0];
        b[h] = r[1];
      }
      const int m = (n * H + y0 + row0 + i + (lrow & 1)) * W + x0 + px;
      const int c = cw0 + 8 * (lrow >> 1);
      *(uint4*)(Y + (size_t)m * k.ystride + c) = make_uint4(a[0], a[1], b[0], b[1]);
    }
    if constexpr (DG) {
      // the patch's sdot / q partials of this wave's channels: one contributor slot per patch
      // (ordered finish, mia_common.h RedQ)
      const int slt = (y0 / TL::PH) * ptx + x0 / TL::PW;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = row16_sum(part[e]), b = row16_sum(partq[e]);
        if (px == 0) {
          red_put(k, 0, slt, n * Cout + cw0 + cle + e, a);
          red_put(k, 1, slt, n * Cout + cw0 + cle + e, b);
        }
      }
    }
    // block-uniform: the run reaches the next image. Its weights (per-image matrices) and
    // constants are loaded and waited for here, so no wait for them (which would also wait for
    // the next halo, in flight behind them) lands in the next patch's MFMAs. (The VGG launches
    // share their weights and bias over the images.)
    if constexpr (FWD || DG) {
      if (more && n1 != wimg) {
        if constexpr (FWD) load_w(n1);
        load_chan(n1);
        wimg = n1;
        __builtin_amdgcn_s_waitcnt(0x0f70);
      }
    }
    buf ^= 1;
  }
}

template <typename T, int CIN, int EPI, int COUT = 128>
static int launch_wres128_(ConvK& k, hipStream_t st) {
  typedef Wres128Tile<CIN, COUT> TL;
  constexpr bool AUXX = (EPI & (epi::SDOT | epi::MASK | epi::ACC)) != 0;
  constexpr bool DG = (EPI & epi::SDOT) != 0;
  constexpr int LDS = 2 * TL::HBUF + TL::NW * (TL::CHB + TL::NZB + (AUXX ? TL::AXB : 0));
  static_assert(LDS <= 160 * 1024, "LDS budget");
  auto fn = conv_wres128_kernel<T, CIN, EPI, COUT>;
  if (const int rc = ensure_dyn_lds((const void*)fn, LDS); rc != MIA_OK) return rc;
  const int ncu = device_cu_count();
  const int ntiles = k.a.N * (k.a.H / TL::PH) * (k.a.W / TL::PW);
  // Cout = nct column tiles of BN channels, each over the CUs' share of contiguous patch runs
  const int nct = k.a.Cout / TL::BN, share = std::max(1, ncu / nct);
  const int per = (ntiles + share - 1) / share;
  const int grid = nct * ((ntiles + per - 1) / per);  // every block has a non-empty run
  k.prered = 0;
  RedQ r;
  int rc = conv_red_begin(k, r, DG ? (k.a.H / TL::PH) * (k.a.W / TL::PW) : 1, st);
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(TL::NT), LDS, st, k);
  rc = check_launch("conv_wres128");
  return rc != MIA_OK ? rc : red_finish(r, st);
}

// Eligible: 2-byte type, Cin 128 → Cout 128, one group, stride 1, 3×3 pad 1, identity placement,
// H % 8 == 0, W % 16 == 0, dense output rows, and the StyledConv forward epilogue on per-image
// weights (noise, bias, leaky ReLU; mia_conv3x3_wmod), the StyledConv input gradient with the
// style dot and the fused backward front (OSC | SDOT | BAB, shared weights) or a shared-weight
// plain epilogue (GEN); Cin 64 → Cout 128 for the forward BIAS | RELU and PRELU launches.
// T_CONV_WRES128 = 0 disables.
bool conv_wres128_eligible(const ConvK& k, int dtype) {
  if (tune(T_CONV_WRES128) == 0) return false;
  const mia_conv_args& a = k.a;
  const ConvGroup& G = k.g[0];
  using namespace epi;
  if (dtype == MIA_F32 || k.ng != 1 || k.stride != 1 || G.kh != 3 || G.kw != 3 ||
      G.pad_y != 1 || G.pad_x != 1 || G.ho != a.H || G.wo != a.W || G.ay != 1 || G.ax != 1 ||
      G.by != 0 || G.bx != 0 || a.shuffle_out || a.H % 8 != 0 || a.W % 16 != 0 ||
      (a.Cin != 128 && a.Cin != 64) || (a.Cout != 128 && a.Cout != 64 && a.Cout != 256) ||
      k.HT != a.H ||
      k.WT != a.W ||
      a.in_scale || a.act_in != MIA_ACT_NONE || G.kpad < 9 * a.Cin || !a.y ||
      k.ystride != a.Cout || k.ysplit > 0)
    return false;
  const int f = epi_mask(k);
  if (a.Cout == 256)  // (two column tiles: VGG conv3_1 forward, the e4e stage-3 conv1, 64²)
    return k.wn == 0 && ((f == (BIAS | RELU) && a.bias) || (f == PRELU && a.act_slope));
  if (a.Cout == 64)  // (the 128 → 64 launches: VGG conv2_1 / e4e stage-2 input gradients)
    return a.Cin == 128 && k.wn == 0 &&
           (f == 0 || f == ACC || (f == (MASK | MSL) && a.mask_a && a.mask_slope));
  if (a.Cin == 64)  // (the 64 → 128 launches: VGG conv2_1 forward, the e4e stage-2 conv1)
    return k.wn == 0 && ((f == (BIAS | RELU) && a.bias) || (f == PRELU && a.act_slope));
  if (f == (NOISE | BIAS | LRELU)) return a.noise && a.bias && k.wn > 0;
  if (f == (OSC | SDOT | BAB)) return k.wn == 0 && k.cout_mod == a.Cout;
  if (k.wn != 0) return false;
  switch (f) {
    case BIAS | RELU: case BIAS: return a.bias != nullptr;     // VGG conv2_2 / e4e conv2 forward
    case PRELU: return a.act_slope != nullptr;                 // e4e conv1 forward
    case MASK: return a.mask_a != nullptr;                     // VGG input gradient (ReLU mask)
    case MASK | MSL: return a.mask_a && a.mask_slope;          // e4e conv2 input gradient
    case ACC: return true;                                     // e4e conv1 input gradient
    default: return false;
  }
}

int launch_conv_wres128(ConvK& k, int dtype, hipStream_t st) {
  using namespace epi;
  const int f = epi_mask(k);
  MIA_DISPATCH_DTYPE(dtype, T, {
    if constexpr (sizeof(T) == 2) {
      if (k.a.Cout == 64) {
        if (f == 0) return launch_wres128_<T, 128, 0, 64>(k, st);
        if (f == ACC) return launch_wres128_<T, 128, ACC, 64>(k, st);
        if (f == (MASK | MSL)) return launch_wres128_<T, 128, MASK | MSL, 64>(k, st);
        return set_error("conv_wres128: no Cout = 64 specialisation for this launch");
      }
      if (k.a.Cin == 64) {
        if (f == (BIAS | RELU)) return launch_wres128_<T, 64, BIAS | RELU>(k, st);
        if (f == PRELU) return launch_wres128_<T, 64, PRELU>(k, st);
        return set_error("conv_wres128: no Cin = 64 specialisation for this launch");
      }
      if (f == (NOISE | BIAS | LRELU)) return launch_wres128_<T, 128, NOISE | BIAS | LRELU>(k, st);
      if (f == (OSC | SDOT | BAB)) return launch_wres128_<T, 128, OSC | SDOT | BAB>(k, st);
      switch (f) {
        case BIAS | RELU: return launch_wres128_<T, 128, BIAS | RELU>(k, st);
        case BIAS: return launch_wres128_<T, 128, BIAS>(k, st);
        case PRELU: return launch_wres128_<T, 128, PRELU>(k, st);
        case MASK: return launch_wres128_<T, 128, MASK>(k, st);
        case MASK | MSL: return launch_wres128_<T, 128, MASK | MSL>(k, st);
        case ACC: return launch_wres128_<T, 128, ACC>(k, st);
        default: break;
      }
    }
  });
  return set_error("conv_wres128: no specialisation for this launch");
}

}  // namespace mia
