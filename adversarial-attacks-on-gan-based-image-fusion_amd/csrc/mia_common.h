// Shared device/host helpers for libmiattack (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/miattack.h"

namespace mia {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

// 16-byte vector of T: 4 fp32 or 8 fp16/bf16 elements — the unit of every global load/store and
// of every LDS chunk (one ds_read_b128 / ds_write_b128).
template <typename T> struct Vec;
template <> struct Vec<float> { typedef f32x4 type; static constexpr int N = 4; };
template <> struct Vec<_Float16> { typedef f16x8 type; static constexpr int N = 8; };
template <> struct Vec<__bf16> { typedef bf16x8 type; static constexpr int N = 8; };

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(_Float16 v) { return (float)v; }
__device__ __forceinline__ float to_f(__bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ _Float16 from_f<_Float16>(float v) { return (_Float16)v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return (__bf16)v; }

constexpr float SQRT2 = 1.41421356237309504880f;

// FusedLeakyReLU (rosinality op/fused_act): leaky_relu(v, 0.2) * sqrt(2); bias already in v.
__device__ __forceinline__ float lrelu_s2(float v) { return (v > 0.f ? v : 0.2f * v) * SQRT2; }
__device__ __forceinline__ float lrelu_s2_grad(float pre) { return pre > 0.f ? SQRT2 : 0.2f * SQRT2; }
// 1 / lrelu_s2_grad: the pre-activation from a stored activation a = lrelu_s2(pre) is a · this
// (a multiply instead of a fp32 division in the backward-front epilogues)
__device__ __forceinline__ float lrelu_s2_inv_grad(float pre) {
  return pre > 0.f ? 0.70710678118654752f : 3.5355339059327376f;
}

// Sum over each 16-lane row, the same butterfly as v += shfl_xor(v, 1, 2, 4, 8) (pairs, quads,
// halves, rows: each add is own + partner, so every lane ends with the bit-identical value the
// shuffles give) on the DPP crossbar — four VALU adds, no LDS round trips (ds_bpermute + a
// lgkmcnt wait per step, serialised per value).
#define MIA_DPP(v, ctrl) \
  __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, (v)), (ctrl), 0xf, 0xf, false))
// LDS-only hand-off between the waves of a block: this wave's LDS accesses retired
// (lgkmcnt(0)) and the block barrier, WITHOUT the vector-memory fence of __syncthreads() (which
// would also wait for global loads / LDS-DMA in flight). The asm's "memory" clobber makes it a
// compiler barrier too: no LDS store is sunk below it and no LDS load hoisted above it
// (__builtin_amdgcn_s_waitcnt / s_barrier alone do not order the compiler's memory accesses).
__device__ __forceinline__ void lds_handoff() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float row16_sum(float v) {
  v += MIA_DPP(v, 0xB1);   // quad_perm [1,0,3,2]: lane ^ 1
  v += MIA_DPP(v, 0x4E);   // quad_perm [2,3,0,1]: lane ^ 2
  v += MIA_DPP(v, 0x141);  // row_half_mirror: lane i ↔ 7 − i within 8 (the other quad)
  v += MIA_DPP(v, 0x140);  // row_mirror: lane i ↔ 15 − i (the other half-row)
  return v;
}

// Wave-level sum (64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

int set_error(const std::string& msg);
int check_launch(const char* what);

// Per-device launch facts, thread-safe (reduce.hip): the current device's CU count (cached per
// device), and hipFuncSetAttribute(MaxDynamicSharedMemorySize, bytes) applied once per (kernel,
// device) — the launchers' lazy initialisation, safe for several host threads and devices.
int device_cu_count();
int ensure_dyn_lds(const void* fn, int bytes);

// Kernel-variant switches (tests' bitwise A/B comparisons and the tuning tools; the product path
// never changes them): read ONCE from the environment (MIA_<NAME>=value) at first use, then only
// through mia_set_tuning() — no getenv on the launch path. The defaults are the measured-best
// choices.
enum TuneKey {
  T_CONV_HALO,       // 0: the 2-byte stride-1 convs on the generic tile instead of the halo tile
  T_CONV_X6,         // 0: the fp32 convs on the on-the-fly split kernels instead of split-once
  T_HALO_EPI,        // halo tiles' epilogue: 0 LDS-staged, 1 specialised (default), 2 runtime
  T_X6_UNR,          // x6 halo kernel: 0 rolled tap loop, 1 unrolled taps, 2 (default) + two
                     // taps per K-step on the 64-column tile
  T_CONV_THIN,       // 0: no thin-channel input-layer kernels
  T_CONV_THIN32,     // 0: no 32-channel thin kernel
  T_CONV_WRES,       // 0: no weights-resident 64 → 64 kernel
  T_CONV_REGEPI,     // 0: no register epilogue on the generic 128×128 tile
  T_CONV_SMALLTILE,  // 64×64 generic tiles below this many 128×128 tiles (2-byte types)
  T_S2DG_X6,         // 0: the stride-2 input gradients on the on-the-fly split up-conv kernel
  T_S2DG_HALO,       // 0: the stride-2 input gradients as 4 sub-pixel phase GEMMs
  T_UPCONV_X6,       // 0: the fp32 up-conv forward on the on-the-fly split kernel
  T_UPCONV_HALO,     // 0: the up-conv forward as 4 sub-pixel phase GEMMs
  T_CONV_WRES32,     // 0: the 32 → 32 layers on the global-gather kernel (conv_thin32)
  T_HALO_C64,        // Cout = 64 (2-byte types) on the 64-channel halo tile: 1 (default), 0 never
  T_X6_64S,          // fp32 Cout = 64: 1 (default) the two-blocks-per-CU x6 tile (conv_halo_x6.hip
                     // HaloX6S, also the VGG tap-pair gradient), 0 the 8-wave 64-column tile
  T_UPCONV_X6S,      // fp32 split-once stride-2 input gradient with Cin ≤ 512: 1 (default) the
                     // 8 × 16-patch two-blocks-per-CU form (conv_upconv.hip DgX6S), 0 the 8-wave one
  T_CONV_WRES128,    // 0: the 2-byte 128 → 128 StyledConv forward on per-image weights on the
                     // halo tile instead of the weights-resident kernel (conv_wres128.hip)
  T_NKEYS
};
int tune(TuneKey key);

// ---- deterministic reductions (reduce.hip) ---------------------------------------------------
// Per-(image, channel) sums that many blocks contribute to (the StyledConv style gradient sdot,
// the backward front's q, the channel sums, per-image losses) never use float atomics: every
// contributor stores its partial into its own SLOT of a partial buffer, and red_finish adds the
// slots of each output IN SLOT ORDER after the launch. The result is bit-identical run to run,
// and an image's sums do not depend on which other images share the launch. Partial layout:
// part[(q·nslots + slot)·count + i] for quantity q (up to 3 per launch), output i < count.
struct RedQ {
  float* dst[3];     // outputs (+= the ordered slot sum); nullptr = quantity absent
  float* part;       // partial buffer (library scratch of this stream, red_scratch)
  int nslots, count; // slots per output, outputs per quantity
};
// library-owned device scratch of at least `bytes` for `st` (grown on demand, kept per stream;
// growth synchronises the stream before releasing the old buffer)
float* red_scratch(hipStream_t st, size_t bytes);
// partial buffer for the quantities of dst[] (nslots × count each); zero = clear it first (for
// launches in which some slots may have no contributor). Returns MIA_OK or an error code.
int red_begin(RedQ& r, float* d0, float* d1, float* d2, int nslots, int count, hipStream_t st,
              bool zero = false);
// dst_q[i] += Σ_{slot = 0 … nslots−1} part[q][slot][i] in a fixed order that depends on nslots
// only (slot order; beyond 128 slots the in-order sums of 64-slot chunks, added in chunk order)
int red_finish(const RedQ& r, hipStream_t st);

__device__ __forceinline__ void red_store(float* part, int nslots, int count, int q, int slot,
                                          int i, float v) {
  part[((size_t)q * nslots + slot) * count + i] = v;
}

}  // namespace mia

#define MIA_DISPATCH_DTYPE(dtype, T, ...)                                   \
  switch (dtype) {                                                          \
    case MIA_F32: { typedef float T; __VA_ARGS__; break; }                  \
    case MIA_F16: { typedef _Float16 T; __VA_ARGS__; break; }               \
    case MIA_BF16: { typedef __bf16 T; __VA_ARGS__; break; }                \
    default: return mia::set_error("unsupported dtype");                    \
  }

#define MIA_CHECK_ARG(cond, msg) \
  do { if (!(cond)) return mia::set_error(std::string(__func__) + ": " + (msg)); } while (0)
