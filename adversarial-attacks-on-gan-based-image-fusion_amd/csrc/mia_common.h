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

// Wave-level sum (64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

int set_error(const std::string& msg);
int check_launch(const char* what);

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
