// Small fp32 linear algebra of the attack step (K6 style affines, demodulation coefficients, the
// synthetic encoder): a strided LDS-tiled SGEMM and two fused demod kernels. All of it is
// < 1 GFLOP per step at N = 128, so simplicity wins over MFMA here.
#include <string>

#include "mia_common.h"

namespace mia {

thread_local std::string g_last_error;

int set_error(const std::string& msg) {
  g_last_error = msg;
  return MIA_EINVAL;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return MIA_ELAUNCH;
  }
  return MIA_OK;
}

constexpr int GT = 64, GK = 16;

__global__ __launch_bounds__(256) void sgemm_kernel(int M, int Nn, int K, float alpha,
                                                     const float* __restrict__ A, int64_t sam,
                                                     int64_t sak, const float* __restrict__ B,
                                                     int64_t sbk, int64_t sbn, float beta,
                                                     float* __restrict__ C, int64_t scm,
                                                     int64_t scn, const float* __restrict__ bias) {
  __shared__ float As[GK][GT + 1];
  __shared__ float Bs[GK][GT + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
  const bool a_kfast = sak == 1, b_kfast = sbk == 1;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += GK) {
    // consecutive threads walk the operand's contiguous dimension (coalesced loads)
    for (int i = threadIdx.x; i < GK * GT; i += 256) {
      const int kk = a_kfast ? i % GK : i / GT, mm = a_kfast ? i / GK : i % GT;
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? A[gm * sam + gk * sak] : 0.f;
    }
    for (int i = threadIdx.x; i < GK * GT; i += 256) {
      const int kk = b_kfast ? i % GK : i / GT, nn = b_kfast ? i / GK : i % GT;
      const int gn = n0 + nn, gk = k0 + kk;
      Bs[kk][nn] = (gn < Nn && gk < K) ? B[gk * sbk + gn * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gm = m0 + ty * 4 + i, gn = n0 + tx * 4 + j;
      if (gm < M && gn < Nn) {
        float v = alpha * acc[i][j];
        if (beta != 0.f) v += beta * C[gm * scm + gn * scn];
        if (bias) v += bias[gn];
        C[gm * scm + gn * scn] = v;
      }
    }
}

// demod[n][co] = rsqrt(scale2·Σ_ci s²·wsq[co][ci] + 1e-8); one thread per (n, co).
__global__ void style_demod_kernel(const float* __restrict__ s, const float* __restrict__ wsq,
                                   float* __restrict__ demod, int Cin, int Cout, float scale2) {
  extern __shared__ float s2[];
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < Cin; i += blockDim.x) {
    const float v = s[(size_t)n * Cin + i];
    s2[i] = v * v;
  }
  __syncthreads();
  const int co = blockIdx.x * blockDim.x + threadIdx.x;
  if (co >= Cout) return;
  const float* w = wsq + (size_t)co * Cin;
  float acc = 0.f;
  for (int ci = 0; ci < Cin; ++ci) acc += s2[ci] * w[ci];
  demod[(size_t)n * Cout + co] = rsqrtf(scale2 * acc + 1e-8f);
}

// gs[n][ci] += −scale2·s[n][ci]·Σ_co q[n][co]·demod[n][co]²·wsq[co][ci]
__global__ void demod_bwd_kernel(const float* __restrict__ q, const float* __restrict__ demod,
                                 const float* __restrict__ wsq, const float* __restrict__ s,
                                 float* __restrict__ gs, int Cin, int Cout, float scale2) {
  extern __shared__ float r[];
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < Cout; i += blockDim.x) {
    const float d = demod[(size_t)n * Cout + i];
    r[i] = q[(size_t)n * Cout + i] * d * d;
  }
  __syncthreads();
  const int ci = blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= Cin) return;
  float acc = 0.f;
  for (int co = 0; co < Cout; ++co) acc += r[co] * wsq[(size_t)co * Cin + ci];
  gs[(size_t)n * Cin + ci] += -scale2 * s[(size_t)n * Cin + ci] * acc;
}

}  // namespace mia

using namespace mia;

extern "C" int mia_version(void) { return 1; }

extern "C" const char* mia_last_error_string(void) { return g_last_error.c_str(); }

extern "C" int mia_gemm_f32(int M, int Nn, int K, float alpha, const float* A, int64_t sam,
                            int64_t sak, const float* B, int64_t sbk, int64_t sbn, float beta,
                            float* C, int64_t scm, int64_t scn, const float* bias, void* stream) {
  MIA_CHECK_ARG(A && B && C && M > 0 && Nn > 0 && K > 0, "bad args");
  dim3 grid((Nn + GT - 1) / GT, (M + GT - 1) / GT);
  hipLaunchKernelGGL(sgemm_kernel, grid, dim3(256), 0, (hipStream_t)stream, M, Nn, K, alpha, A,
                     sam, sak, B, sbk, sbn, beta, C, scm, scn, bias);
  return check_launch("sgemm");
}

extern "C" int mia_style_demod(const float* s, const float* wsq, float* demod, int N, int Cin,
                               int Cout, float scale2, void* stream) {
  MIA_CHECK_ARG(s && wsq && demod && N > 0 && Cin > 0 && Cout > 0, "bad args");
  dim3 grid((Cout + 255) / 256, N);
  hipLaunchKernelGGL(style_demod_kernel, grid, dim3(256), Cin * sizeof(float), (hipStream_t)stream,
                     s, wsq, demod, Cin, Cout, scale2);
  return check_launch("style_demod");
}

extern "C" int mia_demod_bwd(const float* q, const float* demod, const float* wsq, const float* s,
                             float* gs, int N, int Cin, int Cout, float scale2, void* stream) {
  MIA_CHECK_ARG(q && demod && wsq && s && gs && N > 0, "bad args");
  dim3 grid((Cin + 255) / 256, N);
  hipLaunchKernelGGL(demod_bwd_kernel, grid, dim3(256), Cout * sizeof(float), (hipStream_t)stream,
                     q, demod, wsq, s, gs, Cin, Cout, scale2);
  return check_launch("demod_bwd");
}
