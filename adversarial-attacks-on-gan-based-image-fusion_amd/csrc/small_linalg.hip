// Small fp32 linear algebra of the attack step (K6 style affines, demodulation coefficients, the
// synthetic encoder): a strided LDS-tiled SGEMM and two fused demod kernels. All of it is
// < 1 GFLOP per step at N = 128, so simplicity wins over MFMA here.
#include <algorithm>
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

// ---- grouped multi-segment SGEMM ----------------------------------------------------------
// One launch computes up to kMaxGroups independent products
//   C_g = alpha_g · Σ_seg A_seg·B_seg + beta_g · C_g + bias_g
// (a group with two segments sums two K-ranges from different operands — e.g. the two layers that
// share one W+ latent row in the style-affine backward). Every block owns one TM×TM tile of one
// group; TM = 64 (4×4 per thread) or 32 (2×2 per thread) is picked on the host so that a launch
// has enough blocks to cover the 256 CUs (the attack's GEMMs have M = batch ≤ 128).
constexpr int GK = 32;
constexpr int kMaxGroups = 12;

struct GemmSeg {
  const float* A;
  const float* B;
  int64_t sam, sak, sbk, sbn;
  int K;
};
struct GemmGroup {
  float* C;
  const float* bias;
  int64_t scm, scn;
  int M, N;
  float alpha, beta;
  int nseg, tile0, ntn;
  GemmSeg seg[2];
};
struct GemmBatch {
  int ng;
  GemmGroup g[kMaxGroups];
};

// The K loop is software-pipelined: the operand elements of K-step s+1 are loaded into
// registers before the FMAs of step s, so each step waits on one LDS round trip, not on a
// global-load latency (the style GEMMs have K = 512 … 1024 and only a few tiles per group).
template <int TM>
__global__ __launch_bounds__(256) void sgemm_grouped_kernel(const GemmBatch b) {
  constexpr int R = TM / 16;         // per-thread micro-tile R×R
  constexpr int EPT = GK * TM / 256;  // operand elements per thread per K-step
  __shared__ float As[GK][TM + 1];
  __shared__ float Bs[GK][TM + 1];
  int gi = 0;
#pragma unroll 1
  for (int i = 1; i < b.ng; ++i)
    if ((int)blockIdx.x >= b.g[i].tile0) gi = i;
  const GemmGroup& G = b.g[gi];
  const int t = blockIdx.x - G.tile0;
  const int m0 = (t / G.ntn) * TM, n0 = (t % G.ntn) * TM;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[R][R] = {};
  const int steps0 = (G.seg[0].K + GK - 1) / GK;
  const int nsteps = steps0 + (G.nseg > 1 ? (G.seg[1].K + GK - 1) / GK : 0);
  float ra[EPT], rb[EPT];
  // consecutive threads walk the operand's contiguous dimension (coalesced loads)
  auto load = [&](int s) {
    const GemmSeg& S = s < steps0 ? G.seg[0] : G.seg[1];
    const int k0 = (s < steps0 ? s : s - steps0) * GK;
    const bool a_kfast = S.sak == 1, b_kfast = S.sbk == 1;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int i = threadIdx.x + e * 256;
      int kk = a_kfast ? i % GK : i / TM, mm = a_kfast ? i / GK : i % TM;
      int gm = m0 + mm, gk = k0 + kk;
      ra[e] = (gm < G.M && gk < S.K) ? S.A[gm * S.sam + gk * S.sak] : 0.f;
      kk = b_kfast ? i % GK : i / TM;
      const int nn = b_kfast ? i / GK : i % TM;
      const int gn = n0 + nn;
      gk = k0 + kk;
      rb[e] = (gn < G.N && gk < S.K) ? S.B[gk * S.sbk + gn * S.sbn] : 0.f;
    }
  };
  auto store = [&](int s) {
    const GemmSeg& S = s < steps0 ? G.seg[0] : G.seg[1];
    const bool a_kfast = S.sak == 1, b_kfast = S.sbk == 1;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int i = threadIdx.x + e * 256;
      As[a_kfast ? i % GK : i / TM][a_kfast ? i / GK : i % TM] = ra[e];
      Bs[b_kfast ? i % GK : i / TM][b_kfast ? i / GK : i % TM] = rb[e];
    }
  };
  load(0);
#pragma unroll 1
  for (int s = 0; s < nsteps; ++s) {
    store(s);
    __syncthreads();
    if (s + 1 < nsteps) load(s + 1);
#pragma unroll
    for (int kk = 0; kk < GK; ++kk) {
      float a[R], bb[R];
#pragma unroll
      for (int i = 0; i < R; ++i) a[i] = As[kk][ty * R + i];
#pragma unroll
      for (int j = 0; j < R; ++j) bb[j] = Bs[kk][tx * R + j];
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) acc[i][j] += a[i] * bb[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int gm = m0 + ty * R + i, gn = n0 + tx * R + j;
      if (gm < G.M && gn < G.N) {
        float v = G.alpha * acc[i][j];
        if (G.beta != 0.f) v += G.beta * G.C[gm * G.scm + gn * G.scn];
        if (G.bias) v += G.bias[gn];
        G.C[gm * G.scm + gn * G.scn] = v;
      }
    }
}

// y[n][d] = Σ_s x[n][s][d]  (e4e: the latent gradient rows that all read style 0)
__global__ __launch_bounds__(256) void sum_slices_kernel(const float* __restrict__ x, float* y,
                                                         int S, int D, int64_t total) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t n = i / D;
    const int d = (int)(i - n * D);
    const float* p = x + n * S * D + d;
    float a = 0.f;
    for (int s = 0; s < S; ++s) a += p[(int64_t)s * D];
    y[i] = a;
  }
}

static int run_gemm_groups(const mia_gemm_group* groups, int ngroups, hipStream_t st) {
  int64_t tiles64 = 0;
  for (int i = 0; i < ngroups; ++i) {
    const mia_gemm_group& q = groups[i];
    tiles64 += (int64_t)((q.M + 63) / 64) * ((q.N + 63) / 64);
  }
  const int TM = tiles64 >= 512 ? 64 : 32;  // ≥ 2 blocks per CU either way
  for (int base = 0; base < ngroups; base += kMaxGroups) {
    GemmBatch b{};
    b.ng = std::min(kMaxGroups, ngroups - base);
    int tiles = 0;
    for (int i = 0; i < b.ng; ++i) {
      const mia_gemm_group& q = groups[base + i];
      if (!q.C || q.M <= 0 || q.N <= 0 || q.nseg < 1 || q.nseg > 2)
        return set_error("gemm: bad group (C, M, N > 0 and 1 ≤ nseg ≤ 2 required)");
      GemmGroup& g = b.g[i];
      g.C = q.C; g.bias = q.bias; g.scm = q.scm; g.scn = q.scn; g.M = q.M; g.N = q.N;
      g.alpha = q.alpha; g.beta = q.beta; g.nseg = q.nseg;
      for (int s = 0; s < q.nseg; ++s) {
        const mia_gemm_seg& qs = q.seg[s];
        if (!qs.A || !qs.B || qs.K <= 0) return set_error("gemm: bad segment (A, B, K > 0)");
        g.seg[s] = GemmSeg{qs.A, qs.B, qs.sam, qs.sak, qs.sbk, qs.sbn, qs.K};
      }
      g.ntn = (q.N + TM - 1) / TM;
      g.tile0 = tiles;
      tiles += ((q.M + TM - 1) / TM) * g.ntn;
    }
    if (TM == 64)
      hipLaunchKernelGGL(sgemm_grouped_kernel<64>, dim3(tiles), dim3(256), 0, st, b);
    else
      hipLaunchKernelGGL(sgemm_grouped_kernel<32>, dim3(tiles), dim3(256), 0, st, b);
    const int rc = check_launch("sgemm_grouped");
    if (rc) return rc;
  }
  return MIA_OK;
}

// demod[n][co] = rsqrt(scale2·Σ_ci s²·wsq[co][ci] + 1e-8). One wave per (n, co): its lanes read
// the weight row coalesced (ci = lane + 64·k, summed in k order), then a fixed butterfly
// (wave_sum); 4 output channels per block share the block's s² row in LDS.
__global__ __launch_bounds__(256) void style_demod_kernel(const float* __restrict__ s,
                                                          const float* __restrict__ wsq,
                                                          float* __restrict__ demod, int Cin,
                                                          int Cout, float scale2) {
  extern __shared__ float s2[];
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < Cin; i += blockDim.x) {
    const float v = s[(size_t)n * Cin + i];
    s2[i] = v * v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, co = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (co >= Cout) return;
  const float* w = wsq + (size_t)co * Cin;
  float acc = 0.f;
  int ci = lane;
  for (; ci + 7 * 64 < Cin; ci += 8 * 64) {  // the row loads 8 ahead of the in-order FMAs
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = w[ci + 64 * u];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_fmaf(s2[ci + 64 * u], t[u], acc);
  }
  for (; ci < Cin; ci += 64) acc = __builtin_fmaf(s2[ci], w[ci], acc);
  acc = wave_sum(acc);
  if (lane == 0) demod[(size_t)n * Cout + co] = rsqrtf(scale2 * acc + 1e-8f);
}

// gs[n][ci] += −scale2·s[n][ci]·Σ_co q[n][co]·demod[n][co]²·wsq[co][ci]. A block owns 64 input
// channels of one image; its 4 waves sum a quarter of the output channels each (rows coalesced
// over ci), then the quarters are added in order: a fixed order, 4× the parallelism and a quarter
// of the serial chain of one thread per (n, ci).
__global__ __launch_bounds__(256) void demod_bwd_kernel(const float* __restrict__ q,
                                                        const float* __restrict__ demod,
                                                        const float* __restrict__ wsq,
                                                        const float* __restrict__ s,
                                                        float* __restrict__ gs, int Cin, int Cout,
                                                        float scale2) {
  extern __shared__ float r[];  // [Cout] q·demod², then [4][64] partial sums
  float* const part = r + Cout;
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < Cout; i += blockDim.x) {
    const float d = demod[(size_t)n * Cout + i];
    r[i] = q[(size_t)n * Cout + i] * d * d;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, qtr = threadIdx.x >> 6;
  const int ci = blockIdx.x * 64 + lane;
  const int per = (Cout + 3) / 4, c0 = qtr * per, c1 = min(c0 + per, Cout);
  float acc = 0.f;
  if (ci < Cin) {
    // the weight loads in batches of 8 ahead of their (in-order) FMAs: one L2 round trip per batch
    // instead of one per output channel (same sum order, bit-identical)
    int co = c0;
    for (; co + 8 <= c1; co += 8) {
      float w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = wsq[(size_t)(co + u) * Cin + ci];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = __builtin_fmaf(r[co + u], w[u], acc);  // fused, as before
    }
    for (; co < c1; ++co) acc += r[co] * wsq[(size_t)co * Cin + ci];
  }
  part[qtr * 64 + lane] = acc;
  __syncthreads();
  if (qtr == 0 && ci < Cin) {
    const float t = ((part[lane] + part[64 + lane]) + part[128 + lane]) + part[192 + lane];
    gs[(size_t)n * Cin + ci] += -scale2 * s[(size_t)n * Cin + ci] * t;
  }
}

}  // namespace mia

using namespace mia;

extern "C" int mia_version(void) { return 1; }

extern "C" const char* mia_last_error_string(void) { return g_last_error.c_str(); }

extern "C" int mia_gemm_f32(int M, int Nn, int K, float alpha, const float* A, int64_t sam,
                            int64_t sak, const float* B, int64_t sbk, int64_t sbn, float beta,
                            float* C, int64_t scm, int64_t scn, const float* bias, void* stream) {
  MIA_CHECK_ARG(A && B && C && M > 0 && Nn > 0 && K > 0, "bad args");
  mia_gemm_group g{};
  g.C = C; g.bias = bias; g.scm = scm; g.scn = scn; g.M = M; g.N = Nn;
  g.alpha = alpha; g.beta = beta; g.nseg = 1;
  g.seg[0] = mia_gemm_seg{A, B, sam, sak, sbk, sbn, K};
  return run_gemm_groups(&g, 1, (hipStream_t)stream);
}

extern "C" int mia_gemm_f32_grouped(const mia_gemm_group* groups, int ngroups, void* stream) {
  MIA_CHECK_ARG(groups && ngroups > 0, "bad args");
  return run_gemm_groups(groups, ngroups, (hipStream_t)stream);
}

extern "C" int mia_style_demod(const float* s, const float* wsq, float* demod, int N, int Cin,
                               int Cout, float scale2, void* stream) {
  MIA_CHECK_ARG(s && wsq && demod && N > 0 && Cin > 0 && Cout > 0, "bad args");
  dim3 grid((Cout + 3) / 4, N);
  hipLaunchKernelGGL(style_demod_kernel, grid, dim3(256), Cin * sizeof(float), (hipStream_t)stream,
                     s, wsq, demod, Cin, Cout, scale2);
  return check_launch("style_demod");
}

extern "C" int mia_demod_bwd(const float* q, const float* demod, const float* wsq, const float* s,
                             float* gs, int N, int Cin, int Cout, float scale2, void* stream) {
  MIA_CHECK_ARG(q && demod && wsq && s && gs && N > 0, "bad args");
  dim3 grid((Cin + 63) / 64, N);
  hipLaunchKernelGGL(demod_bwd_kernel, grid, dim3(256), (Cout + 256) * sizeof(float),
                     (hipStream_t)stream,
                     q, demod, wsq, s, gs, Cin, Cout, scale2);
  return check_launch("demod_bwd");
}

extern "C" int mia_sum_slices(const float* x, float* y, int N, int S, int D, void* stream) {
  MIA_CHECK_ARG(x && y && N > 0 && S > 0 && D > 0, "bad args");
  const int64_t total = (int64_t)N * D;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(sum_slices_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, y, S, D,
                     total);
  return check_launch("sum_slices");
}
