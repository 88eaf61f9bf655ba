// Deterministic reductions (mia_common.h, RedQ): library-owned partial buffers per stream and the
// ordered finish. Replaces float atomics across blocks wherever several blocks add into one
// per-(image, channel) sum: with atomics the summation order — and so the fp32 result — changed
// run to run (SURVEY.md §5 asks for bit-identical reruns; the reference runs with
// cudnn.deterministic, code/attack/interpolation.py:195-200).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "mia_common.h"

namespace mia {

namespace {
struct Scratch {
  float* p = nullptr;
  size_t bytes = 0;
};
std::mutex g_mu;
std::unordered_map<hipStream_t, Scratch> g_scratch;
}  // namespace

// ---- kernel-variant switches (mia_common.h TuneKey) ------------------------------------------
namespace {
struct TuneDef {
  const char* name;
  int value;
};
TuneDef g_tune[T_NKEYS] = {
    {"MIA_CONV_HALO", 1}, {"MIA_CONV_X6", 1},       {"MIA_HALO_EPI", 1},    {"MIA_X6_UNR", 2},
    {"MIA_CONV_THIN", 1}, {"MIA_CONV_THIN32", 1},   {"MIA_CONV_WRES", 1},
    {"MIA_CONV_REGEPI", 1},   {"MIA_CONV_SMALLTILE", 512},
    {"MIA_S2DG_X6", 1},   {"MIA_S2DG_HALO", 1},     {"MIA_UPCONV_X6", 1},   {"MIA_UPCONV_HALO", 1},
    {"MIA_CONV_WRES32", 1},
    {"MIA_HALO_C64", 1},  {"MIA_X6_64S", 1},
    {"MIA_UPCONV_X6S", 1}, {"MIA_CONV_WRES128", 1}};
std::once_flag g_tune_once;
void tune_init() {
  for (auto& d : g_tune) {
    const char* e = getenv(d.name);
    if (e && *e) d.value = atoi(e);
  }
}
}  // namespace

int tune(TuneKey key) {
  std::call_once(g_tune_once, tune_init);
  return g_tune[key].value;
}

namespace {
std::mutex g_dev_mu;
std::unordered_map<int, int> g_ncu;                           // device → CU count
std::unordered_map<const void*, std::vector<int>> g_lds_set;  // kernel → devices configured
int current_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return dev;
}
}  // namespace

int device_cu_count() {
  const int dev = current_device();
  std::lock_guard<std::mutex> lock(g_dev_mu);
  auto it = g_ncu.find(dev);
  if (it != g_ncu.end()) return it->second;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    ncu = 256;  // MI355X
  g_ncu[dev] = ncu;
  return ncu;
}

int ensure_dyn_lds(const void* fn, int bytes) {
  const int dev = current_device();
  std::lock_guard<std::mutex> lock(g_dev_mu);
  std::vector<int>& done = g_lds_set[fn];
  if (std::find(done.begin(), done.end(), dev) != done.end()) return MIA_OK;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
    return set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  done.push_back(dev);
  return MIA_OK;
}

float* red_scratch(hipStream_t st, size_t bytes) {
  std::lock_guard<std::mutex> lock(g_mu);
  Scratch& s = g_scratch[st];
  if (s.bytes >= bytes) return s.p;
  if (s.p) {  // kernels queued on this stream may still read / write the old buffer
    if (hipStreamSynchronize(st) != hipSuccess || hipFree(s.p) != hipSuccess) return nullptr;
    s.p = nullptr;
    s.bytes = 0;
  }
  // grow geometrically: the partial footprint of a step varies per layer
  size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
  want = want + want / 4;
  void* p = nullptr;
  if (hipMalloc(&p, want) != hipSuccess) return nullptr;
  s.p = (float*)p;
  s.bytes = want;
  return s.p;
}

// Slots are summed in chunks of RED_CHUNK (in slot order within a chunk, then the chunk sums in
// chunk order): a fixed tree that depends on nslots only, so the result stays bit-reproducible
// and independent of the other images of the call; one finishing thread per output walking
// 16 K slots serially took milliseconds (the 512² / 1024² layers' per-row-segment slots).
constexpr int RED_CHUNK = 64;
static inline int red_nchunks(int nslots) { return nslots <= 2 * RED_CHUNK ? 1 : (nslots + RED_CHUNK - 1) / RED_CHUNK; }

int red_begin(RedQ& r, float* d0, float* d1, float* d2, int nslots, int count, hipStream_t st,
              bool zero) {
  r.dst[0] = d0;
  r.dst[1] = d1;
  r.dst[2] = d2;
  r.nslots = nslots;
  r.count = count;
  r.part = nullptr;
  if (!d0 && !d1 && !d2) return MIA_OK;
  if (nslots < 1 || count < 1) return set_error("red_begin: empty reduction");
  const int nch = red_nchunks(nslots);
  const size_t part_bytes = (size_t)3 * nslots * count * sizeof(float);
  const size_t bytes = part_bytes + (nch > 1 ? (size_t)3 * nch * count * sizeof(float) : 0);
  r.part = red_scratch(st, bytes);
  if (!r.part) return set_error("red_begin: scratch allocation failed");
  if (zero && hipMemsetAsync(r.part, 0, part_bytes, st) != hipSuccess)
    return set_error("red_begin: memset failed");
  return MIA_OK;
}

// Σ_{k<n} src[k·stride] added in k order, the loads issued 8 ahead of their adds (one memory
// round trip per 8 slots instead of per slot; bit-identical to the plain loop)
__device__ __forceinline__ float ordered_sum(const float* __restrict__ src, int n, int stride) {
  float s = 0.f;
  int k = 0;
  for (; k + 8 <= n; k += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = src[(size_t)(k + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += t[u];
  }
  for (; k < n; ++k) s += src[(size_t)k * stride];
  return s;
}

__global__ __launch_bounds__(256) void red_finish_kernel(const float* __restrict__ part,
                                                         float* d0, float* d1, float* d2,
                                                         int nslots, int count) {
  const int q = blockIdx.y;
  float* dst = q == 0 ? d0 : (q == 1 ? d1 : d2);
  if (!dst) return;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  const float* src = part + (size_t)q * nslots * count + i;
  dst[i] += ordered_sum(src, nslots, count);
}

// chunk c of quantity q: tmp[q][c][i] = Σ_{slot in chunk c} part[q][slot][i], in slot order
__global__ __launch_bounds__(256) void red_chunk_kernel(const float* __restrict__ part,
                                                        float* __restrict__ tmp, int has0,
                                                        int has1, int has2, int nslots,
                                                        int count) {
  const int q = blockIdx.z, c = blockIdx.y;
  if (!(q == 0 ? has0 : (q == 1 ? has1 : has2))) return;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  const int k0 = c * RED_CHUNK, k1 = min(k0 + RED_CHUNK, nslots);
  const float* src = part + ((size_t)q * nslots + k0) * count + i;
  tmp[((size_t)q * gridDim.y + c) * count + i] = ordered_sum(src, k1 - k0, count);
}

int red_finish(const RedQ& r, hipStream_t st) {
  if (!r.part) return MIA_OK;
  const int nch = red_nchunks(r.nslots);
  if (nch == 1) {
    hipLaunchKernelGGL(red_finish_kernel, dim3((r.count + 255) / 256, 3), dim3(256), 0, st,
                       r.part, r.dst[0], r.dst[1], r.dst[2], r.nslots, r.count);
    return check_launch("red_finish");
  }
  float* tmp = r.part + (size_t)3 * r.nslots * r.count;
  hipLaunchKernelGGL(red_chunk_kernel, dim3((r.count + 255) / 256, nch, 3), dim3(256), 0, st,
                     r.part, tmp, r.dst[0] != nullptr, r.dst[1] != nullptr, r.dst[2] != nullptr,
                     r.nslots, r.count);
  int rc = check_launch("red_chunk");
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(red_finish_kernel, dim3((r.count + 255) / 256, 3), dim3(256), 0, st, tmp,
                     r.dst[0], r.dst[1], r.dst[2], nch, r.count);
  return check_launch("red_finish");
}

}  // namespace mia

using namespace mia;

// Slots per output: a register-epilogue contributor covers ≥ 16 pixels (one 16-column row
// segment), the thin32 kernel's at most H·W/16 + 2 waves meet one image; only the LDS-staged
// epilogue on images that are not whole tiles (H·W not a multiple of the tile rows) falls back to
// one slot per pixel. The scratch always holds 3 quantities' slots (sdot, bab_q, csum).
extern "C" int64_t mia_conv_workspace_size(int N, int H_out, int W_out, int Cout, int has_sums) {
  if (!has_sums || N <= 0 || H_out <= 0 || W_out <= 0 || Cout <= 0) return 0;
  const int64_t hw = (int64_t)H_out * W_out;
  const int64_t slots = hw % 256 == 0 ? hw / 16 + 2 : hw + 2;
  const int64_t chunks = slots <= 2 * RED_CHUNK ? 0 : (slots + RED_CHUNK - 1) / RED_CHUNK;
  return (int64_t)3 * (slots + chunks) * N * Cout * (int64_t)sizeof(float);
}

// pointwise reductions: one slot per block of ≥ 16 pixels (bias_act / torgb: 16 pixel passes of
// ≥ 1 pixel; chan_dot: ≤ 32 chunks; mse_sum: ≤ 1024 blocks of 256 elements)
extern "C" int64_t mia_reduction_workspace_size(int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0) return 0;
  const int64_t slots = std::max<int64_t>(1024, HW);
  const int64_t chunks = (slots + RED_CHUNK - 1) / RED_CHUNK;
  return (int64_t)3 * (slots + chunks) * N * C * (int64_t)sizeof(float);
}

extern "C" int mia_reserve_reduction_scratch(int64_t bytes, void* stream) {
  MIA_CHECK_ARG(bytes >= 0, "bytes must be >= 0");
  if (bytes == 0) return MIA_OK;
  return red_scratch((hipStream_t)stream, (size_t)bytes) ? MIA_OK
                                                         : set_error("scratch allocation failed");
}

extern "C" int64_t mia_reduction_scratch_bytes(void* stream) {
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_scratch.find((hipStream_t)stream);
  return it == g_scratch.end() ? 0 : (int64_t)it->second.bytes;
}

extern "C" int mia_release_reduction_scratch(void* stream) {
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_scratch.find((hipStream_t)stream);
  if (it == g_scratch.end()) return MIA_OK;
  if (it->second.p) {
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess || hipFree(it->second.p) != hipSuccess)
      return set_error("scratch release failed");
  }
  g_scratch.erase(it);
  return MIA_OK;
}

extern "C" int mia_set_tuning(const char* name, int value) {
  std::call_once(g_tune_once, tune_init);
  MIA_CHECK_ARG(name != nullptr, "null name");
  for (auto& d : g_tune)
    if (strcmp(d.name, name) == 0) {
      d.value = value;
      return MIA_OK;
    }
  return set_error(std::string("unknown tuning switch ") + name);
}

extern "C" int mia_get_tuning(const char* name, int* value) {
  std::call_once(g_tune_once, tune_init);
  MIA_CHECK_ARG(name != nullptr && value != nullptr, "null argument");
  for (auto& d : g_tune)
    if (strcmp(d.name, name) == 0) {
      *value = d.value;
      return MIA_OK;
    }
  return set_error(std::string("unknown tuning switch ") + name);
}
