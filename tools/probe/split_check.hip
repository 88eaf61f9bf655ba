// Probe: one wave, D = A·B for a 16×16×16 fp32 block through mfma_chunk<float> (the bf16 split
// path) vs a host fp64 reference; also the native f32 MFMA for comparison.
#include <cstdio>
#include <cmath>
#include <vector>
#include "../../adversarial-attacks-on-gan-based-image-fusion_amd/csrc/conv_common.h"
using namespace mia;
__global__ void k_split(const float* A, const float* B, float* D, int native) {
  const int lane = threadIdx.x, row = lane & 15, q = lane >> 4;
  f32x4 a, b;
  for (int e = 0; e < 4; ++e) { a[e] = A[row * 16 + 4 * q + e]; b[e] = B[(4 * q + e) * 16 + row]; }
  f32x4 c = {0, 0, 0, 0};
  if (native) {
    for (int e = 0; e < 4; ++e) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[e], c, 0, 0, 0);
  } else {
    c = mfma_chunk<float>(a, b, c);
  }
  // D[row i][col j]: lane (j = lane & 15) holds rows 4q..4q+3
  for (int r = 0; r < 4; ++r) D[(4 * q + r) * 16 + row] = c[r];
}
namespace mia { int set_error(const std::string&) { return 1; } int check_launch(const char*) { return 0; } }
int main() {
  std::vector<float> A(256), B(256), D(256);
  unsigned s = 1;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) / 16777216.f) * 2.f - 1.f; };
  for (auto& v : A) v = rnd();
  for (auto& v : B) v = rnd();
  float *dA, *dB, *dD;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 1024);
  hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
  for (int native = 0; native < 2; ++native) {
    hipLaunchKernelGGL(k_split, dim3(1), dim3(64), 0, 0, dA, dB, dD, native);
    hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
    double mx = 0, mref = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double r = 0;
        for (int k = 0; k < 16; ++k) r += (double)A[i * 16 + k] * B[k * 16 + j];
        mx = fmax(mx, fabs(r - D[i * 16 + j]));
        mref = fmax(mref, fabs(r));
      }
    printf("%s: max abs err %.3e (max |ref| %.3f)\n", native ? "native f32" : "bf16 split", mx, mref);
  }
  return 0;
}
