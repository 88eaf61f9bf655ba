// Probe: which slot pairing of the bf16 split goes wrong. One wave, 16×16 output, k = 16.
#include <cstdio>
#include <cmath>
#include <cstring>
#include <vector>
#include "../../adversarial-attacks-on-gan-based-image-fusion_amd/csrc/conv_common.h"
using namespace mia;
__global__ void k_diag(const float* A, const float* B, float* D, int mode) {
  const int lane = threadIdx.x, row = lane & 15, q = lane >> 4;
  f32x4 a, b;
  for (int e = 0; e < 4; ++e) { a[e] = A[row * 16 + 4 * q + e]; b[e] = B[(4 * q + e) * 16 + row]; }
  const Split3 sa = split3(a), sb = split3(b);
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  const u32x4 bhm = __builtin_bit_cast(u32x4, sb.hm), bhl = __builtin_bit_cast(u32x4, sb.hl);
  const u32x4 ahm = __builtin_bit_cast(u32x4, sa.hm);
  const bf16x8 bhh = __builtin_bit_cast(bf16x8, (u32x4){bhm[0], bhm[1], bhm[0], bhm[1]});
  const bf16x8 ah0 = __builtin_bit_cast(bf16x8, (u32x4){ahm[0], ahm[1], 0u, 0u});
  f32x4 c = {0, 0, 0, 0};
  if (mode == 0) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, bhh, c, 0, 0, 0);  // hh
  if (mode == 1) c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa.hm, bhh, c, 0, 0, 0);  // hh + mh
  if (mode == 2) c = mfma_chunk<float>(a, b, c);
  for (int r = 0; r < 4; ++r) D[(4 * q + r) * 16 + row] = c[r];
}
namespace mia { int set_error(const std::string&) { return 1; } int check_launch(const char*) { return 0; } }
static float tr(float x) { unsigned u; memcpy(&u, &x, 4); u &= 0xffff0000u; memcpy(&x, &u, 4); return x; }
int main() {
  std::vector<float> A(256), B(256), D(256);
  unsigned s = 1;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) / 16777216.f) * 2.f - 1.f; };
  for (auto& v : A) v = rnd();
  for (auto& v : B) v = rnd();
  float *dA, *dB, *dD;
  (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dD, 1024);
  (void)hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(k_diag, dim3(1), dim3(64), 0, 0, dA, dB, dD, mode);
    (void)hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
    double mx = 0, mxfull = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double r = 0, full = 0;
        for (int k = 0; k < 16; ++k) {
          const float a = A[i * 16 + k], b = B[k * 16 + j];
          const float ah = tr(a), bh = tr(b), am = tr(a - ah);
          full += (double)a * b;
          if (mode == 0) r += (double)ah * bh;
          if (mode == 1) r += (double)ah * bh + (double)am * bh;
          if (mode == 2) r = full;
        }
        mx = fmax(mx, fabs(r - D[i * 16 + j]));
        mxfull = fmax(mxfull, fabs(full - D[i * 16 + j]));
      }
    printf("mode %d: max err vs its own expected %.3e, vs exact %.3e\n", mode, mx, mxfull);
  }
  return 0;
}
