// Probe: print the packed bf16 split of 4 fp32 values
#include <cstdio>
#include <cstring>
#include "../../adversarial-attacks-on-gan-based-image-fusion_amd/csrc/conv_common.h"
using namespace mia;
__global__ void k(const float* in, unsigned* out) {
  f32x4 a = {in[0], in[1], in[2], in[3]};
  const Split3 s = split3(a);
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  const u32x4 x = __builtin_bit_cast(u32x4, s.hm), y = __builtin_bit_cast(u32x4, s.hl);
  if (threadIdx.x == 0) for (int i = 0; i < 4; ++i) { out[i] = x[i]; out[4 + i] = y[i]; }
}
namespace mia { int set_error(const std::string&) { return 1; } int check_launch(const char*) { return 0; } }
static float bf(unsigned short h) { unsigned u = (unsigned)h << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
  float a[4] = {1.2345678f, -0.33333334f, 3.1415927f, 1e-3f};
  float* d; unsigned* o; (void)hipMalloc(&d, 16); (void)hipMalloc(&o, 32);
  (void)hipMemcpy(d, a, 16, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  unsigned h[8]; (void)hipMemcpy(h, o, 32, hipMemcpyDeviceToHost);
  for (int e = 0; e < 4; ++e) {
    const unsigned w = h[e / 2], wm = h[2 + e / 2], wl = h[4 + 2 + e / 2];
    const unsigned short hi = (e & 1) ? w >> 16 : w & 0xffff, mi = (e & 1) ? wm >> 16 : wm & 0xffff,
                         lo = (e & 1) ? wl >> 16 : wl & 0xffff;
    printf("a=%.9g hi=%.9g mid=%.9g lo=%.9g sum=%.9g\n", a[e], bf(hi), bf(mi), bf(lo),
           (double)bf(hi) + bf(mi) + bf(lo));
  }
  return 0;
}
