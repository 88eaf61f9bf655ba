// Probe: which B slot (lane group, element) v_mfma_f32_16x16x32_bf16 pairs with each A slot.
#include <cstdio>
#include <cmath>
#include <hip/hip_runtime.h>
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
__global__ void k_map(float* out, int q0, int e0) {
  const int lane = threadIdx.x, q = lane >> 4;
  bf16x8 a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = (__bf16)((q == q0 && e == e0) ? 1.f : 0.f);
    b[e] = (__bf16)ldexpf(1.f, q * 8 + e);
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  if (lane == 0) out[0] = c[0];
}
int main() {
  float* d; (void)hipMalloc(&d, 4);
  for (int q0 = 0; q0 < 4; ++q0) {
    for (int e0 = 0; e0 < 8; ++e0) {
      hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, d, q0, e0);
      float h; (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
      const int s = (int)log2f(h);
      printf("A(q%d,e%d)->B(q%d,e%d)  ", q0, e0, s / 8, s % 8);
    }
    printf("\n");
  }
  return 0;
}
