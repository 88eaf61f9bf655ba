// Host-side sanitizer harness ("-fsanitize=address builds on the CPU-side
// harness"): libmiattack's host code — the C ABI's argument validation, the error-string state,
// the kernel-variant table and the reduction-scratch bookkeeping — compiled with
// -Xarch_host -fsanitize=address,undefined (device code unchanged) and driven through the public
// entry points with valid and invalid arguments. Any heap / stack / UB error aborts the process.
// No kernel is launched: every call below fails validation before reaching the GPU, except the
// scratch reserve / release cycle, which runs only when a device is present (the GPU box).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/miattack.h"

static int g_fail = 0;
#define EXPECT(cond, what)                                               \
  do {                                                                   \
    if (!(cond)) {                                                       \
      std::fprintf(stderr, "FAIL %s (%s:%d)\n", what, __FILE__, __LINE__); \
      ++g_fail;                                                          \
    }                                                                    \
  } while (0)

static void expect_error(int rc, const char* what) {
  EXPECT(rc != MIA_OK, what);
  const char* msg = mia_last_error_string();
  EXPECT(msg != nullptr && std::strlen(msg) > 0, what);
}

int main() {
  EXPECT(mia_version() > 0, "version");
  // tuning table: every documented switch round-trips; unknown / null names are refused
  const char* keys[] = {"MIA_CONV_HALO", "MIA_CONV_X6", "MIA_HALO_EPI", "MIA_X6_UNR",
                        "MIA_CONV_WRES128", "MIA_CONV_THIN", "MIA_CONV_THIN32", "MIA_CONV_WRES",
                        "MIA_CONV_REGEPI", "MIA_CONV_SMALLTILE", "MIA_S2DG_X6",
                        "MIA_S2DG_HALO", "MIA_UPCONV_X6", "MIA_UPCONV_HALO",
                        "MIA_CONV_WRES32", "MIA_HALO_C64", "MIA_X6_64S", "MIA_UPCONV_X6S"};
  for (const char* k : keys) {
    int v = -1, w = -1;
    EXPECT(mia_get_tuning(k, &v) == MIA_OK, k);
    EXPECT(mia_set_tuning(k, v + 7) == MIA_OK && mia_get_tuning(k, &w) == MIA_OK && w == v + 7, k);
    EXPECT(mia_set_tuning(k, v) == MIA_OK, k);
  }
  int v = 0;
  expect_error(mia_get_tuning("MIA_NO_SUCH_SWITCH", &v), "unknown switch");
  expect_error(mia_get_tuning("MIA_THIN_F32", &v), "removed switch");  // round 6
  expect_error(mia_get_tuning("MIA_EPI_PRERED", &v), "removed switch");
  expect_error(mia_set_tuning(nullptr, 1), "null switch");
  expect_error(mia_get_tuning("MIA_CONV_X6", nullptr), "null out");
  std::string longname(5000, 'x');  // the error string grows to hold it
  expect_error(mia_set_tuning(longname.c_str(), 1), "long name");
  EXPECT(std::strstr(mia_last_error_string(), "xxxx") != nullptr, "long name in error string");

  // workspace queries at the edges
  EXPECT(mia_conv_workspace_size(0, 16, 16, 64, 1) == 0, "ws N=0");
  EXPECT(mia_conv_workspace_size(2, 16, 16, 64, 0) == 0, "ws no sums");
  EXPECT(mia_conv_workspace_size(128, 1024, 1024, 32, 1) > 0, "ws 1024²");
  EXPECT(mia_conv_workspace_size(3, 7, 5, 8, 1) > 0, "ws ragged");
  EXPECT(mia_reduction_workspace_size(-1, 4, 4) == 0, "red ws");
  EXPECT(mia_ssim_workspace_size(2, 6, 6) == 0 && mia_ssim_workspace_size(3, 40, 37) > 0, "ssim ws");
  EXPECT(mia_conv_kpad(64, MIA_F16) >= 9 * 64 && mia_conv_kpad(3, MIA_F32) >= 27, "kpad");

  // argument validation of the conv entry points (no launch happens)
  expect_error(mia_conv3x3(nullptr, MIA_F32, nullptr), "conv3x3 null");
  mia_conv_args a;
  std::memset(&a, 0, sizeof(a));
  float dummy[64];
  a.x = a.w = a.y = dummy;
  a.N = 2; a.H = 16; a.W = 16; a.Cin = 64; a.Cout = 64;
  a.Kpad = mia_conv_kpad(64, MIA_F16) + 8;  // wrong
  expect_error(mia_conv3x3(&a, MIA_F16, nullptr), "conv3x3 bad Kpad");
  a.Kpad = mia_conv_kpad(64, MIA_F16);
  a.Cin = 48;  // not a power of two
  expect_error(mia_conv3x3(&a, MIA_F16, nullptr), "conv3x3 Cin");
  a.Cin = 64;
  a.sdot = dummy;  // sdot without aux_x
  expect_error(mia_conv3x3(&a, MIA_F16, nullptr), "conv3x3 sdot");
  a.sdot = nullptr;
  expect_error(mia_conv3x3(&a, 99, nullptr), "conv3x3 dtype");
  a.N = 1 << 20; a.H = 4096; a.W = 4096;  // 32-bit offset overflow guard
  expect_error(mia_conv3x3(&a, MIA_F16, nullptr), "conv3x3 size");
  a.N = 2; a.H = 16; a.W = 16;
  expect_error(mia_conv2d(&a, 3, nullptr, 1, 8, 8, MIA_F16, nullptr), "conv2d stride");
  expect_error(mia_conv2d(&a, 1, nullptr, 5, 8, 8, MIA_F16, nullptr), "conv2d groups");
  expect_error(mia_conv3x3_wmod(&a, 0, MIA_F16, nullptr), "wmod stride");
  expect_error(mia_conv3x3_wmod(&a, (int64_t)a.Cout * a.Kpad, MIA_F32, nullptr), "wmod fp32");
  a.in_scale = dummy;
  expect_error(mia_conv3x3_wmod(&a, (int64_t)a.Cout * a.Kpad, MIA_F16, nullptr), "wmod in_scale");
  expect_error(mia_modulate_weights(dummy, dummy, nullptr, dummy, 2, 64, 48, 9 * 48, MIA_F16,
                                    nullptr), "modw Cin");
  expect_error(mia_modulate_weights(nullptr, dummy, nullptr, dummy, 2, 64, 64,
                                    mia_conv_kpad(64, MIA_F16), MIA_F16, nullptr), "modw null");
  expect_error(mia_ssim2(dummy, dummy, 1, 5, 5, 2.f, nullptr, 0, dummy, nullptr), "ssim small");
  expect_error(mia_ssim2(dummy, dummy, 1, 64, 64, 0.f, (double*)dummy, 1 << 20, dummy, nullptr),
               "ssim dr");
  expect_error(mia_ssim2(dummy, dummy, 4, 64, 64, 2.f, (double*)dummy, 8 * 4, dummy, nullptr),
               "ssim work size");  // the round-3 contract (N doubles) is rejected
  expect_error(mia_gemm_f32_grouped(nullptr, 0, nullptr), "gemm groups");
  // the §8(b)-named K10 pair (round 6): nothing to write, or a 2-byte accumulating gradient
  expect_error(mia_mse_fwd_bwd(dummy, dummy, nullptr, nullptr, 1, 64, 1.f, 1.f, 0, MIA_F32,
                               nullptr), "mse_fwd_bwd no output");
  expect_error(mia_mse_fwd_bwd(dummy, dummy, dummy, dummy, 1, 64, 1.f, 1.f, 1, MIA_F16, nullptr),
               "mse_fwd_bwd fp16 accumulate");
  expect_error(mia_reserve_reduction_scratch(-1, nullptr), "scratch negative");
  EXPECT(mia_reserve_reduction_scratch(0, nullptr) == MIA_OK, "scratch zero");

  // the scratch table's grow / release cycle (device present only)
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    hipStream_t st;
    EXPECT(hipStreamCreate(&st) == hipSuccess, "stream");
    for (int64_t b : {int64_t(1) << 10, int64_t(1) << 22, int64_t(1) << 12, int64_t(1) << 24}) {
      EXPECT(mia_reserve_reduction_scratch(b, st) == MIA_OK, "reserve");
      EXPECT(mia_reduction_scratch_bytes(st) >= b, "reserved bytes");
    }
    EXPECT(mia_release_reduction_scratch(st) == MIA_OK, "release");
    EXPECT(mia_reduction_scratch_bytes(st) == 0, "released");
    EXPECT(mia_release_reduction_scratch(st) == MIA_OK, "release twice");
    (void)hipStreamDestroy(st);
    std::printf("scratch cycle on %d device(s): ok\n", ndev);
  } else {
    std::printf("no device: scratch cycle skipped\n");
  }
  std::printf("host ABI checks: %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
