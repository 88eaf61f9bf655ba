// Fusion-evaluation metric of the reference (code/attack/interpolation.py:903-919 cal_SSMI, used by
// cal_result :1076-1091): SSIM between a reference image and each of N images, computed the way
// skimage.metrics.structural_similarity does with its defaults on rgb2gray images:
//   gray = 0.2125·R + 0.7154·G + 0.0721·B                       (skimage.color.rgb2gray)
//   7×7 uniform window, sample covariance (49/48), K1 = 0.01, K2 = 0.03, C = (K·data_range)²
//   S = (2·ux·uy + C1)(2·vxy + C2) / ((ux² + uy² + C1)(vx + vy + C2))
//   mean of S over the pixels whose window lies inside the image (skimage crops a 3-pixel border,
//   so its reflect padding never reaches the mean).
// The images are NCHW fp32 at the API (the fused / attacked images in [-1, 1]). HBM-bound: every
// block stages the (32+6)² gray window of the reference and of its image in LDS (one read of the
// 3 channels each), forms the five window moments by separable row/column sums, and reduces S in
// fp64 into its own slot of the per-image tile partials (work[n][tile]); a second launch sums an
// image's slots in tile order and divides by the pixel count — no atomics, so an image's SSIM is
// bit-identical run to run and independent of the other images of the call.
#include "mia_common.h"

namespace mia {

constexpr int SS_T = 32, SS_R = 3, SS_W = SS_T + 2 * SS_R;  // 38

__device__ __forceinline__ float gray_at(const float* img, int64_t plane, int idx) {
  return 0.2125f * img[idx] + 0.7154f * img[plane + idx] + 0.0721f * img[2 * plane + idx];
}

// grid (tiles_x, tiles_y, N), 256 threads: the output tile [oy0, oy0+32) × [ox0, ox0+32) of the
// interior [3, H−3) × [3, W−3), 4 pixels per thread
__global__ __launch_bounds__(256) void ssim_tile_kernel(const float* __restrict__ ref,
                                                        const float* __restrict__ imgs, int H,
                                                        int W, float c1, float c2,
                                                        double* __restrict__ part) {
  __shared__ float gx[SS_W][SS_W + 1], gy[SS_W][SS_W + 1];
  // row sums over the 7 columns of a window, 5 moments, for the 38 rows × 32 columns
  __shared__ float rs[5][SS_W][SS_T + 1];
  __shared__ double red[4];
  const int n = blockIdx.z, tid = threadIdx.x;
  const int ox0 = SS_R + blockIdx.x * SS_T, oy0 = SS_R + blockIdx.y * SS_T;
  const int64_t plane = (int64_t)H * W;
  const float* img = imgs + (int64_t)n * 3 * plane;
  for (int i = tid; i < SS_W * SS_W; i += 256) {
    const int r = i / SS_W, c = i - r * SS_W;
    const int y = oy0 - SS_R + r, x = ox0 - SS_R + c;
    float a = 0.f, b = 0.f;
    if (y < H && x < W) {
      const int idx = y * W + x;
      a = gray_at(ref, plane, idx);
      b = gray_at(img, plane, idx);
    }
    gx[r][c] = a;
    gy[r][c] = b;
  }
  __syncthreads();
  for (int i = tid; i < SS_W * SS_T; i += 256) {
    const int r = i / SS_T, c = i - r * SS_T;
    float sx = 0.f, sy = 0.f, sxx = 0.f, syy = 0.f, sxy = 0.f;
#pragma unroll
    for (int d = 0; d < 2 * SS_R + 1; ++d) {
      const float a = gx[r][c + d], b = gy[r][c + d];
      sx += a;
      sy += b;
      sxx += a * a;
      syy += b * b;
      sxy += a * b;
    }
    rs[0][r][c] = sx;
    rs[1][r][c] = sy;
    rs[2][r][c] = sxx;
    rs[3][r][c] = syy;
    rs[4][r][c] = sxy;
  }
  __syncthreads();
  constexpr float inv_np = 1.f / 49.f, cov = 49.f / 48.f;
  double acc = 0.0;
  for (int i = tid; i < SS_T * SS_T; i += 256) {
    const int r = i / SS_T, c = i - r * SS_T;
    if (oy0 + r >= H - SS_R || ox0 + c >= W - SS_R) continue;
    float m[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < 2 * SS_R + 1; ++d) s += rs[q][r + d][c];
      m[q] = s * inv_np;
    }
    const float ux = m[0], uy = m[1];
    const float vx = cov * (m[2] - ux * ux), vy = cov * (m[3] - uy * uy);
    const float vxy = cov * (m[4] - ux * uy);
    const float a1 = 2.f * ux * uy + c1, a2 = 2.f * vxy + c2;
    const float b1 = ux * ux + uy * uy + c1, b2 = vx + vy + c2;
    acc += (double)((a1 * a2) / (b1 * b2));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  const int ntiles = gridDim.x * gridDim.y;
  if (tid == 0)
    part[(int64_t)n * ntiles + blockIdx.y * gridDim.x + blockIdx.x] =
        ((red[0] + red[1]) + red[2]) + red[3];
}

// one wave per image: lane l sums tiles l, l+64, … in order, then a fixed butterfly
__global__ __launch_bounds__(64) void ssim_finish_kernel(const double* __restrict__ part,
                                                         float* __restrict__ out, int ntiles,
                                                         double count) {
  const int n = blockIdx.x, l = threadIdx.x;
  const double* p = part + (int64_t)n * ntiles;
  double s = 0.0;
  for (int k = l; k < ntiles; k += 64) s += p[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (l == 0) out[n] = (float)(s / count);
}

}  // namespace mia

using namespace mia;

static inline int64_t ssim_tiles(int H, int W) {
  return (int64_t)((W - 2 * SS_R + SS_T - 1) / SS_T) * ((H - 2 * SS_R + SS_T - 1) / SS_T);
}

extern "C" int64_t mia_ssim_workspace_size(int N, int H, int W) {
  if (N <= 0 || H < 7 || W < 7) return 0;
  return (int64_t)N * ssim_tiles(H, W) * (int64_t)sizeof(double);
}

// The scratch grew from N doubles to one per image and tile (round 4); the old mia_ssim took no
// size, so a caller sized for the old contract would have had its buffer overrun silently. That
// symbol is gone: mia_ssim2 takes the scratch size and rejects one below
// mia_ssim_workspace_size, and an old caller fails to link instead of corrupting memory.
extern "C" int mia_ssim2(const float* ref, const float* imgs, int N, int H, int W,
                         float data_range, double* work, int64_t work_bytes, float* ssim_out,
                         void* stream) {
  MIA_CHECK_ARG(ref && imgs && work && ssim_out && N > 0, "bad args");
  MIA_CHECK_ARG(H >= 7 && W >= 7, "images smaller than the 7×7 window");
  MIA_CHECK_ARG(work_bytes >= mia_ssim_workspace_size(N, H, W),
                "work_bytes < mia_ssim_workspace_size(N, H, W)");
  MIA_CHECK_ARG(data_range > 0.f, "data_range must be > 0");
  hipStream_t st = (hipStream_t)stream;
  const float c1 = (0.01f * data_range) * (0.01f * data_range);
  const float c2 = (0.03f * data_range) * (0.03f * data_range);
  const int iw = W - 2 * SS_R, ih = H - 2 * SS_R;
  const dim3 grid((iw + SS_T - 1) / SS_T, (ih + SS_T - 1) / SS_T, N);
  hipLaunchKernelGGL(ssim_tile_kernel, grid, dim3(256), 0, st, ref, imgs, H, W, c1, c2, work);
  const int rc = check_launch("ssim_tile_kernel");
  if (rc != MIA_OK) return rc;
  hipLaunchKernelGGL(ssim_finish_kernel, dim3(N), dim3(64), 0, st, work, ssim_out,
                     (int)ssim_tiles(H, W), (double)iw * ih);
  return check_launch("ssim_finish_kernel");
}
