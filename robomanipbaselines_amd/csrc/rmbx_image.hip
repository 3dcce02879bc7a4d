// Policy-input image preprocessing, batched: resize (OpenCV INTER_LINEAR semantics) + crop +
// ToDtype(scale) + affine, from the renderer's u8 HWC frames straight into the policy's CHW
// tensor; and the f32 depth resize of the point-cloud path.
//
// Replaces, per env and camera:
//   * RolloutDiffusionPolicy.get_images (policy/diffusion_policy/RolloutDiffusionPolicy.py:107-138):
//     cv2.resize(image, image_size) -> moveaxis -> v2.ToDtype(float32, scale=True) -> * 2 - 1, and
//     the eval-time centre crop of the robomimic obs encoder (crop_shape, eval_fixed_crop,
//     TrainDiffusionPolicy.py:125-128);
//   * RolloutDiffusionPolicy3d.get_pointcloud (policy/diffusion_policy_3d/RolloutDiffusionPolicy3d.py:
//     138-145): cv2.resize of the rgb and depth images to image_size.
//
// OpenCV semantics restated: for an exact 2x down-scale INTER_LINEAR is routed to the area-fast
// path (2x2 mean, (a + b + c + d + 2) >> 2); otherwise source coordinate fx = (x + 0.5) * scale - 0.5
// clamped at the borders, u8 with 11-bit fixed-point weights and a (sum + 2^21) >> 22 rounding,
// f32 with float weights.  (OpenCV's SIMD vertical pass for u8 rounds slightly differently; images
// are from the substitute renderer, so pixel parity with OpenCV is unpinned anyway.)

#include "rmbx_common.h"

#include <hip/hip_bf16.h>

#include <cstdint>

namespace rmbx {
namespace {

struct Coord {
  int s0, s1;     // source indices
  float w1;       // float weight of s1
  int c0, c1;     // fixed-point weights (sum 2048)
};

__device__ __forceinline__ Coord coord(int d, int dsize, int ssize) {
  const double scale = (double)ssize / dsize;
  float fx = (float)((d + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx -= sx;
  if (sx < 0) {
    fx = 0.f;
    sx = 0;
  }
  if (sx >= ssize - 1) {
    fx = 0.f;
    sx = ssize - 1;
  }
  Coord c;
  c.s0 = sx;
  c.s1 = sx + 1 < ssize ? sx + 1 : sx;
  c.w1 = fx;
  c.c0 = (int)rintf((1.f - fx) * 2048.f);
  c.c1 = 2048 - c.c0;
  return c;
}

struct ImgArgs {
  const uint8_t* src;  // [n][H][W][C]
  int H, W, C;
  int rh, rw;          // resized size
  int y0, x0, ch, cw;  // crop window in resized coordinates
  float a, b;          // out = (v * (1/255)) * a + b
  void* dst;           // [n][C][ch][cw] (f32 / bf16) or [n][ch][cw][C] (u8)
  int dst_dtype;       // 0 f32, 1 bf16, 2 u8 (resized pixels, HWC, no scaling)
  int n_env;
};

__global__ void __launch_bounds__(256) resize_crop_u8_kernel(ImgArgs g) {
#pragma clang fp contract(off)
  const size_t total = (size_t)g.n_env * g.ch * g.cw;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const bool area2 = (g.W == 2 * g.rw) && (g.H == 2 * g.rh);
  const float inv255 = 1.0f / 255.0f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int x = (int)(i % g.cw) + g.x0;
    const int y = (int)((i / g.cw) % g.ch) + g.y0;
    const int e = (int)(i / ((size_t)g.cw * g.ch));
    const uint8_t* img = g.src + (size_t)e * g.H * g.W * g.C;
    for (int c = 0; c < g.C; ++c) {
      int v;
      if (area2) {
        const uint8_t* p = img + ((size_t)(2 * y) * g.W + 2 * x) * g.C + c;
        const size_t rs = (size_t)g.W * g.C;
        v = (p[0] + p[g.C] + p[rs] + p[rs + g.C] + 2) >> 2;
      } else {
        const Coord cx = coord(x, g.rw, g.W), cy = coord(y, g.rh, g.H);
        const uint8_t* r0 = img + (size_t)cy.s0 * g.W * g.C;
        const uint8_t* r1 = img + (size_t)cy.s1 * g.W * g.C;
        const int h0 = r0[cx.s0 * g.C + c] * cx.c0 + r0[cx.s1 * g.C + c] * cx.c1;
        const int h1 = r1[cx.s0 * g.C + c] * cx.c0 + r1[cx.s1 * g.C + c] * cx.c1;
        v = (h0 * cy.c0 + h1 * cy.c1 + (1 << 21)) >> 22;
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
      }
      if (g.dst_dtype == 2) {
        reinterpret_cast<uint8_t*>(g.dst)[(((size_t)e * g.ch + (y - g.y0)) * g.cw + (x - g.x0)) * g.C + c] = (uint8_t)v;
        continue;
      }
      const float f = ((float)v * inv255) * g.a + g.b;
      const size_t o = (((size_t)e * g.C + c) * g.ch + (y - g.y0)) * g.cw + (x - g.x0);
      if (g.dst_dtype == 1)
        reinterpret_cast<__hip_bfloat16*>(g.dst)[o] = __float2bfloat16(f);
      else
        reinterpret_cast<float*>(g.dst)[o] = f;
    }
  }
}

// f32 single-channel resize (cv2.resize of the float depth image), [n][H][W] -> [n][rh][rw]
__global__ void __launch_bounds__(256) resize_f32_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                         int n_env, int H, int W, int rh, int rw) {
#pragma clang fp contract(off)
  const size_t total = (size_t)n_env * rh * rw;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const bool area2 = (W == 2 * rw) && (H == 2 * rh);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int x = (int)(i % rw);
    const int y = (int)((i / rw) % rh);
    const int e = (int)(i / ((size_t)rw * rh));
    const float* img = src + (size_t)e * H * W;
    float v;
    if (area2) {
      const float* p = img + (size_t)(2 * y) * W + 2 * x;
      v = (p[0] + p[1] + p[W] + p[W + 1]) * 0.25f;
    } else {
      const Coord cx = coord(x, rw, W), cy = coord(y, rh, H);
      const float* r0 = img + (size_t)cy.s0 * W;
      const float* r1 = img + (size_t)cy.s1 * W;
      const float h0 = r0[cx.s0] * (1.f - cx.w1) + r0[cx.s1] * cx.w1;
      const float h1 = r1[cx.s0] * (1.f - cx.w1) + r1[cx.s1] * cx.w1;
      v = h0 * (1.f - cy.w1) + h1 * cy.w1;
    }
    dst[i] = v;
  }
}

int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_resize_crop_u8(const uint8_t* src, int n_env, int H, int W, int C, int rh, int rw, int y0,
                                   int x0, int ch, int cw, float a, float b, void* dst, int dst_dtype,
                                   void* stream) {
  RMBX_CHECK_ARG(src && dst, "rmbx_resize_crop_u8: null pointer");
  RMBX_CHECK_ARG(H > 0 && W > 0 && C > 0 && C <= 4 && rh > 0 && rw > 0, "rmbx_resize_crop_u8: bad sizes");
  RMBX_CHECK_ARG(y0 >= 0 && x0 >= 0 && ch > 0 && cw > 0 && y0 + ch <= rh && x0 + cw <= rw,
                 "rmbx_resize_crop_u8: crop (%d,%d,%d,%d) outside %dx%d", y0, x0, ch, cw, rh, rw);
  RMBX_CHECK_ARG(dst_dtype >= 0 && dst_dtype <= 2, "rmbx_resize_crop_u8: dst_dtype must be 0, 1 or 2");
  if (n_env == 0) return RMBX_OK;
  rmbx::ImgArgs g{src, H, W, C, rh, rw, y0, x0, ch, cw, a, b, dst, dst_dtype, n_env};
  hipLaunchKernelGGL(rmbx::resize_crop_u8_kernel, dim3(rmbx::grid_for((size_t)n_env * ch * cw)), dim3(256), 0,
                     (hipStream_t)stream, g);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_resize_f32(const float* src, float* dst, int n_env, int H, int W, int rh, int rw,
                               void* stream) {
  RMBX_CHECK_ARG(src && dst, "rmbx_resize_f32: null pointer");
  RMBX_CHECK_ARG(H > 0 && W > 0 && rh > 0 && rw > 0, "rmbx_resize_f32: bad sizes");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::resize_f32_kernel, dim3(rmbx::grid_for((size_t)n_env * rh * rw)), dim3(256), 0,
                     (hipStream_t)stream, src, dst, n_env, H, W, rh, rw);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
