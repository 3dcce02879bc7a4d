// Winograd F(4x4, 3x3) input / output transforms as separate memory-bound passes, for the
// "explicit" fp32 Winograd convolution of the wide ResNet-18 layers (256 and 512 channels):
//
//   V[p][t][c]  = (B^T d B)[p]      d = the 6x6 input window of output tile t, channel c
//   M[p][t][co] = sum_c V[p][t][c] U[p][co][c]        36 GEMMs: rmbx_linear_f32x6_batched (the
//                                                      fp32-accurate bf16x6 GEMM, U = G g G^T)
//   Y[t][co]    = relu?(A^T M A + bias + res)          the 4x4 outputs of tile t
//
// Replaces the stride-1 3x3 conv + FrozenBatchNorm (+ residual) + ReLU steps of ResNet-18's
// layer-3/4 BasicBlocks in ACT's backbone (third_party/act [absent], torchvision resnet18) on the
// fp32 policy path.  At 256/512 channels the per-tile HBM round trip of V and M (2.25x the input
// each way) costs less than the fused kernel's f32-MFMA time the bf16x6 GEMM saves
// (scripts/prof_wino_x6.py); at 64/128 channels it does not, and the fused
// rmbx_conv3x3_winograd4_f32 stays.
//
// Points {0, +-1, +-2, inf} (Lavin): B^T rows
//   [4 0 -5 0 1 0] [0 -4 -4 1 1 0] [0 4 -4 -1 1 0] [0 -2 -1 2 1 0] [0 2 -1 -2 1 0] [0 4 0 -5 0 1]
// A^T rows [1 1 1 1 1 0] [0 1 -1 2 -2 0] [0 1 1 4 4 0] [0 1 -1 8 -8 1]; the same transforms and
// f32 operation order class as the fused kernel (error ~1e-5 relative, tests/test_wino_x6_gpu.py).
//
// Layout: NHWC activations; tile t = (img, ty, tx) row-major over [N][ceil(H/4)][ceil(W/4)];
// V and M are [36][T][C] so each position p is one row-major GEMM operand.  One thread per
// (tile, channel): consecutive threads walk consecutive channels, so every load and store is a
// contiguous run of the channel dim (fully coalesced).
#include "rmbx_common.h"

#include <cstdint>

namespace rmbx {
namespace {

__device__ __forceinline__ void bt6(const float* x, float* y) {
  y[0] = 4.f * x[0] - 5.f * x[2] + x[4];
  y[1] = -4.f * x[1] - 4.f * x[2] + x[3] + x[4];
  y[2] = 4.f * x[1] - 4.f * x[2] - x[3] + x[4];
  y[3] = -2.f * x[1] - x[2] + 2.f * x[3] + x[4];
  y[4] = 2.f * x[1] - x[2] - 2.f * x[3] + x[4];
  y[5] = 4.f * x[1] - 5.f * x[3] + x[5];
}

__device__ __forceinline__ void at6(const float* m, float* z) {
  z[0] = m[0] + m[1] + m[2] + m[3] + m[4];
  z[1] = m[1] - m[2] + 2.f * m[3] - 2.f * m[4];
  z[2] = m[1] + m[2] + 4.f * m[3] + 4.f * m[4];
  z[3] = m[1] - m[2] + 8.f * m[3] - 8.f * m[4] + m[5];
}

__global__ void __launch_bounds__(256) wino4_input_kernel(const float* __restrict__ in, float* __restrict__ V, int H,
                                                          int W, int C, int ty_n, int tx_n, long long T) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * C) return;
  const int c = (int)(idx % C);
  const long long t = idx / C;
  const int tx = (int)(t % tx_n);
  const long long q = t / tx_n;
  const int ty = (int)(q % ty_n);
  const long long img = q / ty_n;
  const int y0 = 4 * ty - 1, x0 = 4 * tx - 1;
  const float* base = in + img * H * (long long)W * C + c;
  float d[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int y = y0 + i, x = x0 + j;
      d[i][j] = ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) ? base[((long long)y * W + x) * C] : 0.f;
    }
  float r[6][6];  // B^T along each row
#pragma unroll
  for (int i = 0; i < 6; ++i) bt6(d[i], r[i]);
  const long long ps = T * C;  // position stride
  float* out = V + t * C + c;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], v[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) col[i] = r[i][j];
    bt6(col, v);  // B^T down the column: v[i] = V at position (i, j)
#pragma unroll
    for (int i = 0; i < 6; ++i) out[(i * 6 + j) * ps] = v[i];
  }
}

__global__ void __launch_bounds__(256) wino4_output_kernel(const float* __restrict__ M, const float* __restrict__ bias,
                                                           const float* __restrict__ res, float* __restrict__ out,
                                                           int H, int W, int C, int ty_n, int tx_n, long long T,
                                                           int relu) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * C) return;
  const int c = (int)(idx % C);
  const long long t = idx / C;
  const int tx = (int)(t % tx_n);
  const long long q = t / tx_n;
  const int ty = (int)(q % ty_n);
  const long long img = q / ty_n;
  const long long ps = T * C;
  const float* src = M + t * C + c;
  float r[4][6];  // A^T down each column of M
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], z[4];
#pragma unroll
    for (int i = 0; i < 6; ++i) col[i] = src[(i * 6 + j) * ps];
    at6(col, z);
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i][j] = z[i];
  }
  const float b = bias ? bias[c] : 0.f;
  const long long obase = img * H * (long long)W * C + c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float z[4];
    at6(r[i], z);
    const int y = 4 * ty + i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = 4 * tx + j;
      if (y < H && x < W) {
        const long long o = obase + ((long long)y * W + x) * C;
        float v = z[j] + b;
        if (res) v += res[o];
        if (relu) v = fmaxf(v, 0.f);
        out[o] = v;
      }
    }
  }
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_wino4_input_f32(const float* in, int N, int H, int W, int C, float* V, void* stream) {
  RMBX_CHECK_ARG(in && V && N >= 0 && H > 0 && W > 0 && C > 0, "rmbx_wino4_input_f32: bad arguments");
  const int ty = (H + 3) / 4, tx = (W + 3) / 4;
  const long long T = (long long)N * ty * tx;
  if (T == 0) return RMBX_OK;
  const long long n = T * C;
  hipLaunchKernelGGL(rmbx::wino4_input_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     in, V, H, W, C, ty, tx, T);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_wino4_output_f32(const float* M, int N, int H, int W, int C, const float* bias, const float* res,
                                     float* out, int relu, void* stream) {
  RMBX_CHECK_ARG(M && out && N >= 0 && H > 0 && W > 0 && C > 0, "rmbx_wino4_output_f32: bad arguments");
  const int ty = (H + 3) / 4, tx = (W + 3) / 4;
  const long long T = (long long)N * ty * tx;
  if (T == 0) return RMBX_OK;
  const long long n = T * C;
  hipLaunchKernelGGL(rmbx::wino4_output_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     M, bias, res, out, H, W, C, ty, tx, T, relu ? 1 : 0);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
