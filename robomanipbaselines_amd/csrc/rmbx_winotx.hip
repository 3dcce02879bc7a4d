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

// Input transform emitting the position GEMMs' A in the pre-split form (rmbx_linear_f16x3_presplit
// _batched): block = one tile, thread = channels tid, tid + 256, ...; the tile's 36 x C transformed
// values are scaled by one power of two 2^t putting their max |v| in [2^13, 2^14) (a block max
// reduction), hi = f16(v 2^t), lo = f16(v 2^t - hi) into planes [2][36][T][C], rinv[t] = 2^-t.  One
// scale per tile for all 36 positions: a position whose values are far below the tile's max keeps
// its pieces exact to 2^-38 of that max (f16 subnormal low pieces below 2^-16 of it), well inside
// the transform's own rounding.  The scale comes from the tile's own inputs (batch-invariant).
__global__ void __launch_bounds__(256) wino4_input_split_kernel(const float* __restrict__ in, uint16_t* __restrict__ Vp,
                                                                float* __restrict__ rinv, int H, int W, int C,
                                                                int ty_n, int tx_n, long long T) {
  // thread = two adjacent channels 2 tid, 2 tid + 1 (8-byte loads, 4-byte piece stores); C = 2 blockDim
  __shared__ float red[4];
  const long long t = blockIdx.x;
  const int tx = (int)(t % tx_n);
  const long long q = t / tx_n;
  const int ty = (int)(q % ty_n);
  const long long img = q / ty_n;
  const int y0 = 4 * ty - 1, x0 = 4 * tx - 1;
  const int c = 2 * threadIdx.x;
  const float* base = in + img * H * (long long)W * C + c;
  float v[2][36];
  float mx = 0.f;
  {
    float d[2][6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int y = y0 + i, x = x0 + j;
        float2 dv = make_float2(0.f, 0.f);
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) dv = *(const float2*)(base + ((long long)y * W + x) * C);
        d[0][i][j] = dv.x;
        d[1][i][j] = dv.y;
      }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float r[6][6];
#pragma unroll
      for (int i = 0; i < 6; ++i) bt6(d[k][i], r[i]);
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        float col[6], vv[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = r[i][j];
        bt6(col, vv);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          v[k][i * 6 + j] = vv[i];
          mx = fmaxf(mx, fabsf(vv[i]));
        }
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  const int nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = red[0];
  for (int w = 1; w < nw; ++w) mx = fmaxf(mx, red[w]);
  int e = 14;
  if (mx > 0.f && mx <= 3.4e38f) frexpf(mx, &e);  // NaN / inf: scale 1, propagated
  const float sc = ldexpf(1.f, 14 - e);
  if (threadIdx.x == 0) rinv[t] = ldexpf(1.f, e - 14);
  const long long ps = T * C, plane = 36 * ps;
  uint32_t* o = reinterpret_cast<uint32_t*>(Vp + t * C + c);
#pragma unroll
  for (int p = 0; p < 36; ++p) {
    const float a0 = v[0][p] * sc, a1 = v[1][p] * sc;
    const _Float16 h0 = (_Float16)a0, h1 = (_Float16)a1;
    const _Float16 l0 = (_Float16)(a0 - (float)h0), l1 = (_Float16)(a1 - (float)h1);
    o[p * ps / 2] = __builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    o[(plane + p * ps) / 2] = __builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
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

extern "C" int rmbx_wino4_input_split(const float* in, int N, int H, int W, int C, void* V_planes, float* rinv,
                                      void* stream) {
  RMBX_CHECK_ARG(in && V_planes && rinv && N >= 0 && H > 0 && W > 0 && C > 0 && C <= 512 && C % 2 == 0,
                 "rmbx_wino4_input_split: bad arguments (C even, <= 512)");
  RMBX_CHECK_ARG(((uintptr_t)in % 8) == 0 && ((uintptr_t)V_planes % 4) == 0, "rmbx_wino4_input_split: unaligned");
  const int ty = (H + 3) / 4, tx = (W + 3) / 4;
  const long long T = (long long)N * ty * tx;
  if (T == 0) return RMBX_OK;
  RMBX_CHECK_ARG(T < (1ll << 31), "rmbx_wino4_input_split: too many tiles");
  hipLaunchKernelGGL(rmbx::wino4_input_split_kernel, dim3((unsigned)T), dim3(C / 2), 0, (hipStream_t)stream, in,
                     (uint16_t*)V_planes, rinv, H, W, C, ty, tx, T);
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

// ---------------------------------------------------------------------------------------------
// Direct f32 convolution for few input channels (the 3-channel 7x7 / stride-2 stem of the
// diffusion policy's GroupNorm ResNet-18 image encoder, robomimic ResNet18Conv inside
// third_party/diffusion_policy [absent], run by policy/diffusion_policy/RolloutDiffusionPolicy.py in
// fp32): out[n][oy][ox][co] = sum_{ky,kx,c} in[n][iy][ix][c] w[co][ky][kx][c] (+ bias), NHWC.
// MIOpen's deterministic solver set for this shape is its naive kernel (4.3 s per 4096-image
// call); this one keeps the fixed f32 summation order (deterministic) at the VALU rate.  Thread =
// one output pixel x 16 output channels (consecutive threads: consecutive pixels of one channel
// group); the filter bank [Cout][KH*KW*C] sits in LDS and is read as a broadcast.
// ---------------------------------------------------------------------------------------------
namespace rmbx {
namespace {

constexpr int DC_MAX_W = 64 * 7 * 7 * 4;  // filter floats held in LDS (Cout <= 64, K <= 196)

__global__ void __launch_bounds__(256) conv_direct_f32_kernel(const float* __restrict__ in, const float* __restrict__ w,
                                                              const float* __restrict__ bias, float* __restrict__ out,
                                                              int N, int H, int W, int C, int Ho, int Wo, int Cout,
                                                              int KH, int KW, int stride, int pad) {
  __shared__ float sw[DC_MAX_W];
  const int K = KH * KW * C;
  for (int i = threadIdx.x; i < Cout * K; i += blockDim.x) sw[i] = w[i];
  __syncthreads();
  const int groups = Cout / 16;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long npix = (long long)N * Ho * Wo;
  if (idx >= npix * groups) return;
  const int cg = (int)(idx / npix);  // a wave shares its filter group: broadcast weight reads
  const long long p = idx - cg * npix;
  const int ox = (int)(p % Wo);
  const long long q = p / Wo;
  const int oy = (int)(q % Ho);
  const long long n = q / Ho;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = bias ? bias[16 * cg + j] : 0.f;
  const float* wb = sw + (16 * cg) * K;
  for (int ky = 0; ky < KH; ++ky) {
    const int iy = oy * stride - pad + ky;
    if ((unsigned)iy >= (unsigned)H) continue;
    for (int kx = 0; kx < KW; ++kx) {
      const int ix = ox * stride - pad + kx;
      if ((unsigned)ix >= (unsigned)W) continue;
      const float* src = in + ((n * H + iy) * W + ix) * C;
      const int k0 = (ky * KW + kx) * C;
      for (int c = 0; c < C; ++c) {
        const float v = src[c];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = fmaf(v, wb[j * K + k0 + c], acc[j]);
      }
    }
  }
  float4* o = (float4*)(out + p * Cout + 16 * cg);
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = make_float4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]);
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_conv2d_direct_f32(const float* in, int N, int H, int W, int C, const float* w, const float* bias,
                                      float* out, int Cout, int KH, int KW, int stride, int pad, void* stream) {
  RMBX_CHECK_ARG(in && w && out && N >= 0 && H > 0 && W > 0 && C > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0,
                 "rmbx_conv2d_direct_f32: bad arguments");
  RMBX_CHECK_ARG(Cout % 16 == 0 && Cout * KH * KW * C <= rmbx::DC_MAX_W,
                 "rmbx_conv2d_direct_f32: Cout=%d must be a multiple of 16 and the filter bank fit %d floats", Cout,
                 rmbx::DC_MAX_W);
  RMBX_CHECK_ARG(((uintptr_t)out) % 16 == 0, "rmbx_conv2d_direct_f32: out must be 16-B aligned");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  RMBX_CHECK_ARG(Ho > 0 && Wo > 0, "rmbx_conv2d_direct_f32: empty output");
  const long long n = (long long)N * Ho * Wo * (Cout / 16);
  if (n == 0) return RMBX_OK;
  RMBX_CHECK_ARG((n + 255) / 256 < (1ll << 31), "rmbx_conv2d_direct_f32: too many pixels");
  hipLaunchKernelGGL(rmbx::conv_direct_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, in, w, bias, out, N, H, W, C, Ho, Wo, Cout, KH, KW, stride, pad);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
