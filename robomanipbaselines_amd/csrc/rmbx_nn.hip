// Fused epilogues of the policy vision trunk (ResNet-18, NHWC / channels_last activations).
//
// The reference's backbone (torchvision resnet18 with FrozenBatchNorm2d inside ACT's DETR,
// third_party/act [absent submodule]; policy/mlp/MlpPolicy.py:34-39 for the MLP policy) runs
// conv -> BN -> ReLU [-> maxpool] and conv -> BN -> (+ identity / downsample) -> ReLU.  With BN
// folded into the conv weights the remaining per-element work is bias, residual, ReLU and the
// stem max-pool; done as separate framework passes it is 3-4 full HBM round trips of the largest
// activations in the network (the stem output alone is 10 GB at 1024 envs).  These kernels do
// it in one pass, in the dtype of the activations, with the same rounding sequence as the
// unfused bf16 path (every intermediate rounded to the storage dtype, round-to-nearest-even),
// so the fused trunk is bit-identical to the unfused one on the same conv outputs.
//
// Memory-bound: 16-byte vectors (8 bf16 / 4 f32) per lane, consecutive lanes on consecutive
// channel groups so every wave reads and writes whole 128-byte lines.

#include "rmbx_common.h"

#include <cstdint>

namespace rmbx {
namespace {

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);                     // round to nearest even
  return (uint16_t)(u >> 16);
}

// storage-dtype traits: load 16 bytes as VEC floats, round a float to the storage dtype
struct BF16 {
  static constexpr int VEC = 8;
  using vec_t = uint4;
  __device__ static void unpack(const vec_t& v, float* f) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = bf2f((uint16_t)(w[i] & 0xffff));
      f[2 * i + 1] = bf2f((uint16_t)(w[i] >> 16));
    }
  }
  __device__ static vec_t pack(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ static float round(float f) { return bf2f(f2bf(f)); }
};

struct F32 {
  static constexpr int VEC = 4;
  using vec_t = float4;
  __device__ static void unpack(const vec_t& v, float* f) {
    f[0] = v.x;
    f[1] = v.y;
    f[2] = v.z;
    f[3] = v.w;
  }
  __device__ static vec_t pack(const float* f) { return make_float4(f[0], f[1], f[2], f[3]); }
  __device__ static float round(float f) { return f; }
};

// out = act( round( round(x + bias) + round(res + res_bias) ) ), all over [n_pix][C]
template <class T, bool RES, bool RES_BIAS, bool RELU>
__global__ void __launch_bounds__(256) bias_act_kernel(const typename T::vec_t* __restrict__ x,
                                                       const float* __restrict__ bias,
                                                       const typename T::vec_t* __restrict__ res,
                                                       const float* __restrict__ res_bias,
                                                       typename T::vec_t* __restrict__ out,
                                                       size_t n_vec, int cvec) {
#pragma clang fp contract(off)
  constexpr int V = T::VEC;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
    const int c0 = (int)(i % (size_t)cvec) * V;
    float a[V], r[V];
    T::unpack(x[i], a);
#pragma unroll
    for (int k = 0; k < V; ++k) a[k] = T::round(a[k] + bias[c0 + k]);
    if (RES) {
      T::unpack(res[i], r);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        float rv = RES_BIAS ? T::round(r[k] + res_bias[c0 + k]) : r[k];
        a[k] = T::round(a[k] + rv);
      }
    }
    if (RELU) {
#pragma unroll
      for (int k = 0; k < V; ++k) a[k] = a[k] > 0.f ? a[k] : (a[k] != a[k] ? a[k] : 0.f);
    }
    out[i] = T::pack(a);
  }
}

// out[n][ho][wo][c] = max over the 3x3 / stride-2 / pad-1 window of relu(round(x + bias)).
// Rounding and ReLU are monotone, so this equals relu(round(max(x) + bias)).
template <class T>
__global__ void __launch_bounds__(256) bias_relu_maxpool_kernel(const typename T::vec_t* __restrict__ x,
                                                                const float* __restrict__ bias,
                                                                typename T::vec_t* __restrict__ out,
                                                                int N, int H, int W, int cvec, int Ho,
                                                                int Wo) {
#pragma clang fp contract(off)
  constexpr int V = T::VEC;
  const size_t n_out = (size_t)N * Ho * Wo * cvec;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_out; i += stride) {
    const int cv = (int)(i % cvec);
    size_t p = i / cvec;
    const int wo = (int)(p % Wo);
    p /= Wo;
    const int ho = (int)(p % Ho);
    const int n = (int)(p / Ho);
    float m[V];
#pragma unroll
    for (int k = 0; k < V; ++k) m[k] = -INFINITY;
    bool nan[V] = {};
    for (int dy = -1; dy <= 1; ++dy) {
      const int h = 2 * ho + dy;
      if (h < 0 || h >= H) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int w = 2 * wo + dx;
        if (w < 0 || w >= W) continue;
        float v[V];
        T::unpack(x[(((size_t)n * H + h) * W + w) * cvec + cv], v);
#pragma unroll
        for (int k = 0; k < V; ++k) {
          nan[k] |= (v[k] != v[k]);
          m[k] = v[k] > m[k] ? v[k] : m[k];
        }
      }
    }
    const int c0 = cv * V;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float a = T::round(m[k] + bias[c0 + k]);
      a = a > 0.f ? a : 0.f;
      m[k] = nan[k] ? __builtin_nanf("") : a;
    }
    out[i] = T::pack(m);
  }
}

int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  const size_t cap = 256 * 64;  // grid-stride beyond 64 blocks per CU
  return (int)(g < cap ? (g > 0 ? g : 1) : cap);
}

template <class T>
int launch_bias_act(const void* x, const float* bias, const void* res, const float* res_bias, void* out,
                    size_t n_pix, int C, int relu, hipStream_t s) {
  using vt = typename T::vec_t;
  const int cvec = C / T::VEC;
  const size_t n_vec = n_pix * cvec;
  const int g = grid_for(n_vec);
  auto X = (const vt*)x;
  auto R = (const vt*)res;
  auto O = (vt*)out;
#define RMBX_BA(RES, RB, RELU) \
  hipLaunchKernelGGL((bias_act_kernel<T, RES, RB, RELU>), dim3(g), dim3(256), 0, s, X, bias, R, res_bias, O, n_vec, cvec)
  if (!res) {
    if (relu) RMBX_BA(false, false, true); else RMBX_BA(false, false, false);
  } else if (!res_bias) {
    if (relu) RMBX_BA(true, false, true); else RMBX_BA(true, false, false);
  } else {
    if (relu) RMBX_BA(true, true, true); else RMBX_BA(true, true, false);
  }
#undef RMBX_BA
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_nhwc_bias_act(const void* x, const float* bias, const void* res, const float* res_bias,
                                  void* out, size_t n_pix, int C, int relu, int dtype, void* stream) {
  RMBX_CHECK_ARG(x && bias && out, "rmbx_nhwc_bias_act: null pointer");
  RMBX_CHECK_ARG(dtype == 0 || dtype == 1, "rmbx_nhwc_bias_act: dtype must be 0 (f32) or 1 (bf16)");
  const int vec = dtype == 1 ? 8 : 4;
  RMBX_CHECK_ARG(C > 0 && C % vec == 0, "rmbx_nhwc_bias_act: C=%d must be a multiple of %d", C, vec);
  RMBX_CHECK_ARG(((uintptr_t)x | (uintptr_t)out | (uintptr_t)res) % 16 == 0,
                 "rmbx_nhwc_bias_act: tensors must be 16-byte aligned");
  if (n_pix == 0) return RMBX_OK;
  hipStream_t s = (hipStream_t)stream;
  return dtype == 1 ? rmbx::launch_bias_act<rmbx::BF16>(x, bias, res, res_bias, out, n_pix, C, relu, s)
                    : rmbx::launch_bias_act<rmbx::F32>(x, bias, res, res_bias, out, n_pix, C, relu, s);
}

extern "C" int rmbx_nhwc_bias_relu_maxpool(const void* x, const float* bias, void* out, int N, int H, int W,
                                           int C, int dtype, void* stream) {
  RMBX_CHECK_ARG(x && bias && out, "rmbx_nhwc_bias_relu_maxpool: null pointer");
  RMBX_CHECK_ARG(dtype == 0 || dtype == 1, "rmbx_nhwc_bias_relu_maxpool: bad dtype");
  const int vec = dtype == 1 ? 8 : 4;
  RMBX_CHECK_ARG(N >= 0 && H > 0 && W > 0 && C > 0 && C % vec == 0,
                 "rmbx_nhwc_bias_relu_maxpool: bad shape N=%d H=%d W=%d C=%d", N, H, W, C);
  RMBX_CHECK_ARG(((uintptr_t)x | (uintptr_t)out) % 16 == 0, "rmbx_nhwc_bias_relu_maxpool: unaligned");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;  // floor((H + 2 - 3) / 2) + 1
  if (N == 0) return RMBX_OK;
  hipStream_t s = (hipStream_t)stream;
  const int cvec = C / vec;
  const int g = rmbx::grid_for((size_t)N * Ho * Wo * cvec);
  if (dtype == 1)
    hipLaunchKernelGGL(rmbx::bias_relu_maxpool_kernel<rmbx::BF16>, dim3(g), dim3(256), 0, s,
                       (const uint4*)x, bias, (uint4*)out, N, H, W, cvec, Ho, Wo);
  else
    hipLaunchKernelGGL(rmbx::bias_relu_maxpool_kernel<rmbx::F32>, dim3(g), dim3(256), 0, s,
                       (const float4*)x, bias, (float4*)out, N, H, W, cvec, Ho, Wo);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

// ---------------------------------------------------------------------------------------------
// Residual add + LayerNorm of the ACT transformer (post-norm layers: norm(x + sublayer(x))),
// one wavefront per token row, the row held in registers (D <= 1024): s = rnd(x + r) in the
// storage dtype (the unfused add), mean and variance in f32 over s (two passes over registers),
// y = rnd((s - mean) * rstd * w + b).  Replaces the add + nn.LayerNorm pair of
// EncoderLayer/DecoderLayer (ACT transformer.py, third_party/act [absent]).
// ---------------------------------------------------------------------------------------------
namespace rmbx {
namespace {

template <class T, int PER>
__global__ void __launch_bounds__(256) add_layernorm_kernel(const typename T::vec_t* __restrict__ x,
                                                            const typename T::vec_t* __restrict__ r,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            typename T::vec_t* __restrict__ out, int rows, int D,
                                                            float eps, const typename T::vec_t* __restrict__ pos,
                                                            int pos_rows, typename T::vec_t* __restrict__ out_pos) {
  constexpr int V = T::VEC;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = D / V;
  const size_t base = (size_t)row * nvec;
  float s[PER][V];
  float sum = 0.f;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int v = lane + q * 64;
    if (v < nvec) {
      float a[V], c[V];
      T::unpack(x[base + v], a);
      if (r) {
        T::unpack(r[base + v], c);
#pragma unroll
        for (int k = 0; k < V; ++k) a[k] = T::round(a[k] + c[k]);
      }
#pragma unroll
      for (int k = 0; k < V; ++k) {
        s[q][k] = a[k];
        sum += a[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) s[q][k] = 0.f;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
  const float mean = sum / (float)D;
  float var = 0.f;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int v = lane + q * 64;
    if (v < nvec) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float d = s[q][k] - mean;
        var += d * d;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) var += __shfl_xor(var, off);
  const float rstd = rsqrtf(var / (float)D + eps);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const int v = lane + q * 64;
    if (v < nvec) {
      float y[V];
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const int c = v * V + k;
        y[k] = (s[q][k] - mean) * rstd * w[c] + b[c];
      }
      const typename T::vec_t yv = T::pack(y);
      out[base + v] = yv;
      if (out_pos) {
        // the next attention's query input: rnd(y + pos[row % pos_rows]) on the rounded y, as the
        // separate `x + pos` of the unfused module computes it
        float yr[V], pv[V];
        T::unpack(yv, yr);
        T::unpack(pos[(size_t)(row % pos_rows) * nvec + v], pv);
#pragma unroll
        for (int k = 0; k < V; ++k) yr[k] = yr[k] + pv[k];
        out_pos[base + v] = T::pack(yr);
      }
    }
  }
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_add_layernorm_pos(const void* x, const void* r, const float* weight, const float* bias, void* out,
                                      const void* pos, int pos_rows, void* out_pos, int rows, int D, float eps,
                                      int dtype, void* stream);

extern "C" int rmbx_add_layernorm(const void* x, const void* r, const float* weight, const float* bias, void* out,
                                  int rows, int D, float eps, int dtype, void* stream) {
  return rmbx_add_layernorm_pos(x, r, weight, bias, out, nullptr, 0, nullptr, rows, D, eps, dtype, stream);
}

extern "C" int rmbx_add_layernorm_pos(const void* x, const void* r, const float* weight, const float* bias, void* out,
                                      const void* pos, int pos_rows, void* out_pos, int rows, int D, float eps,
                                      int dtype, void* stream) {
  RMBX_CHECK_ARG(!out_pos || (pos && pos_rows > 0), "rmbx_add_layernorm_pos: out_pos needs pos and pos_rows > 0");
  RMBX_CHECK_ARG(((uintptr_t)pos | (uintptr_t)out_pos) % 16 == 0, "rmbx_add_layernorm_pos: unaligned");
  RMBX_CHECK_ARG(x && weight && bias && out, "rmbx_add_layernorm: null pointer");
  RMBX_CHECK_ARG(dtype == 0 || dtype == 1, "rmbx_add_layernorm: dtype must be 0 (f32) or 1 (bf16)");
  const int vec = dtype == 1 ? 8 : 4;
  RMBX_CHECK_ARG(D > 0 && D % vec == 0 && D <= 2048, "rmbx_add_layernorm: D=%d must be a multiple of %d, <= 2048",
                 D, vec);
  RMBX_CHECK_ARG(((uintptr_t)x | (uintptr_t)r | (uintptr_t)out) % 16 == 0, "rmbx_add_layernorm: unaligned");
  if (rows <= 0) return RMBX_OK;
  hipStream_t s = (hipStream_t)stream;
  const int grid = (rows + 3) / 4;
  const int nvec = D / vec;
  if (dtype == 1) {
    if (nvec <= 64)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::BF16, 1>), dim3(grid), dim3(256), 0, s, (const uint4*)x,
                         (const uint4*)r, weight, bias, (uint4*)out, rows, D, eps, (const uint4*)pos, pos_rows,
                         (uint4*)out_pos);
    else if (nvec <= 128)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::BF16, 2>), dim3(grid), dim3(256), 0, s, (const uint4*)x,
                         (const uint4*)r, weight, bias, (uint4*)out, rows, D, eps, (const uint4*)pos, pos_rows,
                         (uint4*)out_pos);
    else
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::BF16, 4>), dim3(grid), dim3(256), 0, s, (const uint4*)x,
                         (const uint4*)r, weight, bias, (uint4*)out, rows, D, eps, (const uint4*)pos, pos_rows,
                         (uint4*)out_pos);
  } else {
    if (nvec <= 64)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 1>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos);
    else if (nvec <= 128)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 2>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos);
    else if (nvec <= 256)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 4>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos);
    else
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 8>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
