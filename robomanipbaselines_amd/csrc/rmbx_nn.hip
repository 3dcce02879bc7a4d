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
#include <type_traits>

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

// optional pre-split outputs (f32 only, rmbx_add_layernorm_split): planes u16 [2][rows][D]
struct LnSplit {
  uint16_t* y_planes;
  float* y_rinv;
  uint16_t* pos_planes;
  float* pos_rinv;
  int rows;
  float* y_norm;  // an upper bound of each row's Euclidean norm |y|_2 (nullable)
};

template <class T, int PER>
__global__ void __launch_bounds__(256) add_layernorm_kernel(const typename T::vec_t* __restrict__ x,
                                                            const typename T::vec_t* __restrict__ r,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            typename T::vec_t* __restrict__ out, int rows, int D,
                                                            float eps, const typename T::vec_t* __restrict__ pos,
                                                            int pos_rows, typename T::vec_t* __restrict__ out_pos,
                                                            LnSplit sp) {
  constexpr int V = T::VEC;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = D / V;
  const size_t base = (size_t)row * nvec;
  float s[PER][V], s2[PER][V];
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
  float ymax = 0.f, pmax = 0.f, ysq = 0.f;  // f32 split outputs: the rows' max |y|, max |y + pos|, sum y^2
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
      if (out) out[base + v] = yv;
      float yr[V];
      T::unpack(yv, yr);
      if (sp.y_planes) {
#pragma unroll
        for (int k = 0; k < V; ++k) ymax = fmaxf(ymax, fabsf(yr[k]));
      }
      if (sp.y_norm) {
#pragma unroll
        for (int k = 0; k < V; ++k) ysq += yr[k] * yr[k];
      }
      if (out_pos || sp.pos_planes) {
        // the next attention's query input: rnd(y + pos[row % pos_rows]) on the rounded y, as the
        // separate `x + pos` of the unfused module computes it
        float pv[V];
        T::unpack(pos[(size_t)(row % pos_rows) * nvec + v], pv);
#pragma unroll
        for (int k = 0; k < V; ++k) yr[k] = yr[k] + pv[k];
        const typename T::vec_t pvv = T::pack(yr);
        if (out_pos) out_pos[base + v] = pvv;
        if (sp.pos_planes) {
          T::unpack(pvv, yr);
#pragma unroll
          for (int k = 0; k < V; ++k) pmax = fmaxf(pmax, fabsf(yr[k]));
        }
      }
      // keep the (rounded) values for the split pass: y in s, y + pos in s2
      {
        float t[V];
        T::unpack(yv, t);
#pragma unroll
        for (int k = 0; k < V; ++k) s[q][k] = t[k];
      }
      if (sp.pos_planes) {
#pragma unroll
        for (int k = 0; k < V; ++k) s2[q][k] = yr[k];
      }
    }
  }
  if constexpr (std::is_same<T, F32>::value) {
    // the f16x3 GEMM's pre-split A (rmbx_linear_f16x3_presplit): a' = a 2^t with the row's max |a'|
    // in [2^13, 2^14), hi = f16(a'), lo = f16(a' - hi), and 2^-t per row
    auto split_row = [&](float (*vals)[V], float mx, uint16_t* planes, float* rinv) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
      int e = 14;
      if (mx > 0.f && mx <= 3.4e38f) frexpf(mx, &e);  // mx = f 2^e, f in [0.5, 1); NaN / inf: scale 1
      const float sc = ldexpf(1.f, 14 - e);
      if (lane == 0) rinv[row] = ldexpf(1.f, e - 14);
      const size_t plane = (size_t)sp.rows * D;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int v = lane + q * 64;
        if (v < nvec) {
          uint16_t h[V], l[V];
#pragma unroll
          for (int k = 0; k < V; ++k) {
            const float a = vals[q][k] * sc;
            const _Float16 hv = (_Float16)a;
            h[k] = __builtin_bit_cast(uint16_t, hv);
            l[k] = __builtin_bit_cast(uint16_t, (_Float16)(a - (float)hv));
          }
          static_assert(V == 4, "f32 rows move as float4");
          const size_t o = (size_t)row * D + (size_t)v * V;
          *(uint2*)(planes + o) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
          *(uint2*)(planes + plane + o) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
        }
      }
    };
    if (sp.y_norm) {
      // |y|_2 from an f32 sum of squares: relative rounding <= ~D 2^-24, covered 2^-12 over
      float q = ysq;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
      if (lane == 0) sp.y_norm[row] = sqrtf(q) * (1.f + 0.000244140625f);
    }
    if (sp.y_planes) split_row(s, ymax, sp.y_planes, sp.y_rinv);
    if (sp.pos_planes) split_row(s2, pmax, sp.pos_planes, sp.pos_rinv);
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

namespace {
int add_layernorm_impl(const void* x, const void* r, const float* weight, const float* bias, void* out,
                       const void* pos, int pos_rows, void* out_pos, int rows, int D, float eps, int dtype,
                       void* stream, rmbx::LnSplit sp) {
  RMBX_CHECK_ARG(!(out_pos || sp.pos_planes) || (pos && pos_rows > 0),
                 "rmbx_add_layernorm_pos: out_pos needs pos and pos_rows > 0");
  RMBX_CHECK_ARG(((uintptr_t)pos | (uintptr_t)out_pos) % 16 == 0, "rmbx_add_layernorm_pos: unaligned");
  RMBX_CHECK_ARG(x && weight && bias && (out || sp.y_planes || sp.pos_planes), "rmbx_add_layernorm: null pointer");
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
                         (uint4*)out_pos, sp);
    else if (nvec <= 128)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::BF16, 2>), dim3(grid), dim3(256), 0, s, (const uint4*)x,
                         (const uint4*)r, weight, bias, (uint4*)out, rows, D, eps, (const uint4*)pos, pos_rows,
                         (uint4*)out_pos, sp);
    else
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::BF16, 4>), dim3(grid), dim3(256), 0, s, (const uint4*)x,
                         (const uint4*)r, weight, bias, (uint4*)out, rows, D, eps, (const uint4*)pos, pos_rows,
                         (uint4*)out_pos, sp);
  } else {
    if (nvec <= 64)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 1>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos, sp);
    else if (nvec <= 128)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 2>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos, sp);
    else if (nvec <= 256)
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 4>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos, sp);
    else
      hipLaunchKernelGGL((rmbx::add_layernorm_kernel<rmbx::F32, 8>), dim3(grid), dim3(256), 0, s, (const float4*)x,
                         (const float4*)r, weight, bias, (float4*)out, rows, D, eps, (const float4*)pos, pos_rows,
                         (float4*)out_pos, sp);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
}  // namespace

extern "C" int rmbx_add_layernorm_pos(const void* x, const void* r, const float* weight, const float* bias, void* out,
                                      const void* pos, int pos_rows, void* out_pos, int rows, int D, float eps,
                                      int dtype, void* stream) {
  return add_layernorm_impl(x, r, weight, bias, out, pos, pos_rows, out_pos, rows, D, eps, dtype, stream,
                            rmbx::LnSplit{nullptr, nullptr, nullptr, nullptr, rows, nullptr});
}

extern "C" int rmbx_add_layernorm_split(const float* x, const float* r, const float* weight, const float* bias,
                                        float* out, void* y_planes, float* y_rinv, float* y_norm, const float* pos,
                                        int pos_rows, float* out_pos, void* pos_planes, float* pos_rinv, int rows, int D,
                                        float eps, void* stream) {
  RMBX_CHECK_ARG(!y_planes == !y_rinv && !pos_planes == !pos_rinv, "rmbx_add_layernorm_split: planes need their rinv");
  RMBX_CHECK_ARG(D % 4 == 0 && ((uintptr_t)y_planes | (uintptr_t)pos_planes) % 8 == 0,
                 "rmbx_add_layernorm_split: D %% 4 and 8-byte aligned planes");
  return add_layernorm_impl(x, r, weight, bias, out, pos, pos_rows, out_pos, rows, D, eps, 0, stream,
                            rmbx::LnSplit{(uint16_t*)y_planes, y_rinv, (uint16_t*)pos_planes, pos_rinv, rows, y_norm});
}

// ---------------------------------------------------------------------------------------------
// GroupNorm (+ Mish) of the DiffusionPolicy / DP3 UNet's Conv1dBlock (nn.GroupNorm(G, C) ->
// nn.Mish() after each Conv1d, policy/diffusion/unet1d.py; the reference's diffusion_policy
// ConditionalUnet1D, third_party [absent]) on [B][C][T] f32: the channels of a group are one
// contiguous span of (C / G) T values, so one 256-thread block per (b, g) reduces it (sum, then
// the sum of squared deviations: two passes over the span, which stays in L1 / L2), and writes
// y = (x - mean) rstd gamma_c + beta_c, optionally mish(y) = y tanh(log1p(exp y)) (torch's form).
// The input may also be the conv GEMM's [B][T][C] rows (flags bit 1): the transpose to [B][C][T]
// then happens in this pass instead of a separate copy.
// One read pass more than the statistics need, against torch's moments kernel + affine kernel +
// Mish kernel (three reads, two writes).
// ---------------------------------------------------------------------------------------------
namespace rmbx {
namespace {

__device__ __forceinline__ float gn_block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wave = threadIdx.x >> 6;
  __syncthreads();  // (red is reused by the next reduction)
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

constexpr int GN_REG = 8;  // values per thread held in registers (spans up to 2048)
// TIN: x is [B][T][C] (the conv GEMM's output rows; element i of a (b, g) span read t-major, i = t cg + c,
// so a wave's loads are contiguous channels); y is [B][C][T] either way
template <bool MISH, bool TIN>
__global__ void __launch_bounds__(256) groupnorm_act_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ b, float* __restrict__ y, int C,
                                                            int T, int G, float eps) {
  __shared__ float red[4];
  const int bg = blockIdx.x, g = bg % G, cg = C / G;
  const int E = cg * T, tid = threadIdx.x;
  const long long bb = bg / G;
  // element i of the span: channel c, time t, its input offset; the output offset is c T + t
  auto at = [&](int i, int& c, int& t) -> long long {
    if constexpr (TIN) {
      t = i / cg;
      c = i - t * cg;
      return (bb * T + t) * C + g * cg + c;
    } else {
      c = i / T;
      t = i - c * T;
      return (long long)bg * E + i;
    }
  };
  float* ys = y + (long long)bg * E;
  if (E <= 256 * GN_REG) {  // the UNet's spans (512-2048 values): one read, the values kept in registers
    float v[GN_REG];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < GN_REG; ++k) {
      const int i = tid + 256 * k;
      int c, t;
      v[k] = i < E ? x[at(i, c, t)] : 0.f;
      s += v[k];
    }
    const float mean = gn_block_sum(s, red) / (float)E;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < GN_REG; ++k) {
      const int i = tid + 256 * k;
      const float d = i < E ? v[k] - mean : 0.f;
      q += d * d;
    }
    const float rstd = 1.f / sqrtf(gn_block_sum(q, red) / (float)E + eps);
#pragma unroll
    for (int k = 0; k < GN_REG; ++k) {
      const int i = tid + 256 * k;
      if (i < E) {
        int c, t;
        at(i, c, t);
        float o = (v[k] - mean) * rstd * w[g * cg + c] + b[g * cg + c];
        if constexpr (MISH) o = o * tanhf(log1pf(expf(o)));
        ys[c * T + t] = o;
      }
    }
    return;
  }
  float s = 0.f;
  for (int i = tid; i < E; i += 256) {
    int c, t;
    s += x[at(i, c, t)];
  }
  const float mean = gn_block_sum(s, red) / (float)E;
  float q = 0.f;
  for (int i = tid; i < E; i += 256) {
    int c, t;
    const float d = x[at(i, c, t)] - mean;
    q += d * d;
  }
  const float var = gn_block_sum(q, red) / (float)E;
  const float rstd = 1.f / sqrtf(var + eps);
  for (int i = tid; i < E; i += 256) {
    int c, t;
    const long long off = at(i, c, t);
    float v = (x[off] - mean) * rstd * w[g * cg + c] + b[g * cg + c];
    if constexpr (MISH) v = v * tanhf(log1pf(expf(v)));
    ys[c * T + t] = v;
  }
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_groupnorm_act(const float* x, const float* weight, const float* bias, float* out, int B, int C,
                                  int T, int groups, float eps, int mish, void* stream) {
  RMBX_CHECK_ARG(x && weight && bias && out, "rmbx_groupnorm_act: null pointer");
  RMBX_CHECK_ARG(B >= 0 && C > 0 && T > 0 && groups > 0 && C % groups == 0,
                 "rmbx_groupnorm_act: bad shape B=%d C=%d T=%d groups=%d", B, C, T, groups);
  RMBX_CHECK_ARG(eps >= 0.f, "rmbx_groupnorm_act: eps must be >= 0");
  const long long nblocks = (long long)B * groups;
  RMBX_CHECK_ARG(nblocks < (1ll << 31) && (long long)(C / groups) * T < (1ll << 31), "rmbx_groupnorm_act: too large");
  if (B == 0) return RMBX_OK;
  RMBX_CHECK_ARG(!(mish & 2) || x != out, "rmbx_groupnorm_act: a time-major input cannot alias the output");
  const dim3 grid((unsigned)nblocks), blk(256);
  hipStream_t st = (hipStream_t)stream;
  switch (mish & 3) {
    case 0: hipLaunchKernelGGL((rmbx::groupnorm_act_kernel<false, false>), grid, blk, 0, st, x, weight, bias, out, C, T, groups, eps); break;
    case 1: hipLaunchKernelGGL((rmbx::groupnorm_act_kernel<true, false>), grid, blk, 0, st, x, weight, bias, out, C, T, groups, eps); break;
    case 2: hipLaunchKernelGGL((rmbx::groupnorm_act_kernel<false, true>), grid, blk, 0, st, x, weight, bias, out, C, T, groups, eps); break;
    default: hipLaunchKernelGGL((rmbx::groupnorm_act_kernel<true, true>), grid, blk, 0, st, x, weight, bias, out, C, T, groups, eps);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
