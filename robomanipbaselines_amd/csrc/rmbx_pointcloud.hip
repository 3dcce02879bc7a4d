// Point-cloud observation of the 3D diffusion policy, batched: depth + rgb -> points ->
// bounding-box crop -> farthest point sampling -> normalisation, one workgroup per env.
//
// Replaces RolloutDiffusionPolicy3d.get_pointcloud
// (policy/diffusion_policy_3d/RolloutDiffusionPolicy3d.py:132-160) after the cv2.resize of the
// images: convert_depth_image_to_pointcloud (common/utils/VisionUtils.py:55-87, no clip limits
// -> keep 0 < d < inf), crop_pointcloud_bb (common/utils/Vision3dUtils.py:6-14, strict bounds),
// downsample_pointcloud_fps (Vision3dUtils.py:17-25 -> pytorch3d sample_farthest_points, start
// index 0, on the points converted to f32) and normalize_data (common/utils/DataUtils.py:9-24).
//
// Arithmetic follows the reference's dtypes: pixel grid in f32, the division by the focal
// scaling and everything after it in f64 (NumPy promotes with the f64 scalar), colours
// u8 -> f32 / 255, FPS squared distances in f32 accumulated over all 6 channels in order,
// running minimum, strict-greater argmax (lowest index wins ties; an all-zero round picks
// point 0), fewer kept points than K -> the remaining slots repeat the last kept point (the
// -1 index of pytorch3d, applied as a NumPy index).  The crop keeps pixel order, so indices in
// the cropped cloud order like pixel indices and no compaction pass is needed: each lane keeps
// its pixels' points in registers for the whole FPS loop.
//
// Mapping: 1024 threads (16 waves) per env, pixel p owned by lane p % 1024 (<= 8 per lane),
// one (value, index) block reduction per FPS step (wave shuffles + 16-entry LDS pass).

#include "rmbx_common.h"

#include <cfloat>
#include <cstdint>

namespace rmbx {
namespace {

constexpr int PC_THREADS = 1024;
constexpr int PC_PPT = 8;  // pixels per thread -> image <= 8192 pixels
constexpr int PC_WAVES = PC_THREADS / 64;

struct PcArgs {
  const float* depth;  // [n][H][W]
  const uint8_t* rgb;  // [n][H][W][3]
  int n_env, H, W, K;
  double focal;        // focal scaling (1 / tan(fovy / 2)) * H / 2, evaluated on the host
  double lo[3], hi[3];
  int has_lo, has_hi;
  int norm_type;       // 0 gaussian: (x - a) / b ; 1 limits: b * (x - a) + c
  double na[6], nb[6], nc[6];
  float* out;          // [n][K][6] normalised f32
  double* raw;         // [n][K][6] f64 before normalisation (optional)
  int32_t* count;      // [n] points after the crop
};

__device__ __forceinline__ void pixel_point(const PcArgs& a, int e, int p, double* v, bool* keep) {
#pragma clang fp contract(off)
  const int i = p / a.W, j = p % a.W;
  const float d32 = a.depth[(size_t)e * a.H * a.W + p];
  const float gi = (float)i - 0.5f * (float)a.H;
  const float gj = (float)j - 0.5f * (float)a.W;
  const double d = (double)d32;
  v[0] = ((double)gj / a.focal) * d;
  v[1] = ((double)gi / a.focal) * d;
  v[2] = d;
  const uint8_t* c = a.rgb + ((size_t)e * a.H * a.W + p) * 3;
  for (int k = 0; k < 3; ++k) v[3 + k] = (double)((float)c[k] / 255.0f);
  bool k0 = (0.0f < d32) && (d32 < INFINITY);
  if (a.has_lo) k0 = k0 && v[0] > a.lo[0] && v[1] > a.lo[1] && v[2] > a.lo[2];
  if (a.has_hi) k0 = k0 && v[0] < a.hi[0] && v[1] < a.hi[1] && v[2] < a.hi[2];
  *keep = k0;
}

// block-wide reduction: max value, lowest index among equal values
__device__ __forceinline__ void block_argmax(float& val, int& idx, float* s_val, int* s_idx) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(val, off);
    const int oi = __shfl_xor(idx, off);
    if (ov > val || (ov == val && oi < idx)) {
      val = ov;
      idx = oi;
    }
  }
  if (lane == 0) {
    s_val[wv] = val;
    s_idx[wv] = idx;
  }
  __syncthreads();
  if (wv == 0) {
    val = lane < PC_WAVES ? s_val[lane] : -FLT_MAX;
    idx = lane < PC_WAVES ? s_idx[lane] : 0x7fffffff;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(val, off);
      const int oi = __shfl_xor(idx, off);
      if (ov > val || (ov == val && oi < idx)) {
        val = ov;
        idx = oi;
      }
    }
    if (lane == 0) {
      s_val[PC_WAVES] = val;
      s_idx[PC_WAVES] = idx;
    }
  }
  __syncthreads();
  val = s_val[PC_WAVES];
  idx = s_idx[PC_WAVES];
}

__device__ __forceinline__ void emit(const PcArgs& a, int e, int k, int p) {
#pragma clang fp contract(off)
  double v[6];
  bool keep;
  pixel_point(a, e, p, v, &keep);
  const size_t o = ((size_t)e * a.K + k) * 6;
  for (int c = 0; c < 6; ++c) {
    double y;
    if (a.norm_type == 0) {
      y = (v[c] - a.na[c]) / a.nb[c];
    } else {
      const double t = v[c] - a.na[c];
      y = a.nb[c] * t + a.nc[c];
    }
    a.out[o + c] = (float)y;
    if (a.raw) a.raw[o + c] = v[c];
  }
}

__global__ void __launch_bounds__(PC_THREADS) pointcloud_fps_kernel(PcArgs a) {
#pragma clang fp contract(off)
  const int e = blockIdx.x;
  const int tid = threadIdx.x;
  const int npix = a.H * a.W;
  __shared__ float s_val[PC_WAVES + 1];
  __shared__ int s_idx[PC_WAVES + 1];
  __shared__ float s_sel[6];

  float pt[PC_PPT][6];
  float dist[PC_PPT];
  bool kept[PC_PPT];
  int n_kept = 0, first = 0x7fffffff, last = -1;
#pragma unroll
  for (int s = 0; s < PC_PPT; ++s) {
    const int p = tid + s * PC_THREADS;
    kept[s] = false;
    dist[s] = FLT_MAX;
    if (p < npix) {
      double v[6];
      bool keep;
      pixel_point(a, e, p, v, &keep);
      kept[s] = keep;
#pragma unroll
      for (int c = 0; c < 6; ++c) pt[s][c] = (float)v[c];
      if (keep) {
        ++n_kept;
        first = p < first ? p : first;
        last = p > last ? p : last;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 6; ++c) pt[s][c] = 0.f;
    }
  }
  // totals: count, first kept, last kept (sum / min / max via the argmax reduction)
  float fv = (float)n_kept;
  {
    // sum of counts
    float v = fv;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((tid & 63) == 0) s_val[tid >> 6] = v;
    __syncthreads();
    float tot = 0.f;
    for (int w = 0; w < PC_WAVES; ++w) tot += s_val[w];
    __syncthreads();
    fv = tot;
  }
  const int total = (int)fv;
  int first_kept = first;
  {
    float v0 = 0.f;
    int i0 = first;
    block_argmax(v0, i0, s_val, s_idx);  // equal values -> lowest index = first kept pixel
    first_kept = i0;
  }
  int last_kept;
  {
    float v0 = 0.f;
    int i0 = -last;  // lowest of -last = highest last
    block_argmax(v0, i0, s_val, s_idx);
    last_kept = -i0;
  }
  if (tid == 0) a.count[e] = total;
  if (total == 0) {
    // empty cloud (the reference raises IndexError): emit zeros
    for (int k = tid; k < a.K * 6; k += PC_THREADS) {
      a.out[(size_t)e * a.K * 6 + k] = 0.f;
      if (a.raw) a.raw[(size_t)e * a.K * 6 + k] = 0.0;
    }
    return;
  }
  const int kn = a.K < total ? a.K : total;
  int sel = first_kept;
  for (int k = 0; k < kn; ++k) {
    if (tid == (sel % PC_THREADS)) {
      const int s = sel / PC_THREADS;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < PC_PPT; ++q)
          if (q == s) v = pt[q][c];
        s_sel[c] = v;
      }
      emit(a, e, k, sel);
    }
    __syncthreads();
    float sv[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) sv[c] = s_sel[c];
    float best = 0.f;
    int bi = 0x7fffffff;
#pragma unroll
    for (int s = 0; s < PC_PPT; ++s) {
      if (!kept[s]) continue;
      float d2 = 0.f;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const float diff = sv[c] - pt[s][c];
        const float sq = diff * diff;
        d2 = d2 + sq;
      }
      const float md = dist[s] < d2 ? dist[s] : d2;  // std::min(dist2, dist)
      dist[s] = md;
      const int p = tid + s * PC_THREADS;
      if (md > best || (md == best && md > 0.f && p < bi)) {
        best = md;
        bi = p;
      }
    }
    if (bi == 0x7fffffff) best = 0.f;
    block_argmax(best, bi, s_val, s_idx);
    sel = (best > 0.f && bi != 0x7fffffff) ? bi : first_kept;
  }
  // fewer kept points than K: pytorch3d leaves -1 indices -> NumPy picks the last kept point
  for (int k = kn + tid; k < a.K; k += PC_THREADS) emit(a, e, k, last_kept);
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_pointcloud_fps(const float* depth, const uint8_t* rgb, int n_env, int H, int W,
                                   double focal_scaling, const double* min_bound, const double* max_bound,
                                   int K, int norm_type, const double* norm_a, const double* norm_b,
                                   const double* norm_c, float* out, double* raw, int32_t* count,
                                   void* stream) {
  RMBX_CHECK_ARG(depth && rgb && out && count && norm_a && norm_b, "rmbx_pointcloud_fps: null pointer");
  RMBX_CHECK_ARG(H > 0 && W > 0 && (long)H * W <= (long)rmbx::PC_THREADS * rmbx::PC_PPT,
                 "rmbx_pointcloud_fps: image %dx%d exceeds %d pixels", W, H, rmbx::PC_THREADS * rmbx::PC_PPT);
  RMBX_CHECK_ARG(K > 0, "rmbx_pointcloud_fps: K must be positive");
  RMBX_CHECK_ARG(norm_type == 0 || (norm_type == 1 && norm_c), "rmbx_pointcloud_fps: bad normalisation");
  if (n_env == 0) return RMBX_OK;
  rmbx::PcArgs a{};
  a.depth = depth;
  a.rgb = rgb;
  a.n_env = n_env;
  a.H = H;
  a.W = W;
  a.K = K;
  a.focal = focal_scaling;
  a.has_lo = min_bound != nullptr;
  a.has_hi = max_bound != nullptr;
  for (int k = 0; k < 3; ++k) {
    a.lo[k] = min_bound ? min_bound[k] : 0.0;
    a.hi[k] = max_bound ? max_bound[k] : 0.0;
  }
  a.norm_type = norm_type;
  for (int c = 0; c < 6; ++c) {
    a.na[c] = norm_a[c];
    a.nb[c] = norm_b[c];
    a.nc[c] = norm_c ? norm_c[c] : 0.0;
  }
  a.out = out;
  a.raw = raw;
  a.count = count;
  hipLaunchKernelGGL(rmbx::pointcloud_fps_kernel, dim3(n_env), dim3(rmbx::PC_THREADS), 0, (hipStream_t)stream, a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
