// Batched camera rendering by ray casting scene primitives (gfx950).
//
// Replaces the per-env, per-camera OpenGL OffScreenViewer rgb + depth renders of
// envs/mujoco/MujocoEnvBase.py:112-126.  One 256-thread workgroup renders a 16x16 pixel tile of
// one env: the workgroup transforms that env's primitives into the camera frame into LDS,
// culls them against the tile's view frustum slice (projected bounding spheres), and every lane
// casts its pixel's ray against the surviving list.  Shading: ambient + headlight + one
// directional light (the scene's <light> and MuJoCo's default headlight), material colour only
// (textures are not sampled).  Outputs are written once per pixel: u8 HWC RGB, f32 linear
// depth, and/or the policy input tensor (CHW, ImageNet-normalised, bf16 or f32) fused so the
// policy never re-reads the u8 image.

#include <hip/hip_bf16.h>

#include "rmbx_common.h"

#include <cstdlib>
#include "rmbx_math.h"
#include "rmbx_model.h"

namespace rmbx {

#define RENDER_TILE 16
#define MAX_PRIM 128

struct PrimCam {
  float c[3];    // centre in camera frame
  float R[9];    // geom axes in camera frame (columns = local axes)
  float s[3];    // size
  float rgb[3];
  int type;
  float rad;   // bounding radius (0 = unbounded)
  float zmin;  // lower bound of any hit's depth (camera z) in the image; -1e30 if unbounded
  float ol[3];  // the camera (ray origin) in the primitive's local frame: R^T (0 - c)
};

__device__ __forceinline__ float dot3f(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// world->camera: R_cam (columns = camera axes in world), p_cam
struct CamFrame {
  float R[9];
  float p[3];
};

// ray (origin 0, direction d) intersections in the primitive's local frame ------------------
__device__ __forceinline__ void to_local(const PrimCam& P, const float* d, float* o_l, float* d_l) {
  // local = R^T (x - c); the origin (the camera) is transformed once per primitive (P.ol)
  for (int i = 0; i < 3; i++) {
    o_l[i] = P.ol[i];
    d_l[i] = P.R[i] * d[0] + P.R[3 + i] * d[1] + P.R[6 + i] * d[2];
  }
}

__device__ bool hit_sphere(const float* o, const float* d, float r, float* t, float* n) {
  const float b = dot3f(o, d);
  const float c = dot3f(o, o) - r * r;
  if (c < 0) return false;  // camera inside: not rendered (OpenGL back-face culling)
  const float a = dot3f(d, d);
  const float disc = b * b - a * c;
  if (disc < 0) return false;
  const float sq = sqrtf(disc);
  float tt = (-b - sq) / a;
  if (tt <= 1e-4f) tt = (-b + sq) / a;
  if (tt <= 1e-4f) return false;
  *t = tt;
  for (int i = 0; i < 3; i++) n[i] = (o[i] + tt * d[i]) / r;
  return true;
}

// finite cylinder along local z, radius r, half-height h; caps optional (capsule uses spheres)
__device__ bool hit_cylinder(const float* o, const float* d, float r, float h, bool caps,
                             float* t, float* n) {
  float best = 1e30f;
  bool hit = false;
  if (o[0] * o[0] + o[1] * o[1] < r * r && fabsf(o[2]) < h + (caps ? 0.f : r)) return false;  // inside
  const float a = d[0] * d[0] + d[1] * d[1];
  if (a > 1e-12f) {
    const float b = o[0] * d[0] + o[1] * d[1];
    const float c = o[0] * o[0] + o[1] * o[1] - r * r;
    const float disc = b * b - a * c;
    if (disc >= 0) {
      const float sq = sqrtf(disc);
      for (int k = 0; k < 2; k++) {
        const float tt = (-b + (k == 0 ? -sq : sq)) / a;
        if (tt > 1e-4f && tt < best) {
          const float z = o[2] + tt * d[2];
          if (fabsf(z) <= h) {
            best = tt;
            n[0] = (o[0] + tt * d[0]) / r;
            n[1] = (o[1] + tt * d[1]) / r;
            n[2] = 0;
            hit = true;
          }
        }
      }
    }
  }
  if (caps && fabsf(d[2]) > 1e-12f) {
    for (int k = 0; k < 2; k++) {
      const float zc = k == 0 ? h : -h;
      const float tt = (zc - o[2]) / d[2];
      if (tt > 1e-4f && tt < best) {
        const float x = o[0] + tt * d[0], y = o[1] + tt * d[1];
        if (x * x + y * y <= r * r) {
          best = tt;
          n[0] = 0;
          n[1] = 0;
          n[2] = k == 0 ? 1.f : -1.f;
          hit = true;
        }
      }
    }
  }
  *t = best;
  return hit;
}

__device__ bool hit_capsule(const float* o, const float* d, float r, float h, float* t, float* n) {
  float tb, nb[3];
  bool hit = hit_cylinder(o, d, r, h, false, &tb, nb);
  float best = hit ? tb : 1e30f;
  if (hit) {
    n[0] = nb[0];
    n[1] = nb[1];
    n[2] = nb[2];
  }
  for (int k = 0; k < 2; k++) {
    const float oc[3] = {o[0], o[1], o[2] - (k == 0 ? h : -h)};
    float ts, ns[3];
    if (hit_sphere(oc, d, r, &ts, ns) && ts < best) {
      const float z = oc[2] + ts * d[2];
      if ((k == 0 && z >= 0) || (k == 1 && z <= 0)) {
        best = ts;
        n[0] = ns[0];
        n[1] = ns[1];
        n[2] = ns[2];
        hit = true;
      }
    }
  }
  *t = best;
  return hit;
}

__device__ bool hit_box(const float* o, const float* d, const float* s, float* t, float* n) {
  float tmin = -1e30f, tmax = 1e30f;
  int axis = 0;
  for (int i = 0; i < 3; i++) {
    if (fabsf(d[i]) < 1e-12f) {
      if (fabsf(o[i]) > s[i]) return false;
      continue;
    }
    const float inv = 1.0f / d[i];
    float t1 = (-s[i] - o[i]) * inv, t2 = (s[i] - o[i]) * inv;
    if (t1 > t2) {
      const float tmp = t1;
      t1 = t2;
      t2 = tmp;
    }
    if (t1 > tmin) {
      tmin = t1;
      axis = i;
    }
    if (t2 < tmax) tmax = t2;
    if (tmin > tmax) return false;
  }
  if (tmax <= 1e-4f) return false;
  if (tmin <= 1e-4f) return false;  // camera inside the box: ignore
  *t = tmin;
  n[0] = n[1] = n[2] = 0;
  n[axis] = d[axis] > 0 ? -1.f : 1.f;  // entry face
  return true;
}

__device__ bool hit_plane(const float* o, const float* d, float* t, float* n) {
  if (fabsf(d[2]) < 1e-12f) return false;
  const float tt = -o[2] / d[2];
  if (tt <= 1e-4f) return false;
  *t = tt;
  n[0] = 0;
  n[1] = 0;
  n[2] = 1;
  return true;
}

struct RenderArgs {
  rmbx_camera cam;
  const int32_t* prim_i32;
  const float* prim_f32;
  int nprim;
  const double* gxpos;
  const double* gxmat;
  const double* xpos;
  const double* xquat;
  int ngeom, nbody;
  uint8_t* rgb;
  float* depth;
  void* policy;
  int policy_dtype;
  const uint8_t* active;
  int n_env;
  int tiles_x, tiles_y;
  int groups;  // blocks per env (each renders a contiguous range of tiles)
  int dbg;     // diagnostic (RMBX_RENDER_DBG; 0 in production): 1 no ray loop, 2 no stores, 4 test counts, 8 sphere bounds only
};

// RMBX_RENDER_MINW: minimum waves per SIMD the register allocation targets: 8 (default; 64
// registers, 136 B/lane of spilled set-up values, none in the ray loop's hot path) -- per
// 1024-env 8-bit frame 5.74-5.79 ms vs 6.46 at 5 waves (94 registers, no spills), 6.06 at 6,
// 5.82 at 7 and 7.35-7.44 unconstrained (98 registers, 4 waves); identical images
// (profiles/r4_render_waves_ab.log); the other targets are build options for the A/B
// (scripts/build_variant.py render4 .. render7)
#ifndef RMBX_RENDER_MINW
#define RMBX_RENDER_MINW 8
#endif
__global__ void __launch_bounds__(256, RMBX_RENDER_MINW) render_kernel(RenderArgs a) {
  __shared__ PrimCam prims[MAX_PRIM];
  __shared__ int order[MAX_PRIM];        // the block's primitives sorted front to back, once
  __shared__ int tile_sorted[MAX_PRIM];  // the tile's survivors in that order
  __shared__ int wcount[4];
  __shared__ CamFrame cf;
  const int ntiles = a.tiles_x * a.tiles_y;
  const int env = blockIdx.x / a.groups;
  const int grp = blockIdx.x % a.groups;
  if (env >= a.n_env) return;
  if (a.active && !a.active[env]) return;
  const int tid = threadIdx.x;
  const int W = a.cam.width, H = a.cam.height;
  const float tanh_ = tanf(0.5f * a.cam.fovy_deg * 3.14159265358979f / 180.0f);
  const float aspect = (float)W / (float)H;
  // cosine of the widest ray (image corner) against the view axis
  const float cos_max = rsqrtf(1.0f + tanh_ * tanh_ * (1.0f + aspect * aspect));
  if (tid == 0) {
    // camera pose in world
    double Rb[9], Rc[9], R[9], t[3];
    const double* bq = a.xquat + ((size_t)env * a.nbody + a.cam.body) * 4;
    const double* bp = a.xpos + ((size_t)env * a.nbody + a.cam.body) * 3;
    quat2mat(bq, Rb);
    quat2mat(a.cam.quat, Rc);
    matmul3(Rb, Rc, R);
    matvec3(Rb, a.cam.pos, t);
    for (int i = 0; i < 9; i++) cf.R[i] = (float)R[i];
    for (int i = 0; i < 3; i++) cf.p[i] = (float)(bp[i] + t[i]);
  }
  __syncthreads();
  // the env's primitives in the camera frame, once per block (the block then renders a range
  // of tiles of this env)
  const int np = a.nprim < MAX_PRIM ? a.nprim : MAX_PRIM;
  for (int p = tid; p < np; p += blockDim.x) {
    const int g = a.prim_i32[4 * p];
    const int type = a.prim_i32[4 * p + 1];
    const float* f = a.prim_f32 + 8 * p;
    PrimCam P;
    const double* gp = a.gxpos + ((size_t)env * a.ngeom + g) * 3;
    const double* gm = a.gxmat + ((size_t)env * a.ngeom + g) * 9;
    float dw[3] = {(float)gp[0] - cf.p[0], (float)gp[1] - cf.p[1], (float)gp[2] - cf.p[2]};
    // camera coords = Rcam^T (x - pcam)
    for (int i = 0; i < 3; i++) P.c[i] = cf.R[i] * dw[0] + cf.R[3 + i] * dw[1] + cf.R[6 + i] * dw[2];
    for (int k = 0; k < 3; k++) {
      const float ax[3] = {(float)gm[k], (float)gm[3 + k], (float)gm[6 + k]};
      for (int i = 0; i < 3; i++)
        P.R[3 * i + k] = cf.R[i] * ax[0] + cf.R[3 + i] * ax[1] + cf.R[6 + i] * ax[2];
    }
    P.s[0] = f[0];
    P.s[1] = f[1];
    P.s[2] = f[2];
    P.rgb[0] = f[3];
    P.rgb[1] = f[4];
    P.rgb[2] = f[5];
    P.type = type;
    float rad = 0;
    if (type == RMBX_GEOM_SPHERE)
      rad = f[0];
    else if (type == RMBX_GEOM_CAPSULE)
      rad = f[0] + f[1];
    else if (type == RMBX_GEOM_CYLINDER)
      rad = sqrtf(f[0] * f[0] + f[1] * f[1]);
    else if (type == RMBX_GEOM_BOX)
      rad = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    P.rad = rad;
    P.zmin = (type == RMBX_GEOM_PLANE || rad <= 0) ? -1e30f : (-P.c[2] - rad);
    for (int i = 0; i < 3; i++) P.ol[i] = -(P.R[i] * P.c[0] + P.R[3 + i] * P.c[1] + P.R[6 + i] * P.c[2]);
    if (!(a.dbg & 8) && type != RMBX_GEOM_PLANE) {
      // tighter bound for large primitives (the 10 m walls, the table): every hit point lies at
      // least the camera-to-primitive distance r away, so its camera depth is >= r * cos_max
      // (cos_max: the widest ray angle of the image).  The walls then sort behind the table and
      // floor and the rays stop before testing them.
      const float* ol = P.ol;
      float r = -1.f;
      if (type == RMBX_GEOM_BOX) {
        float d2 = 0.f;
        for (int i = 0; i < 3; i++) {
          const float e = fabsf(ol[i]) - P.s[i];
          if (e > 0.f) d2 += e * e;
        }
        r = sqrtf(d2);
      } else if (type == RMBX_GEOM_SPHERE) {
        r = sqrtf(ol[0] * ol[0] + ol[1] * ol[1] + ol[2] * ol[2]) - P.s[0];
      } else if (type == RMBX_GEOM_CAPSULE || type == RMBX_GEOM_CYLINDER) {
        const float h = P.s[1];
        const float z = fminf(fmaxf(ol[2], -h), h);
        const float dz = ol[2] - z;
        const float rad_c = type == RMBX_GEOM_CYLINDER ? sqrtf(P.s[0] * P.s[0]) : P.s[0];
        r = sqrtf(ol[0] * ol[0] + ol[1] * ol[1] + dz * dz) - rad_c;
      }
      if (r > 0.f) P.zmin = fmaxf(P.zmin, r * cos_max * (1.0f - 1e-5f) - 1e-5f);
    }
    prims[p] = P;
  }
  __syncthreads();
  // order the primitives front to back by the depth bound (ties by index) once per block: a tile
  // keeps this order for its survivors, and a ray stops at the first primitive whose bound lies
  // behind its nearest hit so far
  for (int p = tid; p < np; p += blockDim.x) {
    const float z = prims[p].zmin;
    int rank = 0;
    for (int j = 0; j < np; j++) {
      const float zq = prims[j].zmin;
      rank += (zq < z) || (zq == z && j < p);
    }
    order[rank] = p;
  }
  const int t_begin = (int)((long long)ntiles * grp / a.groups);
  const int t_end = (int)((long long)ntiles * (grp + 1) / a.groups);
  for (int tile = t_begin; tile < t_end; ++tile) {
  __syncthreads();  // the previous tile's rays are done with tile_sorted (and order is complete)
  const int tx0 = (tile % a.tiles_x) * RENDER_TILE, ty0 = (tile / a.tiles_x) * RENDER_TILE;
  // tile frustum in normalised image coords
  const float x_lo = (2.0f * tx0 / W - 1.0f) * tanh_ * aspect;
  const float x_hi = (2.0f * (tx0 + RENDER_TILE) / W - 1.0f) * tanh_ * aspect;
  const float y_hi = (1.0f - 2.0f * ty0 / H) * tanh_;
  const float y_lo = (1.0f - 2.0f * (ty0 + RENDER_TILE) / H) * tanh_;
  bool keep = false;
  const int p_cull = tid < np ? order[tid] : 0;  // np <= MAX_PRIM <= blockDim.x: one primitive per thread
  if (tid < np) {
    const PrimCam& P = prims[p_cull];
    const int type = P.type;
    const float rad = P.rad;
    // conservative tile test: sphere vs the 4 tile planes (camera looks along -z)
    keep = true;
    if (type != RMBX_GEOM_PLANE && rad > 0) {
      const float z = -P.c[2];
      if (z + rad <= 1e-3f) keep = false;  // behind the camera
      else if (z - rad > 1e-3f) {
        // plane x = s z: signed distance of centre to the plane pair of the tile slab
        const float nx_lo = 1.0f / sqrtf(1 + x_lo * x_lo), nx_hi = 1.0f / sqrtf(1 + x_hi * x_hi);
        const float ny_lo = 1.0f / sqrtf(1 + y_lo * y_lo), ny_hi = 1.0f / sqrtf(1 + y_hi * y_hi);
        if ((P.c[0] - x_lo * z) * nx_lo < -rad) keep = false;
        if ((x_hi * z - P.c[0]) * nx_hi < -rad) keep = false;
        if ((P.c[1] - y_lo * z) * ny_lo < -rad) keep = false;
        if ((y_hi * z - P.c[1]) * ny_hi < -rad) keep = false;
      }
    }
  }
  // compact the survivors in sorted order: ballot per wave, wave offsets through LDS
  const unsigned long long kb = __ballot(keep);
  if ((tid & 63) == 0) wcount[tid >> 6] = __popcll(kb);
  __syncthreads();
  int base = 0;
  for (int w = 0; w < (tid >> 6); ++w) base += wcount[w];
  if (keep) tile_sorted[base + __popcll(kb & ((1ull << (tid & 63)) - 1))] = p_cull;
  const int tile_cnt = wcount[0] + wcount[1] + wcount[2] + wcount[3];
  __syncthreads();
  const int px = tx0 + (tid % RENDER_TILE), py = ty0 + (tid / RENDER_TILE);
  if (px < W && py < H) {
  const float d[3] = {((2.0f * (px + 0.5f) / W) - 1.0f) * tanh_ * aspect,
                      (1.0f - 2.0f * (py + 0.5f) / H) * tanh_, -1.0f};
  float best = 1e30f, bn[3] = {0, 0, 1};
  int bp = -1;
  const int cnt = tile_cnt;
  int ntest = 0;
  for (int k = 0; k < ((a.dbg & 1) ? 0 : cnt); k++) {
    const int p = tile_sorted[k];
    const PrimCam& P = prims[p];
    if (P.zmin > best + 1e-4f) break;  // every later primitive lies behind the current hit
    ++ntest;
    float o_l[3], d_l[3], t, nl[3];
    to_local(P, d, o_l, d_l);
    bool h = false;
    switch (P.type) {
      case RMBX_GEOM_PLANE: h = hit_plane(o_l, d_l, &t, nl); break;
      case RMBX_GEOM_SPHERE: h = hit_sphere(o_l, d_l, P.s[0], &t, nl); break;
      case RMBX_GEOM_CAPSULE: h = hit_capsule(o_l, d_l, P.s[0], P.s[1], &t, nl); break;
      case RMBX_GEOM_CYLINDER: h = hit_cylinder(o_l, d_l, P.s[0], P.s[1], true, &t, nl); break;
      case RMBX_GEOM_BOX: h = hit_box(o_l, d_l, P.s, &t, nl); break;
      default: break;
    }
    if (h && (t < best || (t == best && p < bp))) {
      best = t;
      bp = p;
      // normal back to camera frame
      for (int i = 0; i < 3; i++) bn[i] = P.R[3 * i] * nl[0] + P.R[3 * i + 1] * nl[1] + P.R[3 * i + 2] * nl[2];
    }
  }
  float col[3];
  float depth = a.cam.zfar;
  if (bp < 0) {
    col[0] = 0.9f;  // skybox gradient colour of env_ur5e_common.xml
    col[1] = 1.0f;
    col[2] = 1.0f;
  } else {
    const PrimCam& P = prims[bp];
    const float inv = rsqrtf(dot3f(d, d));
    const float vd[3] = {d[0] * inv, d[1] * inv, d[2] * inv};
    float ndv = -(bn[0] * vd[0] + bn[1] * vd[1] + bn[2] * vd[2]);
    if (ndv < 0) {
      ndv = -ndv;
      bn[0] = -bn[0];
      bn[1] = -bn[1];
      bn[2] = -bn[2];
    }
    // directional light pointing down (world -z) expressed in camera frame
    const float Ld[3] = {-cf.R[6], -cf.R[7], -cf.R[8]};
    float ndl = -(bn[0] * Ld[0] + bn[1] * Ld[1] + bn[2] * Ld[2]);
    ndl = ndl > 0 ? ndl : 0;
    const float shade = 0.1f + 0.6f * ndv + 0.3f * ndl;
    for (int i = 0; i < 3; i++) col[i] = fminf(P.rgb[i] * shade, 1.0f);
    depth = best;  // d has unit -z component: t is the camera-z distance
  }
  const size_t pix = (size_t)py * W + px;
  const size_t hw = (size_t)H * W;
  const bool do_store = !(a.dbg & 2) || col[0] == 12345.f;  // (diagnostic: keep the shading live)
  uint8_t u[3];
  for (int i = 0; i < 3; i++) u[i] = (uint8_t)(col[i] * 255.0f + 0.5f);
  if (a.rgb && do_store) {
    uint8_t* o = a.rgb + ((size_t)env * hw + pix) * 3;
    o[0] = u[0];
    o[1] = u[1];
    o[2] = u[2];
  }
  if (a.depth && do_store) a.depth[(size_t)env * hw + pix] = (a.dbg & 4) ? (float)(ntest + 1000 * cnt) : depth;
  if (a.policy && do_store) {
    if (a.policy_dtype == 2) {
      // 2x2 space-to-depth [n][H/2][W/2][16]: channel (dy*2+dx)*3+c, 12..15 zero
      const int Hs = H >> 1, Ws = W >> 1;
      __hip_bfloat16* o = reinterpret_cast<__hip_bfloat16*>(a.policy) +
                          (((size_t)env * Hs + (py >> 1)) * Ws + (px >> 1)) * 16;
      const int q = ((py & 1) * 2 + (px & 1)) * 3;
      for (int c = 0; c < 3; c++) o[q + c] = __float2bfloat16(((float)u[c] / 255.0f - a.cam.mean[c]) / a.cam.std[c]);
      if ((py & 1) && (px & 1))
        for (int c = 12; c < 16; c++) o[c] = __float2bfloat16(0.0f);
    } else if (a.policy_dtype == 3) {
      // the same space-to-depth layout in f32
      const int Hs = H >> 1, Ws = W >> 1;
      float* o = reinterpret_cast<float*>(a.policy) + (((size_t)env * Hs + (py >> 1)) * Ws + (px >> 1)) * 16;
      const int q = ((py & 1) * 2 + (px & 1)) * 3;
      for (int c = 0; c < 3; c++) o[q + c] = ((float)u[c] / 255.0f - a.cam.mean[c]) / a.cam.std[c];
      if ((py & 1) && (px & 1))
        for (int c = 12; c < 16; c++) o[c] = 0.0f;
    } else if (a.policy_dtype == 4) {
      // the same space-to-depth layout holding the 8-bit pixel values themselves (the f32 stem on
      // the quantised image, rmbx_stem_s2d_conv_maxpool_u8, applies mean / std exactly)
      const int Hs = H >> 1, Ws = W >> 1;
      uint8_t* o = reinterpret_cast<uint8_t*>(a.policy) + (((size_t)env * Hs + (py >> 1)) * Ws + (px >> 1)) * 16;
      const int q = ((py & 1) * 2 + (px & 1)) * 3;
      for (int c = 0; c < 3; c++) o[q + c] = u[c];
      if ((py & 1) && (px & 1))
        for (int c = 12; c < 16; c++) o[c] = 0;
    } else {
      for (int c = 0; c < 3; c++) {
        const float v = ((float)u[c] / 255.0f - a.cam.mean[c]) / a.cam.std[c];
        const size_t idx = ((size_t)env * 3 + c) * hw + pix;
        if (a.policy_dtype == 1)
          reinterpret_cast<__hip_bfloat16*>(a.policy)[idx] = __float2bfloat16(v);
        else
          reinterpret_cast<float*>(a.policy)[idx] = v;
      }
    }
  }
  }  // pixel
  __syncthreads();
  }  // tiles
}

}  // namespace rmbx

extern "C" int rmbx_render(const rmbx_camera* cam, const int32_t* prim_i32, const float* prim_f32,
                           int nprim, const double* gxpos, const double* gxmat, const double* xpos,
                           const double* xquat, int ngeom, int nbody, uint8_t* rgb, float* depth,
                           void* policy_img, int policy_dtype, const uint8_t* active, int n_env,
                           void* stream) {
  RMBX_CHECK_ARG(cam && prim_i32 && prim_f32 && gxpos && gxmat && xpos && xquat, "NULL argument");
  RMBX_CHECK_ARG(nprim > 0 && nprim <= MAX_PRIM, "nprim=%d outside [1, %d]", nprim, MAX_PRIM);
  RMBX_CHECK_ARG(cam->width > 0 && cam->height > 0 && cam->width <= 8192 && cam->height <= 8192,
                 "bad image size %dx%d", cam->width, cam->height);
  RMBX_CHECK_ARG(cam->body >= 0 && cam->body < nbody, "bad camera body %d", cam->body);
  RMBX_CHECK_ARG(policy_dtype >= 0 && policy_dtype <= 4,
                 "policy_dtype must be 0 (f32), 1 (bf16), 2 (bf16 s2d), 3 (f32 s2d) or 4 (u8 s2d)");
  RMBX_CHECK_ARG(policy_dtype < 2 || (cam->width % 2 == 0 && cam->height % 2 == 0),
                 "space-to-depth policy output needs an even image size");
  if (n_env == 0) return RMBX_OK;
  rmbx::RenderArgs a;
  a.cam = *cam;
  a.prim_i32 = prim_i32;
  a.prim_f32 = prim_f32;
  a.nprim = nprim;
  a.gxpos = gxpos;
  a.gxmat = gxmat;
  a.xpos = xpos;
  a.xquat = xquat;
  a.ngeom = ngeom;
  a.nbody = nbody;
  a.rgb = rgb;
  a.depth = depth;
  a.policy = policy_img;
  a.policy_dtype = policy_dtype;
  a.active = active;
  a.n_env = n_env;
  a.tiles_x = (cam->width + RENDER_TILE - 1) / RENDER_TILE;
  a.tiles_y = (cam->height + RENDER_TILE - 1) / RENDER_TILE;
  a.groups = 16;
  const char* dbg_env = std::getenv("RMBX_RENDER_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  const size_t nblocks = (size_t)n_env * a.groups;
  RMBX_CHECK_ARG(nblocks < (1ull << 31), "grid too large");
  hipLaunchKernelGGL(rmbx::render_kernel, dim3((unsigned)nblocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
