// Batched camera rendering of the scene primitives and the visual meshes (gfx950).
//
// Replaces the per-env, per-camera OpenGL OffScreenViewer rgb + depth renders of
// envs/mujoco/MujocoEnvBase.py:112-126.  Two passes per camera:
//   1. visibility of the visual meshes (the UR5e / Robotiq / D435i `class="visual"` geoms,
//      mjcf/rmesh.py): one thread per (env, triangle) transforms the triangle into the camera frame
//      (its body's pose, one transform per env and body in LDS), finds the pixel centres its
//      projection covers (clipped at the camera's znear, as OpenGL's near plane), intersects each of
//      those pixels' camera rays with it (the same ray-triangle test as a ray caster, so depth and
//      coverage are the ray's) and keeps the nearest per pixel with a 64-bit atomic min of
//      (depth bits, triangle) in a caller-provided visibility buffer.  Meshes are many small
//      triangles: projecting each triangle once costs far less than tracing each pixel's ray
//      through a hierarchy of them;
//   2. one 256-thread workgroup per 16x16 pixel tile of one env ray-casts the analytic primitives:
//      the env's primitives in the camera frame in LDS, culled against the tile's frustum slice
//      (bounding spheres and projected boxes), sorted front to back by a depth bound; every lane
//      starts from its pixel's mesh hit and casts its ray against the surviving primitives, stopping
//      at the first whose bound lies behind its nearest hit.
// Shading: ambient + headlight + one directional light (the scene's <light> and MuJoCo's default
// headlight), material colour times the material's texture (primitives: 2d / cube textures sampled
// bilinearly at the hit's local coordinates) plus the directional light's Blinn-Phong specular term,
// flat-shaded triangles; the gradient skybox behind (include/rmbx.h rmbx_scene_tables).  Outputs are
// written once per pixel: u8 HWC RGB, f32 linear depth, the hit geom id, and/or the policy input
// tensor (CHW, ImageNet-normalised, bf16 or f32, or the space-to-depth forms) fused so the policy
// never re-reads the u8 image.

#include <hip/hip_bf16.h>

#include "rmbx_common.h"

#include <algorithm>
#include <cstdlib>
#include "rmbx_math.h"
#include "rmbx_model.h"

namespace rmbx {

#define RENDER_TILE 16
#define MAX_PRIM 128
#define MAX_MESH 64  // bodies with render meshes
#define VIS_EMPTY 0xffffffffffffffffull

struct PrimCam {
  float c[3];    // centre in camera frame
  float R[9];    // geom axes in camera frame (columns = local axes)
  float s[3];    // size
  float rgb[3];
  int type;
  float rad;   // bounding radius (0 = unbounded)
  float zmin;  // lower bound of any hit's depth (camera z) in the image; -1e30 if unbounded
  float ol[3];  // the camera (ray origin) in the primitive's local frame: R^T (0 - c)
  float sx_lo, sx_hi, sy_lo, sy_hi;  // image-plane slopes (x / -z, y / -z) bounding the primitive's
                                     // box (projected corners; unbounded when a corner is not in front)
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
  const float* mesh_tri;      // [ntri][16]: v0, e1, e2, n, tag = (mesh slot << 16) | geom (int bits), rgb
  int ntri, nmesh;
  const int32_t* mesh_body;   // [nmesh] body of each mesh slot
  const float* mesh_rad;      // [nmesh] bounding radius of the slot's triangles about the body origin
  unsigned long long* vis;    // [n][H][W] nearest mesh hit (depth bits << 32 | triangle), VIS_EMPTY: none
  uint8_t* tflag;             // [n][tiles]: 1 where the visibility pass wrote a pixel of the tile
  int32_t* hit_geom;          // optional [n][H][W]: geom id of the pixel's surface (-1: background)
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
  int dbg;     // diagnostic (RMBX_RENDER_DBG; 0 in production): 1 no ray loop, 2 no stores, 4 test counts, 8 sphere
               // bounds only; visibility-pass timing probes: 16 frames only, 32 + set-up, 64 + ray tests, no writes;
               // materials: 128 textures at the base level only, 256 no texture sampling, 512 no footprint;
               // 1024: back faces drawn (the round-5 two-sided triangles; A/B only)
  // materials (NULL geom_matinfo: the flat round-5 shading); include/rmbx.h rmbx_scene_tables
  const int32_t* geom_texid;
  const float* geom_matinfo;
  const uint32_t* tex_rgba;
  const int4* tex_desc;
  const int32_t* tex_level_adr;
  float sky[6];
  // static-background cache (rmbx_render_scene_cached; null: none): prim_static [nprim] 1 for a
  // primitive of a body welded to the world; cache [n][H][W] = (depth bits, rgb | prim << 24) of the
  // static-only scene (prim 0xff: none); dirty [n]: 1 where the cache is rebuilt this call
  const uint8_t* prim_static;
  uint2* cache;
  const uint8_t* dirty;
};

// one texel (RGBA8 word, R in the low byte) as floats in [0, 1]
__device__ __forceinline__ void texel(const uint32_t* t, int idx, float w, float* c) {
  const uint32_t v = __ldg(t + idx);
  c[0] += w * (float)(v & 255u);
  c[1] += w * (float)((v >> 8) & 255u);
  c[2] += w * (float)((v >> 16) & 255u);
}

// bilinear sample at continuous texel coordinates (fx, fy) (texel centres at integers): wrap
// (2d textures: GL_REPEAT) or clamp at the edges (cube faces: GL_CLAMP_TO_EDGE).  The wrap is done
// on the integer-valued floats (exact below 2^24; an integer modulo costs ~40 instructions)
__device__ __forceinline__ void tex_bilinear(const uint32_t* t, int H, int W, float fx, float fy, bool wrap, float* c) {
  const float x0f = floorf(fx), y0f = floorf(fy);
  const float ax = fx - x0f, ay = fy - y0f;
  const float Wf = (float)W, Hf = (float)H;
  int x0, y0, x1, y1;
  if (wrap) {
    const float xw = x0f - Wf * floorf(x0f * __builtin_amdgcn_rcpf(Wf));
    const float yw = y0f - Hf * floorf(y0f * __builtin_amdgcn_rcpf(Hf));
    // (the reciprocal's rounding can leave xw one period off: fold it back)
    x0 = (int)xw;
    y0 = (int)yw;
    x0 += x0 < 0 ? W : (x0 >= W ? -W : 0);
    y0 += y0 < 0 ? H : (y0 >= H ? -H : 0);
    x1 = x0 + 1 == W ? 0 : x0 + 1;
    y1 = y0 + 1 == H ? 0 : y0 + 1;
  } else {
    x0 = (int)fminf(fmaxf(x0f, 0.f), Wf - 1.f);
    y0 = (int)fminf(fmaxf(y0f, 0.f), Hf - 1.f);
    x1 = (int)fminf(fmaxf(x0f + 1.f, 0.f), Wf - 1.f);
    y1 = (int)fminf(fmaxf(y0f + 1.f, 0.f), Hf - 1.f);
  }
  c[0] = c[1] = c[2] = 0.f;
  if (x1 == x0 + 1) {  // the two texels of a row are adjacent words: one 8-byte load per row
    uint2 r0, r1;
    __builtin_memcpy(&r0, t + y0 * W + x0, 8);
    __builtin_memcpy(&r1, t + y1 * W + x0, 8);
    const float w00 = (1.f - ax) * (1.f - ay), w01 = ax * (1.f - ay), w10 = (1.f - ax) * ay, w11 = ax * ay;
    const uint32_t v[4] = {r0.x, r0.y, r1.x, r1.y};
    const float w[4] = {w00, w01, w10, w11};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      c[0] += w[k] * (float)(v[k] & 255u);
      c[1] += w[k] * (float)((v[k] >> 8) & 255u);
      c[2] += w[k] * (float)((v[k] >> 16) & 255u);
    }
  } else {
    texel(t, y0 * W + x0, (1.f - ax) * (1.f - ay), c);
    texel(t, y0 * W + x1, ax * (1.f - ay), c);
    texel(t, y1 * W + x0, (1.f - ax) * ay, c);
    texel(t, y1 * W + x1, ax * ay, c);
  }
  for (int i = 0; i < 3; i++) c[i] *= (1.0f / 255.0f);
}

// texture coordinates (in units of the base level's texels: fx = u W, fy = v H, before the -0.5
// texel-centre shift) of local point q on a primitive of `type` / size s, and the texture's
// density there (base texels per metre along the surface): 2d from (x, y); cube maps on the face of
// the major axis, OpenGL's face orientation (include/rmbx.h rmbx_scene_tables)
__device__ __forceinline__ void tex_coords(int ttype, int H, int W, int type, const float* s, const float* mi,
                                           const float* pl, float& fx, float& fy, float& dens) {
  const bool uni = mi[4] != 0.f;
  if (ttype == 0) {  // 2d: (x, y), texrepeat over the geom's extent, or per metre
    // the geom's half extents in its local x / y (round geoms: the radius)
    const float sx = s[0];
    const float sy = type == RMBX_GEOM_BOX || type == RMBX_GEOM_PLANE ? s[1] : s[0];
    float u = pl[0] * mi[2], v = pl[1] * mi[3];
    float kx = mi[2], ky = mi[3];  // periods per metre
    if (!uni && sx > 0.f && sy > 0.f) {
      kx = mi[2] / (2.f * sx);
      ky = mi[3] / (2.f * sy);
      u = mi[2] * (pl[0] / (2.f * sx) + 0.5f);
      v = mi[3] * (pl[1] / (2.f * sy) + 0.5f);
    }
    fx = u * W;
    fy = v * H;
    dens = fmaxf(kx * W, ky * H);
    return;
  }
  float q[3] = {pl[0], pl[1], pl[2]};
  float hmin = 1.f;
  if (uni) {  // the unit object: local point over the half extents
    float h[3] = {s[0], s[0], s[0]};
    if (type == RMBX_GEOM_BOX) { h[1] = s[1]; h[2] = s[2]; }
    else if (type == RMBX_GEOM_CAPSULE) h[2] = s[1] + s[0];
    else if (type == RMBX_GEOM_CYLINDER) h[2] = s[1];
    else if (type == RMBX_GEOM_PLANE) { h[1] = s[1]; h[2] = 1.f; }
    for (int i = 0; i < 3; i++) q[i] = h[i] > 0.f ? q[i] / h[i] : q[i];
    hmin = fminf(fminf(h[0] > 0.f ? h[0] : 1.f, h[1] > 0.f ? h[1] : 1.f), h[2] > 0.f ? h[2] : 1.f);
  }
  const float x = fabsf(q[0]), y = fabsf(q[1]), z = fabsf(q[2]);
  float sc, tc, ma;
  if (x >= y && x >= z) {
    ma = x; sc = q[0] > 0.f ? -q[2] : q[2]; tc = -q[1];
  } else if (y >= z) {
    ma = y; sc = q[0]; tc = q[1] > 0.f ? q[2] : -q[2];
  } else {
    ma = z; sc = q[2] > 0.f ? q[0] : -q[0]; tc = -q[1];
  }
  ma = fmaxf(ma, 1e-30f);
  const float im = 1.0f / ma;
  fx = 0.5f * (sc * im + 1.f) * W;
  fy = 0.5f * (tc * im + 1.f) * H;
  dens = 0.5f * (float)max(W, H) * im / hmin;
}

// the texture colour of a primitive at local hit point pl: OpenGL's GL_LINEAR_MIPMAP_LINEAR
// (trilinear) with an isotropic footprint: a pixel spans foot = t pix / max(n.v, 1e-3) metres of
// the surface at camera depth t (pix: one pixel's step of the ray slope), the level of detail is
// log2(foot x the texture's density there); bilinear in the two nearest levels of the box-filtered
// mip pyramid
__device__ void sample_texture(const RenderArgs& a, int tex, int type, const float* s, const float* mi,
                               const float* pl, float foot, float* c) {
  const int4 td = a.tex_desc[tex];  // (type, H, W, first texel)
  const uint32_t* t = a.tex_rgba + td.w;
  const int H = td.y, W = td.z;
  float fx, fy, dens;
  tex_coords(td.x, H, W, type, s, mi, pl, fx, fy, dens);
  const float rho = (a.dbg & 512) ? 0.f : foot * dens;  // (timing probe 512: no footprint)
  // levels down to 1 x 1: 32 - clz(max(H, W)); level l's first texel from the host table
  const int levels = 32 - __builtin_clz((unsigned)max(H, W));
  float lod = fminf(fmaxf(__log2f(fmaxf(rho, 1e-30f)), 0.f), (float)(levels - 1));
  if (a.dbg & 128) lod = 0.f;  // (timing probe: the base level only)
  const int l0 = (int)lod;
  const float fr = lod - (float)l0;
  const bool wrap = td.x == 0;
  const int* ladr = a.tex_level_adr + RMBX_TEX_LEVELS * tex;
  const float iW = 1.0f / (float)W, iH = 1.0f / (float)H;
  float c0[3] = {0.f, 0.f, 0.f}, c1[3] = {0.f, 0.f, 0.f};
  {
    const int Hl = max(H >> l0, 1), Wl = max(W >> l0, 1);
    tex_bilinear(t + ladr[l0], Hl, Wl, fx * (Wl * iW) - 0.5f, fy * (Hl * iH) - 0.5f, wrap, c0);
  }
  if (fr > 0.f && l0 + 1 < levels) {
    const int Hl = max(H >> (l0 + 1), 1), Wl = max(W >> (l0 + 1), 1);
    tex_bilinear(t + ladr[l0 + 1], Hl, Wl, fx * (Wl * iW) - 0.5f, fy * (Hl * iH) - 0.5f, wrap, c1);
  } else {
    c1[0] = c0[0];
    c1[1] = c0[1];
    c1[2] = c0[2];
  }
  for (int i = 0; i < 3; i++) c[i] = c0[i] + fr * (c1[i] - c0[i]);
}

// camera pose of env `env` in world: R (columns = camera axes), p
__device__ __forceinline__ void camera_frame(const RenderArgs& a, int env, CamFrame& cf) {
#pragma clang fp contract(off)  // bit-identical in every kernel it is inlined into
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

// a mesh slot's body frame in the camera frame: R = Rcam^T Rbody (row-major), c = Rcam^T (x - pcam)
__device__ __forceinline__ void mesh_frame(const RenderArgs& a, int env, int k, const CamFrame& cf, float* R,
                                           float* c) {
#pragma clang fp contract(off)
  const int b = a.mesh_body[k];
  double Rb[9];
  quat2mat(a.xquat + ((size_t)env * a.nbody + b) * 4, Rb);
  const double* bp = a.xpos + ((size_t)env * a.nbody + b) * 3;
  const float dw[3] = {(float)bp[0] - cf.p[0], (float)bp[1] - cf.p[1], (float)bp[2] - cf.p[2]};
  for (int i = 0; i < 3; i++) {
    c[i] = cf.R[i] * dw[0] + cf.R[3 + i] * dw[1] + cf.R[6 + i] * dw[2];
    for (int k2 = 0; k2 < 3; k2++)
      R[3 * i + k2] = cf.R[i] * (float)Rb[k2] + cf.R[3 + i] * (float)Rb[3 + k2] + cf.R[6 + i] * (float)Rb[6 + k2];
  }
}

// ---------------------------------------------------------------------------------------------
// Pass 1: mesh visibility.  Block = 256 consecutive triangles of one env; blocks are laid out so
// each XCD (blocks bid = xcd mod 8) walks a contiguous range of triangle chunks for all envs, the
// chunk outer and the env inner, keeping its chunks' 16 KiB of triangles in its L2.  A triangle
// whose projection spans more than RASTER_SMALL pixel centres is covered by its whole wave.
// ---------------------------------------------------------------------------------------------
#define RASTER_THREADS 256
#ifndef RASTER_SMALL
#define RASTER_SMALL 32  // pixel centres a lane covers itself (larger: its wave); 2-32 A/B: profiles/r5_render_raster_small_ab.log
#endif

struct TriCam {
  float v0[3], e1[3], e2[3];  // the triangle in the camera frame
  int x0, x1, y0, y1;         // the pixel centres its projection can cover (inclusive; empty if x0 > x1)
  // the projection's edges (the near-plane-clipped polygon: 3 or 4 edges) as pixel-space half
  // planes ea x + eb y + ec >= 0 (unit normals, a tolerance folded into ec): a cheap conservative
  // reject before the ray test, which alone decides coverage
  float ea[4], eb[4], ec[4];
};

// the triangle in the camera frame, its near-plane-clipped projection (vertices in front of the
// near plane and the points where edges cross it) in pixel coordinates, the range of pixel centres
// that projection can cover and its edges
__device__ __forceinline__ void tri_setup(const RenderArgs& a, const float4* tp, const float* R, const float* c,
                                          float tanh_, float aspect, TriCam& T) {
  // no FMA contraction here and in tri_cover: a triangle's depths must be bit-identical whichever
  // path covered it (its own lane or its wave) and however the compiler inlined it
#pragma clang fp contract(off)
  const float4 A = tp[0], B = tp[1], C = tp[2];
  const float l0[3] = {A.x, A.y, A.z}, l1[3] = {A.w, B.x, B.y}, l2[3] = {B.z, B.w, C.x};
  for (int i = 0; i < 3; i++) {
    T.v0[i] = c[i] + R[3 * i] * l0[0] + R[3 * i + 1] * l0[1] + R[3 * i + 2] * l0[2];
    T.e1[i] = R[3 * i] * l1[0] + R[3 * i + 1] * l1[1] + R[3 * i + 2] * l1[2];
    T.e2[i] = R[3 * i] * l2[0] + R[3 * i + 1] * l2[1] + R[3 * i + 2] * l2[2];
  }
  const int W = a.cam.width, H = a.cam.height;
  T.x0 = 1;
  T.x1 = 0;
  T.y0 = T.y1 = 0;
  {
    // back faces are culled (MuJoCo's default mjRND_CULL_FACE, OpenGL counter-clockwise front
    // faces): the winding normal e1 x e2 must point towards the eye at the origin
    const float nw[3] = {T.e1[1] * T.e2[2] - T.e1[2] * T.e2[1], T.e1[2] * T.e2[0] - T.e1[0] * T.e2[2],
                         T.e1[0] * T.e2[1] - T.e1[1] * T.e2[0]};
    if (!(nw[0] * T.v0[0] + nw[1] * T.v0[1] + nw[2] * T.v0[2] < 0.f) && !(a.dbg & 1024)) return;
  }
  const float znear = a.cam.znear;
  const float fx = 0.5f * W / (tanh_ * aspect), fy = 0.5f * H / tanh_;
  const float P[3][3] = {{T.v0[0], T.v0[1], T.v0[2]},
                         {T.v0[0] + T.e1[0], T.v0[1] + T.e1[1], T.v0[2] + T.e1[2]},
                         {T.v0[0] + T.e2[0], T.v0[1] + T.e2[1], T.v0[2] + T.e2[2]}};
  // the clipped polygon in pixel coordinates (pixel centre (px, py) at (px + 0.5, py + 0.5))
  float X[4], Y[4];
  int n = 0;
#pragma unroll
  for (int u = 0; u < 3; u++) {
    const int w = (u + 1) % 3;
    const float zu = -P[u][2], zw = -P[w][2];
    if (zu >= znear) {
      const float iz = 1.f / zu;
      X[n] = P[u][0] * iz * fx + 0.5f * W;
      Y[n] = 0.5f * H - P[u][1] * iz * fy;
      ++n;
    }
    if ((zu >= znear) != (zw >= znear)) {  // the edge crosses the near plane
      const float s = (znear - zu) / (zw - zu);
      const float x = P[u][0] + s * (P[w][0] - P[u][0]), y = P[u][1] + s * (P[w][1] - P[u][1]);
      const float iz = 1.f / znear;
      X[n] = x * iz * fx + 0.5f * W;
      Y[n] = 0.5f * H - y * iz * fy;
      ++n;
    }
  }
  T.x0 = 1;
  T.x1 = 0;
  T.y0 = T.y1 = 0;
  if (n < 3) return;  // entirely in front of the camera's near plane: clipped
  if (n == 3) {
    X[3] = X[2];
    Y[3] = Y[2];
  }
  float xl = fminf(fminf(X[0], X[1]), fminf(X[2], X[3])), xh = fmaxf(fmaxf(X[0], X[1]), fmaxf(X[2], X[3]));
  float yl = fminf(fminf(Y[0], Y[1]), fminf(Y[2], Y[3])), yh = fmaxf(fmaxf(Y[0], Y[1]), fmaxf(Y[2], Y[3]));
  // pixel-centre ranges a hair wider than the projection
  const float eps = 1e-3f;
  T.x0 = max((int)ceilf(fmaxf(xl - 0.5f - eps, -1.f)), 0);
  T.x1 = min((int)floorf(fminf(xh - 0.5f + eps, (float)W)), W - 1);
  T.y0 = max((int)ceilf(fmaxf(yl - 0.5f - eps, -1.f)), 0);
  T.y1 = min((int)floorf(fminf(yh - 0.5f + eps, (float)H)), H - 1);
  // edges: inside is where every unit-normal edge function is >= -tol, oriented by the polygon's
  // signed area; tol = 0.02 px plus the rounding of the edge function at this coordinate magnitude
  float area2 = 0.f;
#pragma unroll
  for (int i = 0; i < 4; i++) area2 += X[i] * Y[(i + 1) & 3] - X[(i + 1) & 3] * Y[i];
  const float orient = area2 >= 0.f ? -1.f : 1.f;
  const float mag = fmaxf(fmaxf(fabsf(xl), fabsf(xh)), fmaxf(fabsf(yl), fabsf(yh))) + (float)(W + H);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int k = (i + 1) & 3;
    const float dx = X[k] - X[i], dy = Y[k] - Y[i];
    const float len = sqrtf(dx * dx + dy * dy);
    if (!(len > 1e-6f * mag)) {  // a collapsed edge (or the repeated vertex of a triangle): no constraint
      T.ea[i] = 0.f;
      T.eb[i] = 0.f;
      T.ec[i] = 1.f;
      continue;
    }
    const float il = orient / len;
    // E(x, y) = (x - Xi) dy - (y - Yi) dx, negative inside for a positive area
    T.ea[i] = dy * il;
    T.eb[i] = -dx * il;
    T.ec[i] = (Y[i] * dx - X[i] * dy) * il + 0.02f + 4e-6f * mag;
  }
}

// one pixel centre: its camera ray (origin 0) against the triangle (Moller-Trumbore); the nearest
// hit per pixel is kept by an atomic min of (depth bits << 32 | triangle index)
__device__ __forceinline__ void tri_cover(const RenderArgs& a, const TriCam& T, unsigned j, int px, int py,
                                          float tanh_, float aspect, unsigned long long* vis, uint8_t* tflag) {
#pragma clang fp contract(off)
  const int W = a.cam.width, H = a.cam.height;
  {
    const float cx = px + 0.5f, cy = py + 0.5f;
    bool in = true;
#pragma unroll
    for (int i = 0; i < 4; i++) in = in && (T.ea[i] * cx + T.eb[i] * cy + T.ec[i] >= 0.f);
    if (!in) return;  // outside the projection (conservatively): the ray cannot hit the triangle
  }
  // the pixel centre's ray (slopes by multiplication: no division per pixel)
  const float sx = tanh_ * aspect, sy = tanh_;
  const float d[3] = {(px + 0.5f) * (2.0f * sx / W) - sx, sy - (py + 0.5f) * (2.0f * sy / H), -1.0f};
  const float* e1 = T.e1;
  const float* e2 = T.e2;
  const float p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
  const float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
  if (fabsf(det) < 1e-30f) return;
  const float id = __builtin_amdgcn_rcpf(det);  // (1 ulp; the barycentric bounds and depth tolerate it)
  const float s[3] = {-T.v0[0], -T.v0[1], -T.v0[2]};
  const float uu = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * id;
  if (uu < 0.f || uu > 1.f) return;
  const float qv[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
  const float vv = (d[0] * qv[0] + d[1] * qv[1] + d[2] * qv[2]) * id;
  if (vv < 0.f || uu + vv > 1.f) return;
  const float t = (e2[0] * qv[0] + e2[1] * qv[1] + e2[2] * qv[2]) * id;
  if (!(t > a.cam.znear)) return;
  unsigned long long* slot = vis + (size_t)py * W + px;
  const unsigned long long key = ((unsigned long long)__float_as_uint(t) << 32) | j;
  // the key only ever decreases, so a value read earlier (older) that is already <= key proves the
  // atomic would not change it: skip it (most covered pixels of a mesh are overdrawn)
  if (a.dbg & 64) {  // (timing probe: the ray tests without the visibility writes)
    if (t == 12345.f) *slot = key;
    return;
  }
  if (__hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > key) atomicMin(slot, key);
  tflag[(py / RENDER_TILE) * a.tiles_x + px / RENDER_TILE] = 1;  // (every writer stores the same 1)
}

__device__ __forceinline__ void mesh_frames_block(const RenderArgs& a, int env, CamFrame& cf, float (*mR)[9],
                                                  float (*mc)[3], int* mvis, float tanh_, float aspect) {
  const int tid = threadIdx.x;
  if (tid == 0) camera_frame(a, env, cf);
  __syncthreads();
  if (tid < a.nmesh) {
    mesh_frame(a, env, tid, cf, mR[tid], mc[tid]);
    // the slot's bounding sphere against the view frustum (behind the near plane or outside an
    // image edge: none of its triangles can cover a pixel)
    const float rad = a.mesh_rad[tid], z = -mc[tid][2];
    bool v = z + rad > a.cam.znear;
    const float sx = tanh_ * aspect, sy = tanh_;
    const float nx = rsqrtf(1.f + sx * sx), ny = rsqrtf(1.f + sy * sy);
    if (v && (mc[tid][0] - sx * z) * nx > rad) v = false;
    if (v && (-mc[tid][0] - sx * z) * nx > rad) v = false;
    if (v && (mc[tid][1] - sy * z) * ny > rad) v = false;
    if (v && (-mc[tid][1] - sy * z) * ny > rad) v = false;
    mvis[tid] = v;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(RASTER_THREADS) raster_kernel(RenderArgs a, int chunks) {
  __shared__ CamFrame cf;
  __shared__ float mR[MAX_MESH][9], mc[MAX_MESH][3];
  __shared__ int mvis[MAX_MESH];
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
  const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int chunk = lin / a.n_env, env = lin - chunk * a.n_env;
  if (chunk >= chunks) return;
  if (a.active && !a.active[env]) return;
  const float tanh_ = tanf(0.5f * a.cam.fovy_deg * 3.14159265358979f / 180.0f);
  const float aspect = (float)a.cam.width / (float)a.cam.height;
  mesh_frames_block(a, env, cf, mR, mc, mvis, tanh_, aspect);
  if (a.dbg & 16) return;  // (timing probe: the per-block frames only)
  // every lane stays to the end (the wave's pixel work is shared by all 64 lanes below)
  const int j = chunk * RASTER_THREADS + threadIdx.x;
  TriCam T;
  T.x0 = 1;
  T.x1 = T.y0 = T.y1 = 0;
  if (j < a.ntri) {
    const float4* tp = reinterpret_cast<const float4*>(a.mesh_tri) + 4 * (size_t)j;
    const int k = __float_as_int(tp[3].x) >> 16;
    if (k >= 0 && k < a.nmesh && mvis[k]) tri_setup(a, tp, mR[k], mc[k], tanh_, aspect, T);
  }
  const bool live = T.x0 <= T.x1 && T.y0 <= T.y1 && !(a.dbg & 32);  // (dbg 32, timing probe: set-up only)
  if ((a.dbg & 32) && T.x0 == -12345) a.vis[0] = 0;  // (keeps the probe's set-up alive)
  const int nx = T.x1 - T.x0 + 1;
  const int span = live ? nx * (T.y1 - T.y0 + 1) : 0;
  unsigned long long* vis = a.vis + (size_t)env * a.cam.width * a.cam.height;
  uint8_t* tflag = a.tflag + (size_t)env * a.tiles_x * a.tiles_y;
  // A small projection (most: a 1 mm-LOD triangle spans a few pixels) is covered by its own lane;
  // the wave's larger ones one after the other by all 64 lanes, the triangle broadcast from its lane
  // by readlane.  (Dealing all of the wave's pixel centres out evenly over the lanes -- a scan and a
  // max-scan through LDS per 64 centres -- measured 2x slower: latency-bound LDS round trips.)
  if (live && span <= RASTER_SMALL)
    for (int py = T.y0; py <= T.y1; ++py)
      for (int px = T.x0; px <= T.x1; ++px) tri_cover(a, T, (unsigned)j, px, py, tanh_, aspect, vis, tflag);
  unsigned long long bigs = __ballot(live && span > RASTER_SMALL);
  const int lane = threadIdx.x & 63;
  while (bigs) {
    const int l = __builtin_ctzll(bigs);
    bigs &= bigs - 1;
    TriCam B;
    for (int i = 0; i < 3; i++) {
      B.v0[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(T.v0[i]), l));
      B.e1[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(T.e1[i]), l));
      B.e2[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(T.e2[i]), l));
    }
    for (int i = 0; i < 4; i++) {
      B.ea[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(T.ea[i]), l));
      B.eb[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(T.eb[i]), l));
      B.ec[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(T.ec[i]), l));
    }
    const int bx0 = __builtin_amdgcn_readlane(T.x0, l), by0 = __builtin_amdgcn_readlane(T.y0, l);
    const int bnx = __builtin_amdgcn_readlane(nx, l), np = __builtin_amdgcn_readlane(span, l);
    const unsigned jb = (unsigned)__builtin_amdgcn_readlane(j, l);
    // lane i walks centres i, i + 64, ...: row and column stepped (64 = q nx + r), no division
    const int q = 64 / bnx, r = 64 - q * bnx;
    int yy = lane / bnx, xx = lane - yy * bnx;
    for (int i = lane; i < np; i += 64) {
      tri_cover(a, B, jb, bx0 + xx, by0 + yy, tanh_, aspect, vis, tflag);
      xx += r;
      yy += q;
      if (xx >= bnx) {
        xx -= bnx;
        ++yy;
      }
    }
  }
}

// RMBX_RENDER_MINW: minimum waves per SIMD the register allocation targets: 8 (default; 64
// registers, 136 B/lane of spilled set-up values, none in the ray loop's hot path) -- per
// 1024-env 8-bit frame 5.74-5.79 ms vs 6.46 at 5 waves (94 registers, no spills), 6.06 at 6,
// 5.82 at 7 and 7.35-7.44 unconstrained (98 registers, 4 waves); identical images
// (profiles/r4_render_waves_ab.log); the other targets are build options for the A/B
// (scripts/build_variant.py render4 .. render7)
#ifndef RMBX_RENDER_MINW
#define RMBX_RENDER_MINW 8
#endif
// CM: 0 = no cache (every primitive in one pass), 1 = the envs whose cache is valid, 2 = the envs
// whose cache is rebuilt this call (rmbx_render_scene_cached launches 1 and 2 over all envs; each
// block of the other kind returns at once)
template <bool VIS, int CM>
__global__ void __launch_bounds__(256, RMBX_RENDER_MINW) render_kernel(RenderArgs a) {
  __shared__ PrimCam prims[MAX_PRIM];
  __shared__ int order[MAX_PRIM];        // the block's primitives sorted front to back, once
  __shared__ int tile_sorted[MAX_PRIM];  // the tile's survivors in that order
  __shared__ int wcount[4];
  __shared__ CamFrame cf;
  __shared__ float mR[VIS ? MAX_MESH : 1][9];  // mesh slots' body rotations in the camera frame
  __shared__ uint8_t pstat[MAX_PRIM];          // cached modes: 1 for a static primitive
  const int ntiles = a.tiles_x * a.tiles_y;
  const int env = blockIdx.x / a.groups;
  const int grp = blockIdx.x % a.groups;
  if (env >= a.n_env) return;
  if (a.active && !a.active[env]) return;
  const int tid = threadIdx.x;
  // 0: no cache (every primitive in one pass); 1: the env's cache is valid (the static scene comes
  // from it, only the other primitives are cast); 2: the cache is rebuilt (a static-only pass writes
  // it, then the mode-1 pass)
  constexpr int mode = CM;
  if (CM != 0 && (a.dirty[env] != 0) != (CM == 2)) return;
  const int W = a.cam.width, H = a.cam.height;
  const float tanh_ = tanf(0.5f * a.cam.fovy_deg * 3.14159265358979f / 180.0f);
  const float aspect = (float)W / (float)H;
  // cosine of the widest ray (image corner) against the view axis
  const float cos_max = rsqrtf(1.0f + tanh_ * tanh_ * (1.0f + aspect * aspect));
  if (tid == 0) camera_frame(a, env, cf);
  __syncthreads();
  if constexpr (VIS) {
    if (tid < a.nmesh) {
      float c[3];
      mesh_frame(a, env, tid, cf, mR[tid], c);
    }
  }
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
    // screen-space bound: the 8 corners of the primitive's box in its frame, projected (tighter
    // than the bounding sphere for long thin primitives)
    P.sx_lo = P.sy_lo = -1e30f;
    P.sx_hi = P.sy_hi = 1e30f;
    if (type != RMBX_GEOM_PLANE && rad > 0) {
      float bh[3] = {rad, rad, rad};
      if (type == RMBX_GEOM_BOX) {
        bh[0] = f[0]; bh[1] = f[1]; bh[2] = f[2];
      } else if (type == RMBX_GEOM_CAPSULE) {
        bh[0] = bh[1] = f[0]; bh[2] = f[0] + f[1];
      } else if (type == RMBX_GEOM_CYLINDER) {
        bh[0] = bh[1] = f[0]; bh[2] = f[1];
      }
      float xl = 1e30f, xh = -1e30f, yl = 1e30f, yh = -1e30f;
      bool front = true;
      for (int v = 0; v < 8; v++) {
        const float l[3] = {(v & 1) ? bh[0] : -bh[0], (v & 2) ? bh[1] : -bh[1], (v & 4) ? bh[2] : -bh[2]};
        float qc[3];
        for (int i = 0; i < 3; i++) qc[i] = P.c[i] + P.R[3 * i] * l[0] + P.R[3 * i + 1] * l[1] + P.R[3 * i + 2] * l[2];
        if (-qc[2] < 1e-3f) {
          front = false;
          break;
        }
        const float iz = 1.0f / -qc[2];
        xl = fminf(xl, qc[0] * iz);
        xh = fmaxf(xh, qc[0] * iz);
        yl = fminf(yl, qc[1] * iz);
        yh = fmaxf(yh, qc[1] * iz);
      }
      if (front) {
        P.sx_lo = xl - 1e-5f;
        P.sx_hi = xh + 1e-5f;
        P.sy_lo = yl - 1e-5f;
        P.sy_hi = yh + 1e-5f;
      }
    }
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
    pstat[p] = mode ? a.prim_static[p] : 0;
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
  const size_t hw = (size_t)H * W;
  // the per-pixel global reads of a tile are issued a tile ahead (the tile flag and, with the cache,
  // the cached static candidate) or at the tile's start (the mesh key), so their latency runs under
  // the previous tile's rays and this tile's culling instead of in front of the ray loop
  auto pix_of = [&](int t) {
    const int x = (t % a.tiles_x) * RENDER_TILE + (tid % RENDER_TILE), y = (t / a.tiles_x) * RENDER_TILE + (tid / RENDER_TILE);
    return (size_t)min(y, H - 1) * W + min(x, W - 1);  // (clamped: the loads of past-the-image lanes are unused)
  };
  uint2 nxt_ce = make_uint2(0u, 0u);
  uint8_t nxt_tv = 0;
  if (t_begin < t_end) {
    if (mode == 1) nxt_ce = a.cache[(size_t)env * hw + pix_of(t_begin)];
    if constexpr (VIS) nxt_tv = a.tflag[(size_t)env * ntiles + t_begin];
  }
  for (int tile = t_begin; tile < t_end; ++tile) {
  __syncthreads();  // the previous tile's rays are done with tile_sorted (and order is complete)
  const uint2 cur_ce = nxt_ce;
  const bool tile_vis = VIS && nxt_tv != 0;
  unsigned long long cur_key = VIS_EMPTY;
  if (VIS && tile_vis) cur_key = a.vis[(size_t)env * hw + pix_of(tile)];
  if (tile + 1 < t_end) {
    if (mode == 1) nxt_ce = a.cache[(size_t)env * hw + pix_of(tile + 1)];
    if constexpr (VIS) nxt_tv = a.tflag[(size_t)env * ntiles + tile + 1];
  }
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
      // the projected box against the tile's slope rectangle
      if (P.sx_hi < x_lo || P.sx_lo > x_hi || P.sy_hi < y_lo || P.sy_lo > y_hi) keep = false;
    }
    if (mode == 1 && pstat[p_cull]) keep = false;  // (the cache holds the static scene)
  }
  // compact the survivors in sorted order: ballot per wave, wave offsets through LDS
  const unsigned long long kb = __ballot(keep);
  if ((tid & 63) == 0) wcount[tid >> 6] = __popcll(kb);
  __syncthreads();
  int base = 0;
  for (int w = 0; w < (tid >> 6); ++w) base += wcount[w];
  if (keep) tile_sorted[base + __popcll(kb & ((1ull << (tid & 63)) - 1))] = p_cull;
  const int tile_cnt = wcount[0] + wcount[1] + wcount[2] + wcount[3];
  // did the visibility pass write a pixel of this tile? (the flag is consumed: cleared below, after
  // every lane has read it, with the pixels' keys, so the workspace is back to empty for the next
  // call without a clearing pass)
  __syncthreads();
  const int px = tx0 + (tid % RENDER_TILE), py = ty0 + (tid / RENDER_TILE);
  if (px < W && py < H) {
  const float d[3] = {((2.0f * (px + 0.5f) / W) - 1.0f) * tanh_ * aspect,
                      (1.0f - 2.0f * (py + 0.5f) / H) * tanh_, -1.0f};
  const size_t pix = (size_t)py * W + px;
  // the mesh candidate (the visibility pass's nearest triangle), kept for the final pass
  float m_best = 1e30f, m_n[3] = {0, 0, 1}, m_rgb[3] = {0.f, 0.f, 0.f};
  int m_geom = -1;
  if constexpr (VIS) {
    // the pixel's nearest mesh triangle from the visibility pass
    const unsigned long long key = cur_key;
    if (key != VIS_EMPTY) {
      a.vis[(size_t)env * hw + pix] = VIS_EMPTY;
      const unsigned j = (unsigned)key;
      const float4* tp = reinterpret_cast<const float4*>(a.mesh_tri) + 4 * (size_t)j;
      const float4 C = tp[2], D = tp[3];
      const int tag = __float_as_int(D.x), k = tag >> 16;
      m_best = __uint_as_float((unsigned)(key >> 32));
      m_geom = tag & 0xffff;
      m_rgb[0] = D.y;
      m_rgb[1] = D.z;
      m_rgb[2] = D.w;
      const float nl[3] = {C.y, C.z, C.w};
      for (int i = 0; i < 3; i++) m_n[i] = mR[k][3 * i] * nl[0] + mR[k][3 * i + 1] * nl[1] + mR[k][3 * i + 2] * nl[2];
    }
  }
  // the static scene's candidate (mode 1: from the cache; mode 2: from pass 0): depth, primitive
  // (0xff: none), 8-bit colour
  float c_t = 1e30f;
  unsigned c_p = 0xffu, c_rgb = 0u;
  if (mode == 1) {
    const uint2 ce = cur_ce;
    c_t = __uint_as_float(ce.x);
    c_p = ce.y >> 24;
    c_rgb = ce.y & 0xffffffu;
  }
  const int cnt = tile_cnt;
  int ntest = 0;
  float best, bn[3], brgb[3], col[3], depth;
  int bp, bgeom;  // the winning primitive / surface geom (-2: a primitive, -3: the cached static scene)
  uint8_t u[3];
  // one pass (modes 0, 1) or two (mode 2: the static-only scene into the cache, then the rest); a
  // single instance of the ray loop and the shading serves every pass, so the cached colours are
  // the ones the one-pass form computes
  auto pixel_pass = [&](const int pass) {
  if (pass == 0) {
    best = 1e30f;
    bgeom = -1;
    bn[0] = bn[1] = 0.f;
    bn[2] = 1.f;
    brgb[0] = brgb[1] = brgb[2] = 0.f;
  } else {
    best = m_best;
    bgeom = m_geom;
    for (int i = 0; i < 3; i++) {
      bn[i] = m_n[i];
      brgb[i] = m_rgb[i];
    }
  }
  bp = -1;
  if (pass == 1 && c_p != 0xffu && c_t < best) {  // (a triangle at the same depth keeps the pixel)
    best = c_t;
    bp = (int)c_p;
    bgeom = -3;
  }
  for (int k = 0; k < ((a.dbg & 1) ? 0 : cnt); k++) {
    const int p = tile_sorted[k];
    const PrimCam& P = prims[p];
    if (P.zmin > best + 1e-4f) break;  // every later primitive lies behind the current hit
    if (mode == 2 && (pass == 0) != (pstat[p] != 0)) continue;  // pass 0: static only; pass 1: the others
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
    if (h && (t < best || (t == best && bp >= 0 && p < bp))) {
      best = t;
      bp = p;
      bgeom = -2;
      // normal back to camera frame
      for (int i = 0; i < 3; i++) bn[i] = P.R[3 * i] * nl[0] + P.R[3 * i + 1] * nl[1] + P.R[3 * i + 2] * nl[2];
    }
  }
  const bool prim_won = bgeom == -2;
  const bool cached = bgeom == -3;
  if (cached) bgeom = a.prim_i32[4 * bp];
  if (prim_won) {  // a primitive won: its geom and material colour
    bgeom = a.prim_i32[4 * bp];
    brgb[0] = prims[bp].rgb[0];
    brgb[1] = prims[bp].rgb[1];
    brgb[2] = prims[bp].rgb[2];
  }
  depth = a.cam.zfar;
  const float inv = rsqrtf(dot3f(d, d));
  const float vd[3] = {d[0] * inv, d[1] * inv, d[2] * inv};
  if (cached) {  // the cached static scene: its 8-bit colour as the shading below made it
    depth = best;
    col[0] = col[1] = col[2] = 0.f;
  } else if (bgeom < 0) {
    if (a.geom_matinfo) {
      // the gradient skybox: rgb2 (down) to rgb1 (up) by the ray's world z
      const float wz = cf.R[6] * vd[0] + cf.R[7] * vd[1] + cf.R[8] * vd[2];
      const float f = 0.5f * (1.f + wz);
      for (int i = 0; i < 3; i++) col[i] = a.sky[3 + i] + f * (a.sky[i] - a.sky[3 + i]);
    } else {
      col[0] = 0.9f;  // skybox gradient colour of env_ur5e_common.xml
      col[1] = 1.0f;
      col[2] = 1.0f;
    }
  } else {
    float ndv = -(bn[0] * vd[0] + bn[1] * vd[1] + bn[2] * vd[2]);
    if (ndv < 0) {
      ndv = -ndv;
      bn[0] = -bn[0];
      bn[1] = -bn[1];
      bn[2] = -bn[2];
    }
    // directional light pointing down (world -z): L = world +z in the camera frame
    const float L[3] = {cf.R[6], cf.R[7], cf.R[8]};
    float ndl = bn[0] * L[0] + bn[1] * L[1] + bn[2] * L[2];
    ndl = ndl > 0 ? ndl : 0;
    const float shade = 0.1f + 0.6f * ndv + 0.3f * ndl;
    if (a.geom_matinfo) {
      const float* mi = a.geom_matinfo + 6 * bgeom;
      float tc[3] = {1.f, 1.f, 1.f};
      if (prim_won) {
        const int tex = (a.dbg & 256) ? -1 : a.geom_texid[bgeom];  // (timing probe 256: no sampling)
        if (tex >= 0) {
          const PrimCam& P = prims[bp];
          float o_l[3], d_l[3];
          to_local(P, d, o_l, d_l);
          const float pl[3] = {o_l[0] + best * d_l[0], o_l[1] + best * d_l[1], o_l[2] + best * d_l[2]};
          // the pixel's footprint on the surface: one pixel's step of the ray slope (2 tan(fovy/2)
          // / H, square pixels) at camera depth t, over the cosine to the normal
          const float foot = best * (2.0f * tanh_ / H) / fmaxf(ndv, 1e-3f);
          sample_texture(a, tex, P.type, P.s, mi, pl, foot, tc);
        }
      }
      float sp = 0.f;
      if (ndl > 0.f && mi[0] > 0.f) {
        // Blinn-Phong half vector of the light and the viewer (-vd)
        float h[3] = {L[0] - vd[0], L[1] - vd[1], L[2] - vd[2]};
        const float hi = rsqrtf(dot3f(h, h));
        const float nh = fmaxf((bn[0] * h[0] + bn[1] * h[1] + bn[2] * h[2]) * hi, 0.f);
        sp = mi[0] * 0.3f * powf(nh, 128.f * mi[1]);
      }
      for (int i = 0; i < 3; i++) col[i] = fminf(brgb[i] * tc[i] * (shade + mi[5]) + sp, 1.0f);
    } else {
      for (int i = 0; i < 3; i++) col[i] = fminf(brgb[i] * shade, 1.0f);
    }
    depth = best;  // d has unit -z component: t is the camera-z distance
  }
  if (cached) {
    u[0] = (uint8_t)(c_rgb & 255u);
    u[1] = (uint8_t)((c_rgb >> 8) & 255u);
    u[2] = (uint8_t)(c_rgb >> 16);
  } else {
    for (int i = 0; i < 3; i++) u[i] = (uint8_t)(col[i] * 255.0f + 0.5f);
  }
  if (pass == 0) {  // the static-only scene of this pixel: into the cache and the final pass
    c_t = best;
    c_p = bp >= 0 ? (unsigned)bp : 0xffu;
    c_rgb = (unsigned)u[0] | ((unsigned)u[1] << 8) | ((unsigned)u[2] << 16);
    a.cache[(size_t)env * hw + pix] = make_uint2(__float_as_uint(c_t), c_rgb | (c_p << 24));
  }
  };  // pixel_pass
  if constexpr (CM == 2) {
#pragma nounroll
    for (int pass = 0; pass < 2; ++pass) pixel_pass(pass);
  } else {
    pixel_pass(1);
  }
  const bool do_store = !(a.dbg & 2) || col[0] == 12345.f;  // (diagnostic: keep the shading live)
  if (a.rgb && do_store) {
    uint8_t* o = a.rgb + ((size_t)env * hw + pix) * 3;
    o[0] = u[0];
    o[1] = u[1];
    o[2] = u[2];
  }
  if (a.depth && do_store) a.depth[(size_t)env * hw + pix] = (a.dbg & 4) ? (float)(ntest + 1000 * cnt) : depth;
  if (a.hit_geom && do_store) a.hit_geom[(size_t)env * hw + pix] = bgeom;
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
  if (VIS && tid == 0 && tile_vis) a.tflag[(size_t)env * ntiles + tile] = 0;
  }  // tiles
}

// Static-background cache validity, one wave per env: the camera body's pose and every static
// primitive's pose are compared (exactly) with the snapshot the env's cache was built from; any
// difference (or the NaN snapshot of a new cache) marks the env dirty -- its render pass rebuilds
// the cache -- and takes the new snapshot.
__global__ void __launch_bounds__(64) render_cache_check_kernel(RenderArgs a, const int32_t* static_prims,
                                                               int nstatic, double* snap, uint8_t* dirty) {
  const int env = blockIdx.x;
  if (a.active && !a.active[env]) return;
  const int n = 7 + 12 * nstatic, body = a.cam.body;
  double* sn = snap + (size_t)env * n;
  auto value = [&](int i) -> double {
    if (i < 3) return a.xpos[((size_t)env * a.nbody + body) * 3 + i];
    if (i < 7) return a.xquat[((size_t)env * a.nbody + body) * 4 + i - 3];
    const int j = (i - 7) / 12, k = (i - 7) - 12 * j;
    const int g = a.prim_i32[4 * static_prims[j]];
    return k < 3 ? a.gxpos[((size_t)env * a.ngeom + g) * 3 + k] : a.gxmat[((size_t)env * a.ngeom + g) * 9 + k - 3];
  };
  bool diff = false;
  for (int i = threadIdx.x; i < n; i += 64) diff = diff || !(value(i) == sn[i]);
  const bool any = __any(diff);
  if (any)
    for (int i = threadIdx.x; i < n; i += 64) sn[i] = value(i);
  if (threadIdx.x == 0) dirty[env] = any ? 1 : 0;
}

}  // namespace rmbx

extern "C" int rmbx_render_scene_cached(const rmbx_camera* cam, const rmbx_scene_tables* scene,
                                        const double* gxpos, const double* gxmat, const double* xpos,
                                        const double* xquat, int ngeom, int nbody, uint8_t* rgb, float* depth,
                                        int32_t* hit_geom, void* policy_img, int policy_dtype,
                                        const uint8_t* active, int n_env, const rmbx_render_cache* cache,
                                        void* stream) {
  RMBX_CHECK_ARG(cam && scene && scene->prim_i32 && scene->prim_f32 && gxpos && gxmat && xpos && xquat,
                 "NULL argument");
  RMBX_CHECK_ARG(scene->nprim > 0 && scene->nprim <= MAX_PRIM, "nprim=%d outside [1, %d]", scene->nprim, MAX_PRIM);
  RMBX_CHECK_ARG(cam->width > 0 && cam->height > 0 && cam->width <= 8192 && cam->height <= 8192,
                 "bad image size %dx%d", cam->width, cam->height);
  RMBX_CHECK_ARG(cam->body >= 0 && cam->body < nbody, "bad camera body %d", cam->body);
  RMBX_CHECK_ARG(policy_dtype >= 0 && policy_dtype <= 4,
                 "policy_dtype must be 0 (f32), 1 (bf16), 2 (bf16 s2d), 3 (f32 s2d) or 4 (u8 s2d)");
  RMBX_CHECK_ARG(policy_dtype < 2 || (cam->width % 2 == 0 && cam->height % 2 == 0),
                 "space-to-depth policy output needs an even image size");
  RMBX_CHECK_ARG(!scene->geom_matinfo ||
                     (scene->geom_texid && (scene->ntex == 0 || (scene->tex_rgba && scene->tex_desc && scene->tex_level_adr))),
                 "materials need geom_texid, and tex_rgba / tex_desc / tex_level_adr when ntex > 0");
  const bool meshes = scene->ntri > 0;
  RMBX_CHECK_ARG(scene->ntri >= 0 && scene->ntri < (1 << 26) && scene->nmesh >= 0 && scene->nmesh <= MAX_MESH,
                 "bad mesh sizes (ntri=%d, nmesh=%d, at most %d mesh bodies)", scene->ntri, scene->nmesh, MAX_MESH);
  RMBX_CHECK_ARG(!meshes || (scene->mesh_tri && scene->mesh_body && scene->mesh_rad && scene->vis &&
                             scene->tflag &&
                             scene->nmesh > 0 && (((uintptr_t)scene->mesh_tri | (uintptr_t)scene->vis) & 15) == 0),
                 "meshes need mesh_tri / mesh_body / mesh_rad / vis (16-byte aligned) / tflag and nmesh > 0");
  if (n_env == 0) return RMBX_OK;
  rmbx::RenderArgs a;
  a.cam = *cam;
  a.prim_i32 = scene->prim_i32;
  a.prim_f32 = scene->prim_f32;
  a.nprim = scene->nprim;
  a.mesh_tri = scene->mesh_tri;
  a.ntri = meshes ? scene->ntri : 0;
  a.nmesh = meshes ? scene->nmesh : 0;
  a.mesh_body = scene->mesh_body;
  a.mesh_rad = scene->mesh_rad;
  a.vis = meshes ? scene->vis : nullptr;
  a.tflag = meshes ? scene->tflag : nullptr;
  a.hit_geom = hit_geom;
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
  a.geom_matinfo = scene->geom_matinfo;
  a.geom_texid = scene->geom_texid;
  a.tex_rgba = scene->tex_rgba;
  a.tex_desc = reinterpret_cast<const int4*>(scene->tex_desc);
  a.tex_level_adr = scene->tex_level_adr;
  for (int i = 0; i < 6; i++) a.sky[i] = scene->sky_rgb[i];
  a.prim_static = nullptr;
  a.cache = nullptr;
  a.dirty = nullptr;
  const char* cache_env = std::getenv("RMBX_RENDER_CACHE");  // 0: render every pixel in full (A/B)
  const bool use_cache = cache && cache->nstatic > 0 && !(cache_env && std::atoi(cache_env) == 0);
  if (use_cache) {
    RMBX_CHECK_ARG(cache->prim_static && cache->static_prims && cache->cache && cache->snap && cache->dirty &&
                       ((uintptr_t)cache->cache & 7) == 0 && cache->nstatic <= scene->nprim,
                   "rmbx_render_scene_cached: bad cache (null pointer, unaligned cache or nstatic=%d > nprim=%d)",
                   cache->nstatic, scene->nprim);
    RMBX_CHECK_ARG(cam->body >= 0 && cam->body < nbody && xpos && xquat, "rmbx_render_scene_cached: bad camera body");
    a.prim_static = cache->prim_static;
    a.cache = reinterpret_cast<uint2*>(cache->cache);
    a.dirty = cache->dirty;
  }
  a.tiles_x = (cam->width + RENDER_TILE - 1) / RENDER_TILE;
  a.tiles_y = (cam->height + RENDER_TILE - 1) / RENDER_TILE;
  // blocks per env of the ray-cast pass (each a contiguous range of tiles), chosen so the grid fills
  // whole rounds of the chip's block slots (CUs x RMBX_RENDER_MINW resident 4-wave blocks): front
  // camera, 1024 envs, cached, 1536 slots (profiles/r6_render_groups_ab.log): 3.35 / 3.39 ms at 6 / 12
  // groups (4 / 8 full rounds) vs 3.70 at 8 (5.3 rounds) and 4.49 at 16 (10.7): the last partial
  // round of 75-tile blocks is the cost.  The largest g in [6, max(12, 2 slots / n)] with the best
  // round fill; RMBX_RENDER_GROUPS overrides (A/B)
  const char* ge = std::getenv("RMBX_RENDER_GROUPS");
  const int ntl = a.tiles_x * a.tiles_y;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  if (ge) {
    a.groups = std::atoi(ge);
  } else {
    const long long slots = (long long)cus * RMBX_RENDER_MINW;
    const int gmax = (int)std::min<long long>(ntl, std::max<long long>(12, (2 * slots + n_env - 1) / n_env));
    int best = std::min(6, ntl);
    double best_fill = -1.0;
    for (int g = std::min(6, ntl); g <= gmax; ++g) {
      const long long b = (long long)n_env * g, rounds = (b + slots - 1) / slots;
      const double fill = (double)b / (double)(rounds * slots);
      if (fill >= best_fill - 1e-12) {
        best_fill = fill;
        best = g;
      }
    }
    a.groups = best;
  }
  RMBX_CHECK_ARG(a.groups >= 1 && a.groups <= a.tiles_x * a.tiles_y, "RMBX_RENDER_GROUPS=%d out of range", a.groups);
  const char* dbg_env = std::getenv("RMBX_RENDER_DBG");
  a.dbg = dbg_env ? std::atoi(dbg_env) : 0;
  const size_t nblocks = (size_t)n_env * a.groups;
  RMBX_CHECK_ARG(nblocks < (1ull << 31), "grid too large");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (use_cache) {
    hipLaunchKernelGGL(rmbx::render_cache_check_kernel, dim3((unsigned)n_env), dim3(64), 0, st, a,
                       cache->static_prims, (int)cache->nstatic, cache->snap, cache->dirty);
    RMBX_CHECK_LAUNCH();
  }
  if (meshes) {
    // pass 1: the meshes' nearest triangle per pixel into the visibility buffer (empty on entry:
    // the ray-cast pass clears every key and tile flag it consumes)
    const int chunks = (scene->ntri + RASTER_THREADS - 1) / RASTER_THREADS;
    const size_t rblocks = (size_t)chunks * n_env;
    RMBX_CHECK_ARG(rblocks < (1ull << 31), "raster grid too large");
    hipLaunchKernelGGL(rmbx::raster_kernel, dim3((unsigned)rblocks), dim3(RASTER_THREADS), 0, st, a, chunks);
    RMBX_CHECK_LAUNCH();
    if (use_cache) {
      hipLaunchKernelGGL((rmbx::render_kernel<true, 1>), dim3((unsigned)nblocks), dim3(256), 0, st, a);
      RMBX_CHECK_LAUNCH();
      hipLaunchKernelGGL((rmbx::render_kernel<true, 2>), dim3((unsigned)nblocks), dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL((rmbx::render_kernel<true, 0>), dim3((unsigned)nblocks), dim3(256), 0, st, a);
    }
  } else if (use_cache) {
    hipLaunchKernelGGL((rmbx::render_kernel<false, 1>), dim3((unsigned)nblocks), dim3(256), 0, st, a);
    RMBX_CHECK_LAUNCH();
    hipLaunchKernelGGL((rmbx::render_kernel<false, 2>), dim3((unsigned)nblocks), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((rmbx::render_kernel<false, 0>), dim3((unsigned)nblocks), dim3(256), 0, st, a);
  }
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_render_scene(const rmbx_camera* cam, const rmbx_scene_tables* scene, const double* gxpos,
                                 const double* gxmat, const double* xpos, const double* xquat, int ngeom,
                                 int nbody, uint8_t* rgb, float* depth, int32_t* hit_geom, void* policy_img,
                                 int policy_dtype, const uint8_t* active, int n_env, void* stream) {
  return rmbx_render_scene_cached(cam, scene, gxpos, gxmat, xpos, xquat, ngeom, nbody, rgb, depth, hit_geom,
                                  policy_img, policy_dtype, active, n_env, nullptr, stream);
}

extern "C" int rmbx_render(const rmbx_camera* cam, const int32_t* prim_i32, const float* prim_f32,
                           int nprim, const double* gxpos, const double* gxmat, const double* xpos,
                           const double* xquat, int ngeom, int nbody, uint8_t* rgb, float* depth,
                           void* policy_img, int policy_dtype, const uint8_t* active, int n_env,
                           void* stream) {
  rmbx_scene_tables sc{};
  sc.prim_i32 = prim_i32;
  sc.prim_f32 = prim_f32;
  sc.nprim = nprim;
  return rmbx_render_scene(cam, &sc, gxpos, gxmat, xpos, xquat, ngeom, nbody, rgb, depth, nullptr, policy_img,
                           policy_dtype, active, n_env, stream);
}
