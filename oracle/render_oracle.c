/* ORACLE -- test infrastructure only (tests/, never the product path).
 *
 * Brute-force f64 ray caster restating the batched renderer (csrc/rmbx_render.hip), which replaces
 * the per-camera OpenGL renders of envs/mujoco/MujocoEnvBase.py:103-126: every ray is tested
 * against EVERY drawn primitive and EVERY triangle of every drawn mesh (no tiles, no culling, no
 * depth-bound ordering, no BVH), so a culling, ordering, traversal or indexing error of the kernel
 * shows up as a pixel whose surface or depth differs.  Geometry conventions (the kernel's
 * documented contract): primitives in their frame (world = R local + c: a geom's gxpos / gxmat, a
 * body's meshes in the body's xpos / xquat, each triangle carrying its geom id and colour);
 * plane = local z = 0, unbounded; sphere / capsule / cylinder / box as MuJoCo sizes them; a camera
 * inside a primitive sees none of it; hits at t <= 1e-4 ignored; triangles one-sided (back faces
 * culled: MuJoCo's default mjRND_CULL_FACE) and clipped at t <= znear; nearest hit wins.  Shading 0.1 + 0.6 |n.v| + 0.3 max(0, n_z) (normal turned to the
 * viewer, light along world -z), times the material colour, clamped at 1; background (0.9, 1, 1);
 * with materials (round 6) the colour times the primitive's texture sample (2d / cube, trilinear
 * over the mip pyramid, level of detail from the pixel's isotropic footprint) plus the emission, the light's
 * Blinn-Phong specular term, and the gradient skybox behind.
 * Parity is "unpinned" against MuJoCo's OpenGL renderer (not in the image); this checks the ray
 * caster against its own specification.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORC_PI 3.14159265358979323846

typedef struct {
  int32_t geom, type;  /* type: 0 plane, 2 sphere, 3 capsule, 5 cylinder, 6 box, 7 mesh (geom: -1) */
  int32_t tri0, ntri;  /* mesh: triangle range in the triangle table */
  double size[3];      /* mesh: size[0] = bounding radius about the frame origin */
  double rgb[3];
  double pos[3], R[9]; /* frame: world = R local + pos (R row-major) */
} orc_prim;

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

static int hit_sphere(const double* o, const double* d, double r, double* t, double* n) {
  const double b = dot3(o, d), c = dot3(o, o) - r * r;
  if (c < 0) return 0;
  const double a = dot3(d, d), disc = b * b - a * c;
  if (disc < 0) return 0;
  const double sq = sqrt(disc);
  double tt = (-b - sq) / a;
  if (tt <= 1e-4) tt = (-b + sq) / a;
  if (tt <= 1e-4) return 0;
  *t = tt;
  for (int i = 0; i < 3; i++) n[i] = (o[i] + tt * d[i]) / r;
  return 1;
}

static int hit_cylinder(const double* o, const double* d, double r, double h, int caps, double* t, double* n) {
  double best = 1e300;
  int hit = 0;
  if (o[0] * o[0] + o[1] * o[1] < r * r && fabs(o[2]) < h + (caps ? 0.0 : r)) return 0;
  const double a = d[0] * d[0] + d[1] * d[1];
  if (a > 1e-24) {
    const double b = o[0] * d[0] + o[1] * d[1], c = o[0] * o[0] + o[1] * o[1] - r * r;
    const double disc = b * b - a * c;
    if (disc >= 0) {
      const double sq = sqrt(disc);
      for (int k = 0; k < 2; k++) {
        const double tt = (-b + (k == 0 ? -sq : sq)) / a;
        if (tt > 1e-4 && tt < best && fabs(o[2] + tt * d[2]) <= h) {
          best = tt;
          n[0] = (o[0] + tt * d[0]) / r;
          n[1] = (o[1] + tt * d[1]) / r;
          n[2] = 0;
          hit = 1;
        }
      }
    }
  }
  if (caps && fabs(d[2]) > 1e-24) {
    for (int k = 0; k < 2; k++) {
      const double zc = k == 0 ? h : -h, tt = (zc - o[2]) / d[2];
      const double x = o[0] + tt * d[0], y = o[1] + tt * d[1];
      if (tt > 1e-4 && tt < best && x * x + y * y <= r * r) {
        best = tt;
        n[0] = n[1] = 0;
        n[2] = k == 0 ? 1 : -1;
        hit = 1;
      }
    }
  }
  *t = best;
  return hit;
}

static int hit_capsule(const double* o, const double* d, double r, double h, double* t, double* n) {
  double best = 1e300, tb, nb[3];
  int hit = hit_cylinder(o, d, r, h, 0, &tb, nb);
  if (hit) {
    best = tb;
    for (int i = 0; i < 3; i++) n[i] = nb[i];
  }
  for (int k = 0; k < 2; k++) {
    const double oc[3] = {o[0], o[1], o[2] - (k == 0 ? h : -h)};
    double ts, ns[3];
    if (hit_sphere(oc, d, r, &ts, ns) && ts < best) {
      const double z = oc[2] + ts * d[2];
      if ((k == 0 && z >= 0) || (k == 1 && z <= 0)) {
        best = ts;
        for (int i = 0; i < 3; i++) n[i] = ns[i];
        hit = 1;
      }
    }
  }
  *t = best;
  return hit;
}

static int hit_box(const double* o, const double* d, const double* s, double* t, double* n) {
  double tmin = -1e300, tmax = 1e300;
  int axis = 0;
  for (int i = 0; i < 3; i++) {
    if (fabs(d[i]) < 1e-24) {
      if (fabs(o[i]) > s[i]) return 0;
      continue;
    }
    double t1 = (-s[i] - o[i]) / d[i], t2 = (s[i] - o[i]) / d[i];
    if (t1 > t2) {
      const double x = t1;
      t1 = t2;
      t2 = x;
    }
    if (t1 > tmin) {
      tmin = t1;
      axis = i;
    }
    if (t2 < tmax) tmax = t2;
    if (tmin > tmax) return 0;
  }
  if (tmax <= 1e-4 || tmin <= 1e-4) return 0;
  *t = tmin;
  n[0] = n[1] = n[2] = 0;
  n[axis] = d[axis] > 0 ? -1 : 1;
  return 1;
}

/* triangle record (mjcf/rmesh.py): f32 [16] = v0, e1, e2, unit normal, tag (int32 bits: mesh slot << 16 |
   geom id), rgb */
static int hit_tri(const double* o, const double* d, const float* tr, double tmin, double* t) {
  const double v0[3] = {tr[0], tr[1], tr[2]}, e1[3] = {tr[3], tr[4], tr[5]}, e2[3] = {tr[6], tr[7], tr[8]};
  /* back faces are culled (MuJoCo's default mjRND_CULL_FACE, OpenGL counter-clockwise front faces):
     a triangle whose winding normal e1 x e2 does not point towards the eye is not drawn */
  const double nw[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
  if (nw[0] * (o[0] - v0[0]) + nw[1] * (o[1] - v0[1]) + nw[2] * (o[2] - v0[2]) <= 0) return 0;
  const double p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
  const double det = dot3(e1, p);
  if (fabs(det) < 1e-300) return 0;
  const double s[3] = {o[0] - v0[0], o[1] - v0[1], o[2] - v0[2]};
  const double u = dot3(s, p) / det;
  if (u < 0 || u > 1) return 0;
  const double q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
  const double v = dot3(d, q) / det;
  if (v < 0 || u + v > 1) return 0;
  const double tt = dot3(e2, q) / det;
  if (tt <= tmin) return 0;
  *t = tt;
  return 1;
}

/* nearest and second-nearest surfaces of distinct geoms along a ray */
typedef struct {
  double t, n[3], rgb[3];
  int geom;
  double t2;  /* nearest hit of any other geom (1e300: none) */
  const orc_prim* prim; /* the nearest surface's primitive (NULL: a mesh triangle) */
  double pl[3];         /* its hit point in the primitive's frame */
} orc_best;

static void consider(orc_best* b, double t, int geom, const double* n, const double* rgb, const orc_prim* prim,
                     const double* pl) {
  if (t < b->t || (t == b->t && geom < b->geom)) {
    if (geom != b->geom && b->t < b->t2) b->t2 = b->t;
    b->t = t;
    b->geom = geom;
    b->prim = prim;
    for (int i = 0; i < 3; i++) {
      b->n[i] = n[i];
      b->rgb[i] = rgb[i];
      b->pl[i] = pl ? pl[i] : 0.0;
    }
  } else if (geom != b->geom && t < b->t2) {
    b->t2 = t;
  }
}

/* Materials (the renderer's contract, include/rmbx.h rmbx_scene_tables): per geom its texture
 * (-1: none) and (specular, shininess, texrepeat x, y, texuniform, emission); textures (type 0 2d /
 * 1 cube, height, width, first texel) over RGB texels in file row order; the skybox gradient rgb1
 * (up) / rgb2 (down).  NULL: flat material colours, no specular, background (0.9, 1, 1). */
typedef struct {
  const int32_t* geom_texid;
  const float* geom_matinfo;
  const uint8_t* tex_rgb;
  const int32_t* tex_desc;
  double sky[6];
} orc_materials;

static void orc_texel(const uint8_t* t, long idx, double w, double* c) {
  for (int i = 0; i < 3; i++) c[i] += w * (double)t[3 * idx + i];
}

/* bilinear at continuous texel coordinates (texel centres at integers), wrapped (2d) or clamped
   at the edges (cube faces) */
static void orc_bilinear(const uint8_t* t, int H, int W, double fx, double fy, int wrap, double* c) {
  const double x0f = floor(fx), y0f = floor(fy), ax = fx - x0f, ay = fy - y0f;
  long x0 = (long)x0f, y0 = (long)y0f, x1 = x0 + 1, y1 = y0 + 1;
  if (wrap) {
    x0 = ((x0 % W) + W) % W; x1 = ((x1 % W) + W) % W;
    y0 = ((y0 % H) + H) % H; y1 = ((y1 % H) + H) % H;
  } else {
    x0 = x0 < 0 ? 0 : (x0 > W - 1 ? W - 1 : x0); x1 = x1 < 0 ? 0 : (x1 > W - 1 ? W - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 > H - 1 ? H - 1 : y0); y1 = y1 < 0 ? 0 : (y1 > H - 1 ? H - 1 : y1);
  }
  c[0] = c[1] = c[2] = 0.0;
  orc_texel(t, y0 * W + x0, (1 - ax) * (1 - ay), c);
  orc_texel(t, y0 * W + x1, ax * (1 - ay), c);
  orc_texel(t, y1 * W + x0, (1 - ax) * ay, c);
  orc_texel(t, y1 * W + x1, ax * ay, c);
  for (int i = 0; i < 3; i++) c[i] /= 255.0;
}

/* texture coordinates in base-level texel units (fx = u W, fy = v H) of local point q and the
   texture's density there (base texels per metre along the surface): 2d from (x, y); cube maps on
   the major axis' face, OpenGL's face orientation */
static void orc_tex_coords(int ttype, int H, int W, const orc_prim* P, const float* mi, const double* pl,
                           double* fx, double* fy, double* dens) {
  const int uni = mi[4] != 0.0f;
  const double* s = P->size;
  if (ttype == 0) { /* 2d: (x, y), texrepeat over the geom's extent, or per metre */
    const double sx = s[0], sy = (P->type == 6 || P->type == 0) ? s[1] : s[0];
    double u = pl[0] * mi[2], v = pl[1] * mi[3], kx = mi[2], ky = mi[3];
    if (!uni && sx > 0 && sy > 0) {
      kx = mi[2] / (2 * sx);
      ky = mi[3] / (2 * sy);
      u = mi[2] * (pl[0] / (2 * sx) + 0.5);
      v = mi[3] * (pl[1] / (2 * sy) + 0.5);
    }
    *fx = u * W;
    *fy = v * H;
    *dens = kx * W > ky * H ? kx * W : ky * H;
    return;
  }
  double q[3] = {pl[0], pl[1], pl[2]}, hmin = 1;
  if (uni) { /* the unit object: local point over the half extents */
    double h[3] = {s[0], s[0], s[0]};
    if (P->type == 6) { h[1] = s[1]; h[2] = s[2]; }
    else if (P->type == 3) h[2] = s[1] + s[0];
    else if (P->type == 5) h[2] = s[1];
    else if (P->type == 0) { h[1] = s[1]; h[2] = 1; }
    for (int i = 0; i < 3; i++) q[i] = h[i] > 0 ? q[i] / h[i] : q[i];
    for (int i = 0; i < 3; i++) {
      const double hi = h[i] > 0 ? h[i] : 1;
      if (i == 0 || hi < hmin) hmin = hi;
    }
  }
  const double x = fabs(q[0]), y = fabs(q[1]), z = fabs(q[2]);
  double sc, tc, ma;
  if (x >= y && x >= z) {
    ma = x; sc = q[0] > 0 ? -q[2] : q[2]; tc = -q[1];
  } else if (y >= z) {
    ma = y; sc = q[0]; tc = q[1] > 0 ? q[2] : -q[2];
  } else {
    ma = z; sc = q[2] > 0 ? q[0] : -q[0]; tc = -q[1];
  }
  if (!(ma > 1e-300)) ma = 1e-300;
  *fx = 0.5 * (sc / ma + 1) * W;
  *fy = 0.5 * (tc / ma + 1) * H;
  *dens = 0.5 * (W > H ? W : H) / ma / hmin;
}

/* the texture colour of a primitive at its local hit point pl, trilinear (GL_LINEAR_MIPMAP_LINEAR)
   with an isotropic footprint: the pixel spans `foot` metres of the surface, the level of detail is
   log2(foot x density); the pyramid's level l (max(H >> l, 1) x max(W >> l, 1)) follows the levels
   before it */
static void orc_texture(const orc_materials* M, int tex, const orc_prim* P, const float* mi, const double* pl,
                        double foot, double* c) {
  const int32_t* td = M->tex_desc + 4 * tex;
  const uint8_t* t = M->tex_rgb + 3 * (long)td[3];
  const int H = td[1], W = td[2];
  double fx, fy, dens;
  orc_tex_coords(td[0], H, W, P, mi, pl, &fx, &fy, &dens);
  const double rho = foot * dens;
  int levels = 1;
  while ((H >> levels) > 0 || (W >> levels) > 0) ++levels;
  double lod = log2(rho > 1e-300 ? rho : 1e-300);
  lod = lod < 0 ? 0 : (lod > levels - 1 ? levels - 1 : lod);
  const int l0 = (int)lod;
  const double fr = lod - l0;
  const int wrap = td[0] == 0;
  long off = 0;
  for (int l = 0; l < l0; l++) off += (long)((H >> l) > 1 ? (H >> l) : 1) * ((W >> l) > 1 ? (W >> l) : 1);
  double c0[3], c1[3];
  int Hl = (H >> l0) > 1 ? (H >> l0) : 1, Wl = (W >> l0) > 1 ? (W >> l0) : 1;
  orc_bilinear(t + 3 * off, Hl, Wl, fx * Wl / W - 0.5, fy * Hl / H - 0.5, wrap, c0);
  if (fr > 0 && l0 + 1 < levels) {
    off += (long)Hl * Wl;
    Hl = (H >> (l0 + 1)) > 1 ? (H >> (l0 + 1)) : 1;
    Wl = (W >> (l0 + 1)) > 1 ? (W >> (l0 + 1)) : 1;
    orc_bilinear(t + 3 * off, Hl, Wl, fx * Wl / W - 0.5, fy * Hl / H - 0.5, wrap, c1);
  } else {
    for (int i = 0; i < 3; i++) c1[i] = c0[i];
  }
  for (int i = 0; i < 3; i++) c[i] = c0[i] + fr * (c1[i] - c0[i]);
}

/* Cast `nray` camera rays: pix [nray][2] = continuous pixel coordinates (x, y), pixel centres at
 * +0.5; cam_R [9] row-major with columns = camera axes in world, cam_p [3]; the ray of (x, y) is
 * R (u tan(fovy/2) aspect, v tan(fovy/2), -1) with u = 2x/W - 1, v = 1 - 2y/H.  Outputs per ray:
 * the hit geom (-1: background), its camera depth t, the shaded colour (f64, before the 8-bit
 * rounding) and the depth of the nearest hit of any OTHER geom (out_depth2, 1e300 if none: a
 * coincident surface there makes the pixel's geom a tie). */
void orc_render_rays(const orc_prim* prims, int nprim, const float* tri, const double* cam_R, const double* cam_p,
                     double fovy_deg, int W, int H, double znear, const double* pix, int nray, int32_t* out_geom,
                     double* out_depth, double* out_rgb, double* out_depth2, const orc_materials* mat) {
  const double tanh_ = tan(0.5 * fovy_deg * ORC_PI / 180.0), aspect = (double)W / (double)H;
  for (int k = 0; k < nray; k++) {
    const double dc[3] = {(2.0 * pix[2 * k] / W - 1.0) * tanh_ * aspect, (1.0 - 2.0 * pix[2 * k + 1] / H) * tanh_, -1.0};
    double dw[3];
    for (int i = 0; i < 3; i++) dw[i] = cam_R[3 * i] * dc[0] + cam_R[3 * i + 1] * dc[1] + cam_R[3 * i + 2] * dc[2];
    orc_best b = {1e300, {0, 0, 1}, {0, 0, 0}, -1, 1e300, NULL, {0, 0, 0}};
    for (int q = 0; q < nprim; q++) {
      const orc_prim* P = prims + q;
      const double* c = P->pos;
      const double* R = P->R;
      const double rel[3] = {cam_p[0] - c[0], cam_p[1] - c[1], cam_p[2] - c[2]};
      double o[3], d[3];
      for (int i = 0; i < 3; i++) {
        o[i] = R[i] * rel[0] + R[3 + i] * rel[1] + R[6 + i] * rel[2];
        d[i] = R[i] * dw[0] + R[3 + i] * dw[1] + R[6 + i] * dw[2];
      }
      double t = 0, nl[3] = {0, 0, 1}, nw[3];
      int h = 0;
      switch (P->type) {
        case 0:
          if (fabs(d[2]) > 1e-24) {
            t = -o[2] / d[2];
            h = t > 1e-4;
          }
          break;
        case 2: h = hit_sphere(o, d, P->size[0], &t, nl); break;
        case 3: h = hit_capsule(o, d, P->size[0], P->size[1], &t, nl); break;
        case 5: h = hit_cylinder(o, d, P->size[0], P->size[1], 1, &t, nl); break;
        case 6: h = hit_box(o, d, P->size, &t, nl); break;
        case 7: {
          /* the body's bounding sphere about its origin (radius computed by the caller from the
             triangles): a ray that misses it misses every triangle */
          const double od = dot3(o, d), dd = dot3(d, d);
          const double far2 = dot3(o, o) - od * od / dd;
          if (far2 > P->size[0] * P->size[0] * (1.0 + 1e-9) && dot3(o, o) > P->size[0] * P->size[0]) break;
          for (int j = P->tri0; j < P->tri0 + P->ntri; j++) {
            double tt;
            const float* tr = tri + 16 * (size_t)j;
            if (hit_tri(o, d, tr, znear, &tt)) {
              int32_t tag;
              memcpy(&tag, tr + 12, sizeof(tag));
              const int gid = tag & 0xffff; /* tag = (mesh slot << 16) | geom id */
              const double nt[3] = {tr[9], tr[10], tr[11]}, rgb[3] = {tr[13], tr[14], tr[15]};
              for (int i = 0; i < 3; i++) nw[i] = R[3 * i] * nt[0] + R[3 * i + 1] * nt[1] + R[3 * i + 2] * nt[2];
              consider(&b, tt, gid, nw, rgb, NULL, NULL);
            }
          }
          break;
        }
        default: break;
      }
      if (h) {
        for (int i = 0; i < 3; i++) nw[i] = R[3 * i] * nl[0] + R[3 * i + 1] * nl[1] + R[3 * i + 2] * nl[2];
        const double pl[3] = {o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]};
        consider(&b, t, P->geom, nw, P->rgb, P, pl);
      }
    }
    out_geom[k] = b.geom;
    out_depth2[k] = b.t2;
    const double inv = 1.0 / sqrt(dot3(dw, dw));
    if (b.geom < 0) {
      out_depth[k] = -1;
      if (mat) { /* gradient skybox by the ray's world z */
        const double f = 0.5 * (1.0 + dw[2] * inv);
        for (int i = 0; i < 3; i++) out_rgb[3 * k + i] = mat->sky[3 + i] + f * (mat->sky[i] - mat->sky[3 + i]);
      } else {
        out_rgb[3 * k] = 0.9;
        out_rgb[3 * k + 1] = 1.0;
        out_rgb[3 * k + 2] = 1.0;
      }
      continue;
    }
    out_depth[k] = b.t;
    const double nn = sqrt(dot3(b.n, b.n));
    double nw_[3] = {b.n[0] / nn, b.n[1] / nn, b.n[2] / nn};
    double ndv = -(nw_[0] * dw[0] + nw_[1] * dw[1] + nw_[2] * dw[2]) * inv;
    if (ndv < 0) { /* the normal turned to the viewer */
      ndv = -ndv;
      for (int i = 0; i < 3; i++) nw_[i] = -nw_[i];
    }
    const double ndl = nw_[2] > 0 ? nw_[2] : 0; /* light towards world +z */
    const double shade = 0.1 + 0.6 * ndv + 0.3 * ndl;
    if (!mat) {
      for (int i = 0; i < 3; i++) {
        const double x = b.rgb[i] * shade;
        out_rgb[3 * k + i] = x < 1.0 ? x : 1.0;
      }
      continue;
    }
    const float* mi = mat->geom_matinfo + 6 * b.geom;
    double tc[3] = {1, 1, 1};
    if (b.prim && mat->geom_texid[b.geom] >= 0) {
      /* the pixel's footprint on the surface: one pixel's step of the ray slope (2 tan(fovy/2) / H)
         at camera depth t, over the cosine to the normal */
      const double foot = b.t * (2.0 * tanh_ / H) / (ndv > 1e-3 ? ndv : 1e-3);
      orc_texture(mat, mat->geom_texid[b.geom], b.prim, mi, b.pl, foot, tc);
    }
    double sp = 0;
    if (ndl > 0 && mi[0] > 0) { /* Blinn-Phong: half vector of the light and the viewer */
      const double hv[3] = {-dw[0] * inv, -dw[1] * inv, 1.0 - dw[2] * inv};
      const double hn = sqrt(dot3(hv, hv));
      double nh = dot3(nw_, hv) / hn;
      nh = nh > 0 ? nh : 0;
      sp = mi[0] * 0.3 * pow(nh, 128.0 * mi[1]);
    }
    for (int i = 0; i < 3; i++) {
      const double x = b.rgb[i] * tc[i] * (shade + mi[5]) + sp;
      out_rgb[3 * k + i] = x < 1.0 ? x : 1.0;
    }
  }
}
