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
 * inside a primitive sees none of it; hits at t <= 1e-4 ignored; triangles two-sided and clipped at
 * t <= znear; nearest hit wins.  Shading 0.1 + 0.6 |n.v| + 0.3 max(0, n_z) (normal turned to the
 * viewer, light along world -z), times the material colour, clamped at 1; background (0.9, 1, 1).
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
} orc_best;

static void consider(orc_best* b, double t, int geom, const double* n, const double* rgb) {
  if (t < b->t || (t == b->t && geom < b->geom)) {
    if (geom != b->geom && b->t < b->t2) b->t2 = b->t;
    b->t = t;
    b->geom = geom;
    for (int i = 0; i < 3; i++) {
      b->n[i] = n[i];
      b->rgb[i] = rgb[i];
    }
  } else if (geom != b->geom && t < b->t2) {
    b->t2 = t;
  }
}

/* Cast `nray` camera rays: pix [nray][2] = continuous pixel coordinates (x, y), pixel centres at
 * +0.5; cam_R [9] row-major with columns = camera axes in world, cam_p [3]; the ray of (x, y) is
 * R (u tan(fovy/2) aspect, v tan(fovy/2), -1) with u = 2x/W - 1, v = 1 - 2y/H.  Outputs per ray:
 * the hit geom (-1: background), its camera depth t, the shaded colour (f64, before the 8-bit
 * rounding) and the depth of the nearest hit of any OTHER geom (out_depth2, 1e300 if none: a
 * coincident surface there makes the pixel's geom a tie). */
void orc_render_rays(const orc_prim* prims, int nprim, const float* tri, const double* cam_R, const double* cam_p,
                     double fovy_deg, int W, int H, double znear, const double* pix, int nray, int32_t* out_geom,
                     double* out_depth, double* out_rgb, double* out_depth2) {
  const double tanh_ = tan(0.5 * fovy_deg * ORC_PI / 180.0), aspect = (double)W / (double)H;
  for (int k = 0; k < nray; k++) {
    const double dc[3] = {(2.0 * pix[2 * k] / W - 1.0) * tanh_ * aspect, (1.0 - 2.0 * pix[2 * k + 1] / H) * tanh_, -1.0};
    double dw[3];
    for (int i = 0; i < 3; i++) dw[i] = cam_R[3 * i] * dc[0] + cam_R[3 * i + 1] * dc[1] + cam_R[3 * i + 2] * dc[2];
    orc_best b = {1e300, {0, 0, 1}, {0, 0, 0}, -1, 1e300};
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
              consider(&b, tt, gid, nw, rgb);
            }
          }
          break;
        }
        default: break;
      }
      if (h) {
        for (int i = 0; i < 3; i++) nw[i] = R[3 * i] * nl[0] + R[3 * i + 1] * nl[1] + R[3 * i + 2] * nl[2];
        consider(&b, t, P->geom, nw, P->rgb);
      }
    }
    out_geom[k] = b.geom;
    out_depth2[k] = b.t2;
    if (b.geom < 0) {
      out_depth[k] = -1;
      out_rgb[3 * k] = 0.9;
      out_rgb[3 * k + 1] = 1.0;
      out_rgb[3 * k + 2] = 1.0;
      continue;
    }
    out_depth[k] = b.t;
    const double inv = 1.0 / sqrt(dot3(dw, dw));
    const double nn = sqrt(dot3(b.n, b.n));
    double ndv = -(b.n[0] * dw[0] + b.n[1] * dw[1] + b.n[2] * dw[2]) * inv / nn;
    double nz = b.n[2] / nn;
    if (ndv < 0) {
      ndv = -ndv;
      nz = -nz;
    }
    const double ndl = nz > 0 ? nz : 0;
    const double shade = 0.1 + 0.6 * ndv + 0.3 * ndl;
    for (int i = 0; i < 3; i++) {
      const double x = b.rgb[i] * shade;
      out_rgb[3 * k + i] = x < 1.0 ? x : 1.0;
    }
  }
}
