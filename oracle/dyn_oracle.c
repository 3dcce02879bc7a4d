/*
 * ORACLE — test infrastructure only.  Used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py; never linked into or called by the product path.
 *
 * Serial C restatement of one MuJoCo mj_step (mujoco==3.1.6, the reference's physics
 * dependency, pyproject.toml:34, called through gymnasium's do_simulation at
 * envs/mujoco/MujocoEnvBase.py:83 with frame_skip 8, MujocoEnvBase.py:12-13) for the subset of
 * MuJoCo features the MujocoUR5eCable scene uses, with `option integrator="implicitfast"`
 * (envs/assets/mujoco/envs/ur5e/env_ur5e_common.xml:3):
 *
 *   mj_kinematics -> mj_comPos (cinert, cdof) -> mj_crb (dense M + armature)
 *   -> mj_comVel (cvel, cdof_dot) -> mj_rne (qfrc_bias, gravity) -> mj_passive (damping,
 *   joint springs) -> fixed tendons + mj_fwdActuation (affine general actuators, ctrl/force
 *   clamps) -> collision (AABB broadphase over compiler-filtered pairs; sphere/capsule/box/
 *   plane narrowphase) -> constraints (connect/weld/joint equality, joint limits, pyramidal
 *   condim-3 contacts, solref/solimp soft-constraint impedance) -> primal Newton solver with
 *   exact line search -> force/torque site sensors (mj_rnePostConstraint) -> implicitfast
 *   velocity update (M + h*D) and position integration.
 *
 * Parity status vs real MuJoCo: UNPINNED (MuJoCo is not installed in this image and the
 * reference ships no physics fixtures).  This file is the CPU oracle the HIP
 * engine is checked against (single substep <= 1e-9, bounded-horizon trajectories <= 1e-4).
 * Compiled with -ffp-contract=off.  Spatial vectors are [angular; linear] about the world
 * origin.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rmbx_model.h"

#define MINVAL 1e-15
#define MAXCON_PAIR 8

typedef struct {
  const rmbx_model* m;
  int nefc_max;
  /* state */
  double time;
  double *qpos, *qvel, *qacc_ws, *ctrl;
  double* body_pos_env; /* per-env override of body_pos for static bodies [nbody*3] */
  /* kinematics */
  double *xpos, *xquat, *xmat, *xipos, *xanchor, *xaxis, *gxpos, *gxmat, *sxpos, *sxmat;
  double *cdof, *cinert, *crb, *cvel, *cdofdot, *cacc, *cfrc;
  double *M, *L, *H, *A;
  double *qfrc_bias, *qfrc_passive, *qfrc_actuator, *qfrc_smooth, *qacc_smooth,
      *qfrc_constraint, *qacc, *tmpv, *tmpv2, *tmpv3, *grad, *search, *Ms, *res;
  double *ten_len, *ten_vel, *act_force;
  /* contacts */
  int ncon;
  double *con_pos, *con_frame, *con_dist, *con_mu;
  int *con_b1, *con_b2, *con_condim, *con_pair, *con_efcadr;
  /* constraints */
  int nefc, ne; /* ne: equality rows come first */
  double *J, *efc_pos, *efc_aref, *efc_D, *efc_R, *efc_force, *efc_jar, *efc_Js, *efc_vel, *efc_tmp;
  int* efc_type; /* 0 equality, 1 inequality */
  double sensordata[6];
  int solver_iter;
  double trace_grad[128], trace_impr[128], trace_kink[128];  /* per Newton iteration: scaled |grad| and improvement (-1: not reached) */
  int bad;     /* substep of the last divergence reset (orc_step) */
  int substep; /* 1-based substep being integrated */
} Data;

/* ------------------------------------------------------------------------------------------
 * small math
 * ---------------------------------------------------------------------------------------- */
static void quat2mat(const double* q, double* R) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z);
  R[1] = 2 * (x * y - w * z);
  R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z);
  R[4] = 1 - 2 * (x * x + z * z);
  R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y);
  R[7] = 2 * (y * z + w * x);
  R[8] = 1 - 2 * (x * x + y * y);
}
static void quatmul(const double* a, const double* b, double* r) {
  double t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, sizeof(t));
}
static void quatnorm(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) {
    q[0] = 1;
    q[1] = q[2] = q[3] = 0;
    return;
  }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
static void axisangle_quat(const double* ax, double ang, double* q) {
  double s = sin(0.5 * ang);
  q[0] = cos(0.5 * ang);
  q[1] = ax[0] * s;
  q[2] = ax[1] * s;
  q[3] = ax[2] * s;
}
static void matvec3(const double* R, const double* v, double* r) {
  double t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  double t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  double t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
static void mattvec3(const double* R, const double* v, double* r) {
  double t0 = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
  double t1 = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
  double t2 = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
static void matmul3(const double* A, const double* B, double* C) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(C, t, sizeof(t));
}
static void cross3(const double* a, const double* b, double* r) {
  double t0 = a[1] * b[2] - a[2] * b[1];
  double t1 = a[2] * b[0] - a[0] * b[2];
  double t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double norm3(const double* a) { return sqrt(dot3(a, a)); }

/* spatial inertia about origin, 10 numbers: m, h(3) = m*c, I(6) = xx yy zz xy xz yz */
static void inert_mul(const double* I, const double* v, double* r) {
  const double m = I[0], *h = I + 1;
  const double* w = v;
  const double* u = v + 3;
  double n[3], f[3], hxu[3], hxw[3];
  n[0] = I[4] * w[0] + I[7] * w[1] + I[8] * w[2];
  n[1] = I[7] * w[0] + I[5] * w[1] + I[9] * w[2];
  n[2] = I[8] * w[0] + I[9] * w[1] + I[6] * w[2];
  cross3(h, u, hxu);
  cross3(h, w, hxw);
  for (int i = 0; i < 3; i++) {
    r[i] = n[i] + hxu[i];
    f[i] = m * u[i] - hxw[i];
  }
  r[3] = f[0];
  r[4] = f[1];
  r[5] = f[2];
}
/* motion cross: V x U */
static void cross_motion(const double* V, const double* U, double* r) {
  double a[3], b[3], c[3];
  cross3(V, U, a);
  cross3(V, U + 3, b);
  cross3(V + 3, U, c);
  r[0] = a[0];
  r[1] = a[1];
  r[2] = a[2];
  r[3] = b[0] + c[0];
  r[4] = b[1] + c[1];
  r[5] = b[2] + c[2];
}
/* force cross: V x* F */
static void cross_force(const double* V, const double* F, double* r) {
  double a[3], b[3], c[3];
  cross3(V, F, a);
  cross3(V + 3, F + 3, b);
  cross3(V, F + 3, c);
  r[0] = a[0] + b[0];
  r[1] = a[1] + b[1];
  r[2] = a[2] + b[2];
  r[3] = c[0];
  r[4] = c[1];
  r[5] = c[2];
}
static double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* dense Cholesky (lower), returns 0 on success */
static int cholesky(double* A, int n) {
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    if (!(s > MINVAL)) s = MINVAL;
    double d = sqrt(s);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / d;
    }
  }
  return 0;
}
static void chol_solve(const double* L, int n, const double* b, double* x) {
  for (int i = 0; i < n; i++) {
    double t = b[i];
    for (int k = 0; k < i; k++) t -= L[i * n + k] * x[k];
    x[i] = t / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double t = x[i];
    for (int k = i + 1; k < n; k++) t -= L[k * n + i] * x[k];
    x[i] = t / L[i * n + i];
  }
}

/* ------------------------------------------------------------------------------------------
 * allocation
 * ---------------------------------------------------------------------------------------- */
static double* dalloc(size_t n) { return (double*)calloc(n ? n : 1, sizeof(double)); }
static int* ialloc(size_t n) { return (int*)calloc(n ? n : 1, sizeof(int)); }

void* orc_create(const rmbx_model* m) {
  Data* d = (Data*)calloc(1, sizeof(Data));
  int nq = m->nq, nv = m->nv, nb = m->nbody, nj = m->njnt, ng = m->ngeom, mc = m->max_contacts;
  d->m = m;
  d->nefc_max = 4 * mc + 6 * m->neq + 2 * nj + 8;
  d->qpos = dalloc(nq);
  d->qvel = dalloc(nv);
  d->qacc_ws = dalloc(nv);
  d->ctrl = dalloc(m->nu);
  d->body_pos_env = dalloc(3 * nb);
  memcpy(d->body_pos_env, m->body_pos, sizeof(double) * 3 * nb);
  memcpy(d->qpos, m->qpos0, sizeof(double) * nq);
  d->xpos = dalloc(3 * nb);
  d->xquat = dalloc(4 * nb);
  d->xmat = dalloc(9 * nb);
  d->xipos = dalloc(3 * nb);
  d->xanchor = dalloc(3 * nj);
  d->xaxis = dalloc(3 * nj);
  d->gxpos = dalloc(3 * ng);
  d->gxmat = dalloc(9 * ng);
  d->sxpos = dalloc(3 * m->nsite);
  d->sxmat = dalloc(9 * m->nsite);
  d->cdof = dalloc(6 * nv);
  d->cdofdot = dalloc(6 * nv);
  d->cinert = dalloc(10 * nb);
  d->crb = dalloc(10 * nb);
  d->cvel = dalloc(6 * nb);
  d->cacc = dalloc(6 * nb);
  d->cfrc = dalloc(6 * nb);
  d->M = dalloc((size_t)nv * nv);
  d->L = dalloc((size_t)nv * nv);
  d->H = dalloc((size_t)nv * nv);
  d->A = dalloc((size_t)nv * nv);
  double** vs[] = {&d->qfrc_bias, &d->qfrc_passive, &d->qfrc_actuator, &d->qfrc_smooth,
                   &d->qacc_smooth, &d->qfrc_constraint, &d->qacc, &d->tmpv, &d->tmpv2,
                   &d->tmpv3, &d->grad, &d->search, &d->Ms, &d->res};
  for (unsigned i = 0; i < sizeof(vs) / sizeof(vs[0]); i++) *vs[i] = dalloc(nv);
  d->ten_len = dalloc(m->ntendon);
  d->ten_vel = dalloc(m->ntendon);
  d->act_force = dalloc(m->nu);
  d->con_pos = dalloc(3 * mc);
  d->con_frame = dalloc(9 * mc);
  d->con_dist = dalloc(mc);
  d->con_mu = dalloc(mc);
  d->con_b1 = ialloc(mc);
  d->con_b2 = ialloc(mc);
  d->con_condim = ialloc(mc);
  d->con_pair = ialloc(mc);
  d->con_efcadr = ialloc(mc);
  int ne = d->nefc_max;
  d->J = dalloc((size_t)ne * nv);
  d->efc_pos = dalloc(ne);
  d->efc_aref = dalloc(ne);
  d->efc_D = dalloc(ne);
  d->efc_R = dalloc(ne);
  d->efc_force = dalloc(ne);
  d->efc_jar = dalloc(ne);
  d->efc_Js = dalloc(ne);
  d->efc_vel = dalloc(ne);
  d->efc_tmp = dalloc(ne);
  d->efc_type = ialloc(ne);
  return d;
}

void orc_destroy(void* p) {
  Data* d = (Data*)p;
  if (!d) return;
  /* leak-free teardown of every array allocated above */
  void* ptrs[] = {d->qpos, d->qvel, d->qacc_ws, d->ctrl, d->body_pos_env, d->xpos, d->xquat, d->xmat,
                  d->xipos, d->xanchor, d->xaxis, d->gxpos, d->gxmat, d->sxpos, d->sxmat, d->cdof,
                  d->cdofdot, d->cinert, d->crb, d->cvel, d->cacc, d->cfrc, d->M, d->L, d->H, d->A,
                  d->qfrc_bias, d->qfrc_passive, d->qfrc_actuator, d->qfrc_smooth, d->qacc_smooth,
                  d->qfrc_constraint, d->qacc, d->tmpv, d->tmpv2, d->tmpv3, d->grad, d->search, d->Ms, d->res,
                  d->ten_len, d->ten_vel, d->act_force, d->con_pos, d->con_frame, d->con_dist,
                  d->con_mu, d->con_b1, d->con_b2, d->con_condim, d->con_pair, d->con_efcadr, d->J,
                  d->efc_pos, d->efc_aref, d->efc_D, d->efc_R, d->efc_force, d->efc_jar, d->efc_Js,
                  d->efc_vel, d->efc_tmp, d->efc_type};
  for (unsigned i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); i++) free(ptrs[i]);
  free(d);
}

/* ------------------------------------------------------------------------------------------
 * mj_kinematics
 * ---------------------------------------------------------------------------------------- */
static void kinematics(Data* d) {
  const rmbx_model* m = d->m;
  d->xpos[0] = d->xpos[1] = d->xpos[2] = 0;
  d->xquat[0] = 1;
  d->xquat[1] = d->xquat[2] = d->xquat[3] = 0;
  quat2mat(d->xquat, d->xmat);
  for (int b = 1; b < m->nbody; b++) {
    int p = m->body_parent[b];
    int ja = m->body_jntadr[b], jn = m->body_jntnum[b];
    double* xp = d->xpos + 3 * b;
    double* xq = d->xquat + 4 * b;
    if (jn > 0 && m->jnt_type[ja] == RMBX_JNT_FREE) {
      int a = m->jnt_qposadr[ja];
      xp[0] = d->qpos[a];
      xp[1] = d->qpos[a + 1];
      xp[2] = d->qpos[a + 2];
      memcpy(xq, d->qpos + a + 3, 4 * sizeof(double));
      quatnorm(xq);
      memcpy(d->xanchor + 3 * ja, xp, 3 * sizeof(double));
      d->xaxis[3 * ja] = 0;
      d->xaxis[3 * ja + 1] = 0;
      d->xaxis[3 * ja + 2] = 1;
    } else {
      double t[3];
      matvec3(d->xmat + 9 * p, d->body_pos_env + 3 * b, t);
      for (int i = 0; i < 3; i++) xp[i] = d->xpos[3 * p + i] + t[i];
      quatmul(d->xquat + 4 * p, m->body_quat + 4 * b, xq);
      for (int j = ja; j < ja + jn; j++) {
        double R[9], anc[3], ax[3];
        quat2mat(xq, R);
        matvec3(R, m->jnt_pos + 3 * j, t);
        for (int i = 0; i < 3; i++) anc[i] = xp[i] + t[i];
        matvec3(R, m->jnt_axis + 3 * j, ax);
        memcpy(d->xanchor + 3 * j, anc, sizeof(anc));
        memcpy(d->xaxis + 3 * j, ax, sizeof(ax));
        int qa = m->jnt_qposadr[j];
        double qd = d->qpos[qa] - m->qpos0[qa];
        if (m->jnt_type[j] == RMBX_JNT_HINGE) {
          double qr[4];
          axisangle_quat(m->jnt_axis + 3 * j, qd, qr);
          quatmul(xq, qr, xq);
          quatnorm(xq);
          quat2mat(xq, R);
          matvec3(R, m->jnt_pos + 3 * j, t);
          for (int i = 0; i < 3; i++) xp[i] = anc[i] - t[i];
        } else if (m->jnt_type[j] == RMBX_JNT_SLIDE) {
          for (int i = 0; i < 3; i++) xp[i] += ax[i] * qd;
        }
      }
    }
    quat2mat(xq, d->xmat + 9 * b);
    double t[3];
    matvec3(d->xmat + 9 * b, m->body_ipos + 3 * b, t);
    for (int i = 0; i < 3; i++) d->xipos[3 * b + i] = xp[i] + t[i];
  }
  for (int g = 0; g < m->ngeom; g++) {
    if (m->geom_ctype[g] < 0) continue;
    int b = m->geom_body[g];
    double t[3], R[9];
    matvec3(d->xmat + 9 * b, m->geom_cpos + 3 * g, t);
    for (int i = 0; i < 3; i++) d->gxpos[3 * g + i] = d->xpos[3 * b + i] + t[i];
    quat2mat(m->geom_cquat + 4 * g, R);
    matmul3(d->xmat + 9 * b, R, d->gxmat + 9 * g);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_body[s];
    double t[3], R[9];
    matvec3(d->xmat + 9 * b, m->site_pos + 3 * s, t);
    for (int i = 0; i < 3; i++) d->sxpos[3 * s + i] = d->xpos[3 * b + i] + t[i];
    quat2mat(m->site_quat + 4 * s, R);
    matmul3(d->xmat + 9 * b, R, d->sxmat + 9 * s);
  }
}

/* ------------------------------------------------------------------------------------------
 * mj_comPos (cinert about origin, cdof) + mj_crb (dense M)
 * ---------------------------------------------------------------------------------------- */
static void com_pos(Data* d) {
  const rmbx_model* m = d->m;
  memset(d->cinert, 0, sizeof(double) * 10 * m->nbody);
  for (int b = 1; b < m->nbody; b++) {
    double mass = m->body_mass[b];
    double* I = d->cinert + 10 * b;
    const double* c = d->xipos + 3 * b;
    const double* R = d->xmat + 9 * b;
    const double* Ib = m->body_inertia + 9 * b;
    double T[9], Iw[9], Rt[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) Rt[3 * i + j] = R[3 * j + i];
    matmul3(R, Ib, T);
    matmul3(T, Rt, Iw);
    double cc = dot3(c, c);
    I[0] = mass;
    I[1] = mass * c[0];
    I[2] = mass * c[1];
    I[3] = mass * c[2];
    I[4] = Iw[0] + mass * (cc - c[0] * c[0]);
    I[5] = Iw[4] + mass * (cc - c[1] * c[1]);
    I[6] = Iw[8] + mass * (cc - c[2] * c[2]);
    I[7] = Iw[1] - mass * c[0] * c[1];
    I[8] = Iw[2] - mass * c[0] * c[2];
    I[9] = Iw[5] - mass * c[1] * c[2];
  }
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_body[j], da = m->jnt_dofadr[j];
    const double* ax = d->xaxis + 3 * j;
    const double* anc = d->xanchor + 3 * j;
    double* S = d->cdof + 6 * da;
    switch (m->jnt_type[j]) {
      case RMBX_JNT_HINGE: {
        S[0] = ax[0];
        S[1] = ax[1];
        S[2] = ax[2];
        cross3(anc, ax, S + 3);
        break;
      }
      case RMBX_JNT_SLIDE:
        S[0] = S[1] = S[2] = 0;
        S[3] = ax[0];
        S[4] = ax[1];
        S[5] = ax[2];
        break;
      case RMBX_JNT_FREE: {
        memset(S, 0, sizeof(double) * 36);
        S[3] = 1;
        S[6 + 4] = 1;
        S[12 + 5] = 1;
        const double* R = d->xmat + 9 * b;
        const double* x = d->xpos + 3 * b;
        for (int k = 0; k < 3; k++) {
          double* Sk = S + 6 * (3 + k);
          double a[3] = {R[k], R[3 + k], R[6 + k]};
          Sk[0] = a[0];
          Sk[1] = a[1];
          Sk[2] = a[2];
          cross3(x, a, Sk + 3);
        }
        break;
      }
      default:
        break;
    }
  }
}

static void crb(Data* d) {
  const rmbx_model* m = d->m;
  int nv = m->nv;
  memcpy(d->crb, d->cinert, sizeof(double) * 10 * m->nbody);
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parent[b];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[10 * p + k] += d->crb[10 * b + k];
  }
  memset(d->M, 0, sizeof(double) * nv * nv);
  for (int i = 0; i < nv; i++) {
    double F[6];
    inert_mul(d->crb + 10 * m->dof_body[i], d->cdof + 6 * i, F);
    for (int j = i; j >= 0; j = m->dof_parent[j]) {
      double v = dot6(d->cdof + 6 * j, F);
      d->M[i * nv + j] = v;
      d->M[j * nv + i] = v;
    }
    d->M[i * nv + i] += m->dof_armature[i];
  }
}

/* ------------------------------------------------------------------------------------------
 * mj_comVel + mj_rne (bias) ; passive ; tendon ; actuation
 * ---------------------------------------------------------------------------------------- */
static void com_vel(Data* d) {
  const rmbx_model* m = d->m;
  memset(d->cvel, 0, 6 * sizeof(double));
  for (int b = 1; b < m->nbody; b++) {
    double* cv = d->cvel + 6 * b;
    memcpy(cv, d->cvel + 6 * m->body_parent[b], 6 * sizeof(double));
    for (int j = m->body_jntadr[b]; j < m->body_jntadr[b] + m->body_jntnum[b]; j++) {
      int da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == RMBX_JNT_FREE) {
        for (int k = 0; k < 3; k++) memset(d->cdofdot + 6 * (da + k), 0, 6 * sizeof(double));
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) cv[i] += d->cdof[6 * (da + k) + i] * d->qvel[da + k];
        for (int k = 3; k < 6; k++) cross_motion(cv, d->cdof + 6 * (da + k), d->cdofdot + 6 * (da + k));
        for (int k = 3; k < 6; k++)
          for (int i = 0; i < 6; i++) cv[i] += d->cdof[6 * (da + k) + i] * d->qvel[da + k];
      } else {
        cross_motion(cv, d->cdof + 6 * da, d->cdofdot + 6 * da);
        for (int i = 0; i < 6; i++) cv[i] += d->cdof[6 * da + i] * d->qvel[da];
      }
    }
  }
}

/* RNE with given qacc (NULL = zero) into cacc/cfrc; returns per-dof projection in out */
static void rne(Data* d, const double* qacc, double* out) {
  const rmbx_model* m = d->m;
  double* ca = d->cacc;
  ca[0] = ca[1] = ca[2] = 0;
  ca[3] = -m->gravity[0];
  ca[4] = -m->gravity[1];
  ca[5] = -m->gravity[2];
  for (int b = 1; b < m->nbody; b++) {
    double* a = ca + 6 * b;
    memcpy(a, ca + 6 * m->body_parent[b], 6 * sizeof(double));
    int da = m->body_dofadr[b], dn = m->body_dofnum[b];
    for (int k = da; k < da + dn; k++) {
      for (int i = 0; i < 6; i++) a[i] += d->cdofdot[6 * k + i] * d->qvel[k];
      if (qacc)
        for (int i = 0; i < 6; i++) a[i] += d->cdof[6 * k + i] * qacc[k];
    }
    double Ia[6], Iv[6], vxIv[6];
    inert_mul(d->cinert + 10 * b, a, Ia);
    inert_mul(d->cinert + 10 * b, d->cvel + 6 * b, Iv);
    cross_force(d->cvel + 6 * b, Iv, vxIv);
    for (int i = 0; i < 6; i++) d->cfrc[6 * b + i] = Ia[i] + vxIv[i];
  }
}
static void rne_backward(Data* d, double* out) {
  const rmbx_model* m = d->m;
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parent[b];
    if (p > 0)
      for (int i = 0; i < 6; i++) d->cfrc[6 * p + i] += d->cfrc[6 * b + i];
  }
  if (out)
    for (int k = 0; k < m->nv; k++) out[k] = dot6(d->cdof + 6 * k, d->cfrc + 6 * m->dof_body[k]);
}

static void passive_actuation(Data* d) {
  const rmbx_model* m = d->m;
  int nv = m->nv;
  for (int k = 0; k < nv; k++) d->qfrc_passive[k] = -m->dof_damping[k] * d->qvel[k];
  for (int j = 0; j < m->njnt; j++) {
    if (m->jnt_stiffness[j] == 0) continue;
    if (m->jnt_type[j] == RMBX_JNT_HINGE || m->jnt_type[j] == RMBX_JNT_SLIDE) {
      int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
      d->qfrc_passive[da] -= m->jnt_stiffness[j] * (d->qpos[qa] - m->jnt_springref[j]);
    }
  }
  for (int t = 0; t < m->ntendon; t++) {
    double L = 0, V = 0;
    for (int w = m->ten_adr[t]; w < m->ten_adr[t] + m->ten_num[t]; w++) {
      int j = m->wrap_jnt[w];
      L += m->wrap_coef[w] * d->qpos[m->jnt_qposadr[j]];
      V += m->wrap_coef[w] * d->qvel[m->jnt_dofadr[j]];
    }
    d->ten_len[t] = L;
    d->ten_vel[t] = V;
  }
  memset(d->qfrc_actuator, 0, sizeof(double) * nv);
  for (int u = 0; u < m->nu; u++) {
    double c = d->ctrl[u];
    if (m->act_ctrllimited[u]) {
      if (c < m->act_ctrlrange[2 * u]) c = m->act_ctrlrange[2 * u];
      if (c > m->act_ctrlrange[2 * u + 1]) c = m->act_ctrlrange[2 * u + 1];
    }
    double len, vel;
    int id = m->act_trnid[u];
    if (m->act_trntype[u] == RMBX_TRN_JOINT) {
      len = d->qpos[m->jnt_qposadr[id]];
      vel = d->qvel[m->jnt_dofadr[id]];
    } else {
      len = d->ten_len[id];
      vel = d->ten_vel[id];
    }
    const double* bp = m->act_bias + 3 * u;
    double f = m->act_gain[u] * c + bp[0] + bp[1] * len + bp[2] * vel;
    if (m->act_forcelimited[u]) {
      if (f < m->act_forcerange[2 * u]) f = m->act_forcerange[2 * u];
      if (f > m->act_forcerange[2 * u + 1]) f = m->act_forcerange[2 * u + 1];
    }
    d->act_force[u] = f;
    if (m->act_trntype[u] == RMBX_TRN_JOINT) {
      d->qfrc_actuator[m->jnt_dofadr[id]] += f;
    } else {
      for (int w = m->ten_adr[id]; w < m->ten_adr[id] + m->ten_num[id]; w++)
        d->qfrc_actuator[m->jnt_dofadr[m->wrap_jnt[w]]] += m->wrap_coef[w] * f;
    }
  }
}

/* ------------------------------------------------------------------------------------------
 * collision
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  double pos[3], n[3], dist;
} Contact;

static void closest_seg_seg(const double* p1, const double* q1, const double* p2, const double* q2,
                            double* c1, double* c2) {
  double d1[3], d2[3], r[3];
  for (int i = 0; i < 3; i++) {
    d1[i] = q1[i] - p1[i];
    d2[i] = q2[i] - p2[i];
    r[i] = p1[i] - p2[i];
  }
  double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  double s, t;
  if (a <= MINVAL && e <= MINVAL) {
    s = t = 0;
  } else if (a <= MINVAL) {
    s = 0;
    t = f / e;
    t = t < 0 ? 0 : (t > 1 ? 1 : t);
  } else {
    double c = dot3(d1, r);
    if (e <= MINVAL) {
      t = 0;
      s = -c / a;
      s = s < 0 ? 0 : (s > 1 ? 1 : s);
    } else {
      double b = dot3(d1, d2);
      double den = a * e - b * b;
      if (den > MINVAL) {
        s = (b * f - c * e) / den;
        s = s < 0 ? 0 : (s > 1 ? 1 : s);
      } else {
        s = 0;
      }
      t = (b * s + f) / e;
      if (t < 0) {
        t = 0;
        s = -c / a;
        s = s < 0 ? 0 : (s > 1 ? 1 : s);
      } else if (t > 1) {
        t = 1;
        s = (b - c) / a;
        s = s < 0 ? 0 : (s > 1 ? 1 : s);
      }
    }
  }
  for (int i = 0; i < 3; i++) {
    c1[i] = p1[i] + d1[i] * s;
    c2[i] = p2[i] + d2[i] * t;
  }
}

/* sphere (center c, radius r) vs sphere -> normal from A to B */
static int col_sphere_sphere(const double* ca, double ra, const double* cb, double rb, double margin,
                             Contact* out) {
  double v[3] = {cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2]};
  double l = norm3(v);
  double dist = l - ra - rb;
  if (dist >= margin) return 0;
  double n[3];
  if (l < MINVAL) {
    n[0] = 1;
    n[1] = 0;
    n[2] = 0;
  } else {
    n[0] = v[0] / l;
    n[1] = v[1] / l;
    n[2] = v[2] / l;
  }
  for (int i = 0; i < 3; i++) {
    out->n[i] = n[i];
    out->pos[i] = ca[i] + n[i] * (ra + 0.5 * dist);
  }
  out->dist = dist;
  return 1;
}

static void capsule_ends(const double* c, const double* R, double h, double* p, double* q) {
  for (int i = 0; i < 3; i++) {
    p[i] = c[i] - R[3 * i + 2] * h;
    q[i] = c[i] + R[3 * i + 2] * h;
  }
}

static int col_capsule_capsule(const double* ca, const double* Ra, const double* sa, const double* cb,
                               const double* Rb, const double* sb, double margin, Contact* out) {
  double p1[3], q1[3], p2[3], q2[3], c1[3], c2[3];
  capsule_ends(ca, Ra, sa[1], p1, q1);
  capsule_ends(cb, Rb, sb[1], p2, q2);
  closest_seg_seg(p1, q1, p2, q2, c1, c2);
  return col_sphere_sphere(c1, sa[0], c2, sb[0], margin, out);
}

/* point (world) vs box: distance and normal from box to point; inside -> negative */
static double point_box(const double* p, const double* cb, const double* Rb, const double* hb, double* n,
                        double* surf) {
  double dlt[3] = {p[0] - cb[0], p[1] - cb[1], p[2] - cb[2]}, l[3];
  mattvec3(Rb, dlt, l);
  int inside = 1;
  double q[3];
  for (int i = 0; i < 3; i++) {
    q[i] = l[i] < -hb[i] ? -hb[i] : (l[i] > hb[i] ? hb[i] : l[i]);
    if (q[i] != l[i]) inside = 0;
  }
  double nl[3], dist;
  if (!inside) {
    double v[3] = {l[0] - q[0], l[1] - q[1], l[2] - q[2]};
    dist = norm3(v);
    nl[0] = v[0] / dist;
    nl[1] = v[1] / dist;
    nl[2] = v[2] / dist;
  } else {
    int k = 0;
    double best = hb[0] - fabs(l[0]);
    for (int i = 1; i < 3; i++) {
      double pen = hb[i] - fabs(l[i]);
      if (pen < best) {
        best = pen;
        k = i;
      }
    }
    nl[0] = nl[1] = nl[2] = 0;
    nl[k] = l[k] >= 0 ? 1 : -1;
    q[k] = nl[k] * hb[k];
    dist = -best;
  }
  matvec3(Rb, nl, n);
  double qw[3];
  matvec3(Rb, q, qw);
  for (int i = 0; i < 3; i++) surf[i] = cb[i] + qw[i];
  return dist;
}

/* sphere vs box, normal from sphere (A) to box (B) */
static int col_sphere_box(const double* cs, double r, const double* cb, const double* Rb, const double* hb,
                          double margin, Contact* out) {
  double n[3], surf[3];
  double dist = point_box(cs, cb, Rb, hb, n, surf) - r;
  if (dist >= margin) return 0;
  for (int i = 0; i < 3; i++) {
    out->n[i] = -n[i];
    out->pos[i] = surf[i] + n[i] * (0.5 * dist);
  }
  out->dist = dist;
  return 1;
}

/* capsule (A) vs box (B): endpoint spheres plus the segment point closest to the box */
static int col_capsule_box(const double* ca, const double* Ra, const double* sa, const double* cb,
                           const double* Rb, const double* hb, double margin, Contact* out) {
  double p[3], q[3];
  capsule_ends(ca, Ra, sa[1], p, q);
  Contact c0, c1, cm;
  int h0 = col_sphere_box(p, sa[0], cb, Rb, hb, margin, &c0);
  int h1 = col_sphere_box(q, sa[0], cb, Rb, hb, margin, &c1);
  /* closest segment point: ternary search of the convex point-box distance */
  double lo = 0, hi = 1;
  for (int it = 0; it < 40; it++) {
    double t1 = lo + (hi - lo) / 3, t2 = hi - (hi - lo) / 3, x1[3], x2[3], nn[3], ss[3];
    for (int i = 0; i < 3; i++) {
      x1[i] = p[i] + (q[i] - p[i]) * t1;
      x2[i] = p[i] + (q[i] - p[i]) * t2;
    }
    double f1 = point_box(x1, cb, Rb, hb, nn, ss), f2 = point_box(x2, cb, Rb, hb, nn, ss);
    if (f1 < f2)
      hi = t2;
    else
      lo = t1;
  }
  double tm = 0.5 * (lo + hi), xm[3];
  for (int i = 0; i < 3; i++) xm[i] = p[i] + (q[i] - p[i]) * tm;
  int hm = col_sphere_box(xm, sa[0], cb, Rb, hb, margin, &cm);
  if (h0 && h1) {
    out[0] = c0;
    out[1] = c1;
    return 2;
  }
  /* single contact: deepest of the candidates */
  int n = 0;
  Contact best;
  if (h0) {
    best = c0;
    n = 1;
  }
  if (h1 && (!n || c1.dist < best.dist)) {
    best = c1;
    n = 1;
  }
  if (hm && (!n || cm.dist < best.dist)) {
    best = cm;
    n = 1;
  }
  if (n) out[0] = best;
  return n;
}

/* box (A) vs box (B): SAT axis of least penetration + vertex-in-box manifold (<= 4) */
/* candidate order of the multi-point contact routines: depth quantised to 1 nm (ties keep
 * generation order, so face-face configurations do not flip under last-bit geometry changes) */
static int contact_deeper(const Contact* a, const Contact* b) {
  return floor(a->dist * 1e9) < floor(b->dist * 1e9);
}

#define BOX_INSIDE_TOL 1e-9 /* m */

static int col_box_box(const double* ca, const double* Ra, const double* ha, const double* cb,
                       const double* Rb, const double* hb, double margin, Contact* out) {
  double axes[15][3];
  int na = 0;
  for (int k = 0; k < 3; k++) {
    axes[na][0] = Ra[k];
    axes[na][1] = Ra[3 + k];
    axes[na][2] = Ra[6 + k];
    na++;
  }
  for (int k = 0; k < 3; k++) {
    axes[na][0] = Rb[k];
    axes[na][1] = Rb[3 + k];
    axes[na][2] = Rb[6 + k];
    na++;
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double c[3];
      cross3(axes[i], axes[3 + j], c);
      double l = norm3(c);
      if (l < 1e-6) {
        axes[na][0] = axes[na][1] = axes[na][2] = 0;
      } else {
        axes[na][0] = c[0] / l;
        axes[na][1] = c[1] / l;
        axes[na][2] = c[2] / l;
      }
      na++;
    }
  double dc[3] = {cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2]};
  double best = -1e300;
  int bk = -1;
  for (int k = 0; k < 15; k++) {
    const double* a = axes[k];
    if (a[0] == 0 && a[1] == 0 && a[2] == 0) continue;
    double ra = 0, rb = 0;
    for (int i = 0; i < 3; i++) {
      double ua[3] = {Ra[i], Ra[3 + i], Ra[6 + i]}, ub[3] = {Rb[i], Rb[3 + i], Rb[6 + i]};
      ra += ha[i] * fabs(dot3(a, ua));
      rb += hb[i] * fabs(dot3(a, ub));
    }
    double sep = fabs(dot3(dc, a)) - ra - rb; /* > 0 separated */
    if (sep >= margin) return 0;
    /* prefer face axes on near-ties (edge axes need a 1e-6 margin to win) */
    /* B's face axes yield to A's within 1e-12 m (parallel faces tie up to rounding), edge axes
     * to faces within 1 um */
    double score = k < 3 ? sep : (k < 6 ? sep - 1e-12 : sep - 1e-6);
    if (score > best) {
      best = score;
      bk = k;
    }
  }
  if (bk < 0) return 0; /* non-finite geometry (a diverged env): no axis scored */
  double n[3] = {axes[bk][0], axes[bk][1], axes[bk][2]};
  if (dot3(n, dc) < 0) {
    n[0] = -n[0];
    n[1] = -n[1];
    n[2] = -n[2];
  }
  /* n points from A to B */
  Contact cand[16];
  int nc = 0;
  for (int side = 0; side < 2; side++) {
    const double* c = side == 0 ? cb : ca;
    const double* R = side == 0 ? Rb : Ra;
    const double* h = side == 0 ? hb : ha;
    const double* co = side == 0 ? ca : cb;
    const double* Ro = side == 0 ? Ra : Rb;
    const double* ho = side == 0 ? ha : hb;
    for (int v = 0; v < 8; v++) {
      double l[3] = {(v & 1) ? h[0] : -h[0], (v & 2) ? h[1] : -h[1], (v & 4) ? h[2] : -h[2]}, w[3];
      matvec3(R, l, w);
      double x[3] = {c[0] + w[0], c[1] + w[1], c[2] + w[2]};
      /* inside the other box (with margin)?  A vertex within BOX_INSIDE_TOL of a face plane
       * counts as inside, so aligned equal faces (the gripper pads closing on each other) give
       * the same manifold however the last bits of the poses fall */
      double dl[3] = {x[0] - co[0], x[1] - co[1], x[2] - co[2]}, lo[3];
      mattvec3(Ro, dl, lo);
      const double tol = margin + BOX_INSIDE_TOL;
      if (fabs(lo[0]) > ho[0] + tol || fabs(lo[1]) > ho[1] + tol || fabs(lo[2]) > ho[2] + tol)
        continue;
      /* penetration along n relative to the other box's support plane */
      double sup = 0;
      for (int i = 0; i < 3; i++) {
        double u[3] = {Ro[i], Ro[3 + i], Ro[6 + i]};
        sup += ho[i] * fabs(dot3(n, u));
      }
      double sgn = side == 0 ? 1.0 : -1.0; /* B vertices go against n into A */
      double proj = sgn * dot3(dl, n);      /* for B vertex: distance above A's far face */
      double dist = sgn * 0 + (side == 0 ? (dot3(dl, n) - sup) : (-dot3(dl, n) - sup));
      (void)proj;
      if (dist >= margin) continue;
      if (nc < 16) {
        Contact* k = cand + nc++;
        k->dist = dist;
        for (int i = 0; i < 3; i++) {
          k->n[i] = n[i];
          k->pos[i] = x[i] - sgn * n[i] * (0.5 * dist);
        }
      }
    }
  }
  if (nc == 0) {
    /* edge-edge: closest points between the two nearest edges along n */
    double pa[3], pb[3], sa_[3], sb_[3];
    double neg[3] = {-n[0], -n[1], -n[2]};
    /* support points */
    for (int i = 0; i < 3; i++) {
      pa[i] = ca[i];
      pb[i] = cb[i];
    }
    int fa = -1, fb = -1, nfa = 0, nfb = 0; /* the box axes parallel to the contact plane */
    for (int k = 0; k < 3; k++) {
      double ua[3] = {Ra[k], Ra[3 + k], Ra[6 + k]}, ub[3] = {Rb[k], Rb[3 + k], Rb[6 + k]};
      /* the extent's end facing the other box, or its centre when the axis is perpendicular to n
         within 1e-9 (a parallel face / edge: every point along it supports; a ~1e-17 dot product
         would otherwise pick an end by rounding) */
      const double da = dot3(ua, n), db = dot3(ub, neg);
      const int pa_free = fabs(da) < 1e-9, pb_free = fabs(db) < 1e-9;
      double sa2 = pa_free ? 0.0 : (da > 0 ? ha[k] : -ha[k]);
      double sb2 = pb_free ? 0.0 : (db > 0 ? hb[k] : -hb[k]);
      if (pa_free) { fa = k; ++nfa; }
      if (pb_free) { fb = k; ++nfb; }
      for (int i = 0; i < 3; i++) {
        pa[i] += ua[i] * sa2;
        pb[i] += ub[i] * sb2;
      }
    }
    (void)sa_;
    (void)sb_;
    double dist = dot3(n, pb) - dot3(n, pa);
    if (dist >= margin) return 0;
    if (nfa == 1 && nfb == 1) {
      /* edge against edge: closest points of the two support segments pa + s ua (|s| <= ha) and
         pb + t ub (|t| <= hb), clamped (crossed edges touch where they cross) */
      const double ua[3] = {Ra[fa], Ra[3 + fa], Ra[6 + fa]}, ub[3] = {Rb[fb], Rb[3 + fb], Rb[6 + fb]};
      const double w[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
      const double b = dot3(ua, ub), d = dot3(ua, w), e = dot3(ub, w);
      const double den = 1.0 - b * b;
      if (den > 1e-12) { /* (parallel edges keep the centres) */
        double sv = (b * e - d) / den;
        sv = sv < -ha[fa] ? -ha[fa] : (sv > ha[fa] ? ha[fa] : sv);
        double tv = e + sv * b;
        tv = tv < -hb[fb] ? -hb[fb] : (tv > hb[fb] ? hb[fb] : tv);
        sv = tv * b - d;
        sv = sv < -ha[fa] ? -ha[fa] : (sv > ha[fa] ? ha[fa] : sv);
        for (int i = 0; i < 3; i++) {
          pa[i] += ua[i] * sv;
          pb[i] += ub[i] * tv;
        }
      }
    }
    for (int i = 0; i < 3; i++) {
      out[0].n[i] = n[i];
      out[0].pos[i] = 0.5 * (pa[i] + pb[i]);
    }
    out[0].dist = dist;
    return 1;
  }
  /* keep the 4 deepest */
  for (int i = 0; i < nc; i++)
    for (int j = i + 1; j < nc; j++)
      if (contact_deeper(&cand[j], &cand[i])) {
        Contact t = cand[i];
        cand[i] = cand[j];
        cand[j] = t;
      }
  int k = nc < 4 ? nc : 4;
  for (int i = 0; i < k; i++) out[i] = cand[i];
  return k;
}

/* plane (A, normal = local z) vs primitive (B) */
static int col_plane(const double* cp, const double* Rp, int tb, const double* cb, const double* Rb,
                     const double* sb, double margin, Contact* out) {
  double n[3] = {Rp[2], Rp[5], Rp[8]};
  double pts[8][3], rad = 0;
  int np = 0;
  if (tb == RMBX_GEOM_SPHERE) {
    memcpy(pts[0], cb, sizeof(double) * 3);
    np = 1;
    rad = sb[0];
  } else if (tb == RMBX_GEOM_CAPSULE) {
    capsule_ends(cb, Rb, sb[1], pts[0], pts[1]);
    np = 2;
    rad = sb[0];
  } else if (tb == RMBX_GEOM_BOX) {
    for (int v = 0; v < 8; v++) {
      double l[3] = {(v & 1) ? sb[0] : -sb[0], (v & 2) ? sb[1] : -sb[1], (v & 4) ? sb[2] : -sb[2]}, w[3];
      matvec3(Rb, l, w);
      for (int i = 0; i < 3; i++) pts[v][i] = cb[i] + w[i];
    }
    np = 8;
  }
  int nc = 0;
  Contact cand[8];
  for (int k = 0; k < np; k++) {
    double v[3] = {pts[k][0] - cp[0], pts[k][1] - cp[1], pts[k][2] - cp[2]};
    double dist = dot3(v, n) - rad;
    if (dist >= margin) continue;
    Contact* c = cand + nc++;
    c->dist = dist;
    for (int i = 0; i < 3; i++) {
      c->n[i] = n[i];
      c->pos[i] = pts[k][i] - n[i] * (rad + 0.5 * dist);
    }
  }
  for (int i = 0; i < nc; i++)
    for (int j = i + 1; j < nc; j++)
      if (contact_deeper(&cand[j], &cand[i])) {
        Contact t = cand[i];
        cand[i] = cand[j];
        cand[j] = t;
      }
  int k = nc < 4 ? nc : 4;
  for (int i = 0; i < k; i++) out[i] = cand[i];
  return k;
}

/* ------------------------------------------------------------------------------------------
 * Convex narrow phase (meshes through their convex hulls, exact cylinders): MPR, restating
 * libccd's ccdMPRPenetration (mpr.c) as MuJoCo 3.1.6's mjc_Convex calls it [ext]: support points
 * of the Minkowski difference from the geoms' support functions (mjccd_support: sphere,
 * capsule, cylinder, box, mesh hull; inflated by margin / 2), tolerance 1e-6 (mjOption
 * mpr_tolerance), at most 50 refinement iterations (mpr_iterations); one contact per pair with
 * dist = margin - depth, normal = the penetration direction (from geom 1 to geom 2) and
 * position = the midpoint of the two witness points.
 * ---------------------------------------------------------------------------------------- */
#define CCD_EPS 2.2204460492503131e-16 /* DBL_EPSILON (libccd CCD_DOUBLE) */
#define MPR_TOLERANCE 1e-6
#define MPR_ITERATIONS 50

typedef struct {
  const double *c, *R, *s, *hv;
  int type, nhv;
  double margin;
} ConvexObj;

typedef struct {
  double v[3], v1[3], v2[3];
} SupportPt;

static int ccd_is_zero(double x) { return fabs(x) < CCD_EPS; }
static int ccd_eq(double a, double b) {
  double ab = fabs(a - b);
  if (ab < CCD_EPS) return 1;
  double fa = fabs(a), fb = fabs(b);
  return fb > fa ? ab < CCD_EPS * fb : ab < CCD_EPS * fa;
}
static int vec_eq(const double* a, const double* b) {
  return ccd_eq(a[0], b[0]) && ccd_eq(a[1], b[1]) && ccd_eq(a[2], b[2]);
}
static void vec_normalize(double* v) {
  double k = 1.0 / sqrt(dot3(v, v));
  v[0] *= k;
  v[1] *= k;
  v[2] *= k;
}
static double sgn0(double x) { return x < 0 ? -1.0 : (x > 0 ? 1.0 : 0.0); }

/* mjccd_support: farthest point of the object along the world direction dir */
static void convex_support(const ConvexObj* o, const double* dir, double* out) {
  double ld[3], res[3] = {0, 0, 0};
  mattvec3(o->R, dir, ld);
  const double* s = o->s;
  if (o->type == RMBX_GEOM_SPHERE || o->type == RMBX_GEOM_CAPSULE) {
    double n = norm3(ld);
    if (n > MINVAL)
      for (int i = 0; i < 3; i++) res[i] = ld[i] * (s[0] / n);
    if (o->type == RMBX_GEOM_CAPSULE) res[2] += sgn0(ld[2]) * s[1];
  } else if (o->type == RMBX_GEOM_CYLINDER) {
    double n = sqrt(ld[0] * ld[0] + ld[1] * ld[1]);
    if (n > MINVAL) {
      res[0] = ld[0] * (s[0] / n);
      res[1] = ld[1] * (s[0] / n);
    }
    res[2] = sgn0(ld[2]) * s[1];
  } else if (o->type == RMBX_GEOM_BOX) {
    for (int i = 0; i < 3; i++) res[i] = sgn0(ld[i]) * s[i];
  } else { /* mesh: hull vertex of largest projection (first on ties) */
    int best = 0;
    double bd = -1e300;
    for (int k = 0; k < o->nhv; k++) {
      double dd = dot3(o->hv + 3 * k, ld);
      if (dd > bd) {
        bd = dd;
        best = k;
      }
    }
    for (int i = 0; i < 3; i++) res[i] = o->hv[3 * best + i];
  }
  if (o->margin > 0) {
    double n = norm3(ld);
    if (n > MINVAL)
      for (int i = 0; i < 3; i++) res[i] += ld[i] * (0.5 * o->margin / n);
  }
  double w[3];
  matvec3(o->R, res, w);
  for (int i = 0; i < 3; i++) out[i] = o->c[i] + w[i];
}

static void mpr_support(const ConvexObj* a, const ConvexObj* b, const double* dir, SupportPt* p) {
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  convex_support(a, dir, p->v1);
  convex_support(b, nd, p->v2);
  for (int i = 0; i < 3; i++) p->v[i] = p->v1[i] - p->v2[i];
}

static double point_segment_dist2(const double* P, const double* x0, const double* b, double* witness) {
  double d[3] = {b[0] - x0[0], b[1] - x0[1], b[2] - x0[2]}, a[3] = {x0[0] - P[0], x0[1] - P[1], x0[2] - P[2]};
  double t = -1.0 * dot3(a, d);
  t /= dot3(d, d);
  double dist;
  if (t < 0 || ccd_is_zero(t)) {
    memcpy(witness, x0, sizeof(double) * 3);
  } else if (t > 1 || ccd_eq(t, 1.0)) {
    memcpy(witness, b, sizeof(double) * 3);
  } else {
    for (int i = 0; i < 3; i++) witness[i] = d[i] * t + x0[i];
  }
  double w[3] = {witness[0] - P[0], witness[1] - P[1], witness[2] - P[2]};
  dist = dot3(w, w);
  return dist;
}

/* ccdVec3PointTriDist2 with a witness point (here P is the origin) */
static double point_tri_dist2(const double* P, const double* x0, const double* B, const double* C, double* witness) {
  double d1[3], d2[3], a[3];
  for (int i = 0; i < 3; i++) {
    d1[i] = B[i] - x0[i];
    d2[i] = C[i] - x0[i];
    a[i] = x0[i] - P[i];
  }
  double v = dot3(d1, d1), w = dot3(d2, d2), p = dot3(a, d1), q = dot3(a, d2), r = dot3(d1, d2);
  double dd = w * v - r * r, s, t;
  if (ccd_is_zero(dd)) {
    s = t = -1.0;
  } else {
    s = (q * r - w * p) / dd;
    t = (-s * r - q) / w;
  }
  if ((ccd_is_zero(s) || s > 0) && (ccd_eq(s, 1.0) || s < 1) && (ccd_is_zero(t) || t > 0) &&
      (ccd_eq(t, 1.0) || t < 1) && (ccd_eq(t + s, 1.0) || t + s < 1)) {
    for (int i = 0; i < 3; i++) witness[i] = x0[i] + d1[i] * s + d2[i] * t;
    double e[3] = {witness[0] - P[0], witness[1] - P[1], witness[2] - P[2]};
    return dot3(e, e);
  }
  double w2[3];
  double dist = point_segment_dist2(P, x0, B, witness);
  double dist2 = point_segment_dist2(P, x0, C, w2);
  if (dist2 < dist) {
    dist = dist2;
    memcpy(witness, w2, sizeof(w2));
  }
  dist2 = point_segment_dist2(P, B, C, w2);
  if (dist2 < dist) {
    dist = dist2;
    memcpy(witness, w2, sizeof(w2));
  }
  return dist;
}

static void portal_dir(const SupportPt* pt, double* dir) {
  double v2v1[3], v3v1[3];
  for (int i = 0; i < 3; i++) {
    v2v1[i] = pt[2].v[i] - pt[1].v[i];
    v3v1[i] = pt[3].v[i] - pt[1].v[i];
  }
  cross3(v2v1, v3v1, dir);
  vec_normalize(dir);
}

static int portal_reach_tolerance(const SupportPt* pt, const SupportPt* v4, const double* dir) {
  double dv1 = dot3(pt[1].v, dir), dv2 = dot3(pt[2].v, dir), dv3 = dot3(pt[3].v, dir), dv4 = dot3(v4->v, dir);
  double d1 = dv4 - dv1, d2 = dv4 - dv2, d3 = dv4 - dv3;
  d1 = d1 < d2 ? d1 : d2;
  d1 = d1 < d3 ? d1 : d3;
  return ccd_eq(d1, MPR_TOLERANCE) || d1 < MPR_TOLERANCE;
}

static void expand_portal(SupportPt* pt, const SupportPt* v4) {
  double v4v0[3];
  cross3(v4->v, pt[0].v, v4v0);
  double dot = dot3(pt[1].v, v4v0);
  if (dot > 0) {
    dot = dot3(pt[2].v, v4v0);
    if (dot > 0)
      pt[1] = *v4;
    else
      pt[3] = *v4;
  } else {
    dot = dot3(pt[3].v, v4v0);
    if (dot > 0)
      pt[2] = *v4;
    else
      pt[1] = *v4;
  }
}

/* 0 portal found, 1 origin on v1 (touch), 2 origin on segment v0-v1, -1 no intersection */
static int discover_portal(const ConvexObj* a, const ConvexObj* b, SupportPt* pt) {
  double dir[3], va[3], vb[3];
  memcpy(pt[0].v1, a->c, sizeof(double) * 3);
  memcpy(pt[0].v2, b->c, sizeof(double) * 3);
  for (int i = 0; i < 3; i++) pt[0].v[i] = pt[0].v1[i] - pt[0].v2[i];
  const double zero[3] = {0, 0, 0};
  if (vec_eq(pt[0].v, zero)) pt[0].v[0] += CCD_EPS * 10.0;
  for (int i = 0; i < 3; i++) dir[i] = -pt[0].v[i];
  vec_normalize(dir);
  mpr_support(a, b, dir, &pt[1]);
  double dot = dot3(pt[1].v, dir);
  if (ccd_is_zero(dot) || dot < 0) return -1;
  cross3(pt[0].v, pt[1].v, dir);
  if (ccd_is_zero(dot3(dir, dir))) return vec_eq(pt[1].v, zero) ? 1 : 2;
  vec_normalize(dir);
  mpr_support(a, b, dir, &pt[2]);
  dot = dot3(pt[2].v, dir);
  if (ccd_is_zero(dot) || dot < 0) return -1;
  for (int i = 0; i < 3; i++) {
    va[i] = pt[1].v[i] - pt[0].v[i];
    vb[i] = pt[2].v[i] - pt[0].v[i];
  }
  cross3(va, vb, dir);
  vec_normalize(dir);
  if (dot3(dir, pt[0].v) > 0) {
    SupportPt t = pt[1];
    pt[1] = pt[2];
    pt[2] = t;
    for (int i = 0; i < 3; i++) dir[i] = -dir[i];
  }
  for (int guard = 0; guard < 1000; guard++) {
    mpr_support(a, b, dir, &pt[3]);
    dot = dot3(pt[3].v, dir);
    if (ccd_is_zero(dot) || dot < 0) return -1;
    int cont = 0;
    cross3(pt[1].v, pt[3].v, va);
    dot = dot3(va, pt[0].v);
    if (dot < 0 && !ccd_is_zero(dot)) {
      pt[2] = pt[3];
      cont = 1;
    }
    if (!cont) {
      cross3(pt[3].v, pt[2].v, va);
      dot = dot3(va, pt[0].v);
      if (dot < 0 && !ccd_is_zero(dot)) {
        pt[1] = pt[3];
        cont = 1;
      }
    }
    if (!cont) return 0;
    for (int i = 0; i < 3; i++) {
      va[i] = pt[1].v[i] - pt[0].v[i];
      vb[i] = pt[2].v[i] - pt[0].v[i];
    }
    cross3(va, vb, dir);
    vec_normalize(dir);
  }
  return -1;
}

static int refine_portal(const ConvexObj* a, const ConvexObj* b, SupportPt* pt) {
  double dir[3];
  SupportPt v4;
  for (int guard = 0; guard < 1000; guard++) {
    portal_dir(pt, dir);
    double dot = dot3(pt[1].v, dir);
    if (ccd_is_zero(dot) || dot > 0) return 0; /* portal encapsulates the origin */
    mpr_support(a, b, dir, &v4);
    dot = dot3(v4.v, dir);
    if (!(ccd_is_zero(dot) || dot > 0) || portal_reach_tolerance(pt, &v4, dir)) return -1;
    expand_portal(pt, &v4);
  }
  return -1;
}

static void find_pos(const SupportPt* pt, double* pos) {
  double dir[3], vec[3], bc[4];
  portal_dir(pt, dir);
  cross3(pt[1].v, pt[2].v, vec);
  bc[0] = dot3(vec, pt[3].v);
  cross3(pt[3].v, pt[2].v, vec);
  bc[1] = dot3(vec, pt[0].v);
  cross3(pt[0].v, pt[1].v, vec);
  bc[2] = dot3(vec, pt[3].v);
  cross3(pt[2].v, pt[1].v, vec);
  bc[3] = dot3(vec, pt[0].v);
  double sum = bc[0] + bc[1] + bc[2] + bc[3];
  if (ccd_is_zero(sum) || sum < 0) {
    bc[0] = 0;
    cross3(pt[2].v, pt[3].v, vec);
    bc[1] = dot3(vec, dir);
    cross3(pt[3].v, pt[1].v, vec);
    bc[2] = dot3(vec, dir);
    cross3(pt[1].v, pt[2].v, vec);
    bc[3] = dot3(vec, dir);
    sum = bc[1] + bc[2] + bc[3];
  }
  double inv = 1.0 / sum, p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < 3; i++) {
      p1[i] += pt[k].v1[i] * bc[k];
      p2[i] += pt[k].v2[i] * bc[k];
    }
  for (int i = 0; i < 3; i++) pos[i] = (p1[i] * inv + p2[i] * inv) * 0.5;
}

/* 1 with (depth, dir, pos) when the objects intersect, else 0 */
static int mpr_penetration(const ConvexObj* a, const ConvexObj* b, double* depth, double* dir, double* pos) {
  SupportPt pt[4];
  int res = discover_portal(a, b, pt);
  if (res < 0) return 0;
  if (res == 1) { /* touching contact: no normal */
    *depth = 0;
    dir[0] = dir[1] = dir[2] = 0;
    for (int i = 0; i < 3; i++) pos[i] = (pt[1].v1[i] + pt[1].v2[i]) * 0.5;
    return 1;
  }
  if (res == 2) { /* origin on the segment v0-v1 */
    for (int i = 0; i < 3; i++) {
      pos[i] = (pt[1].v1[i] + pt[1].v2[i]) * 0.5;
      dir[i] = pt[1].v[i];
    }
    *depth = sqrt(dot3(dir, dir));
    vec_normalize(dir);
    return 1;
  }
  if (refine_portal(a, b, pt) < 0) return 0;
  SupportPt v4;
  for (int it = 0;; it++) {
    double pd[3];
    portal_dir(pt, pd);
    mpr_support(a, b, pd, &v4);
    if (portal_reach_tolerance(pt, &v4, pd) || it > MPR_ITERATIONS) {
      const double zero[3] = {0, 0, 0};
      *depth = sqrt(point_tri_dist2(zero, pt[1].v, pt[2].v, pt[3].v, dir));
      if (ccd_is_zero(*depth))
        dir[0] = dir[1] = dir[2] = 0;
      else
        vec_normalize(dir);
      find_pos(pt, pos);
      return 1;
    }
    expand_portal(pt, &v4);
  }
}

static void convex_obj(const Data* d, int g, double margin, ConvexObj* o) {
  const rmbx_model* m = d->m;
  o->c = d->gxpos + 3 * g;
  o->R = d->gxmat + 9 * g;
  o->s = m->geom_csize + 3 * g;
  o->type = m->geom_ctype[g];
  o->hv = o->type == RMBX_GEOM_MESH ? m->hull_vert + 3 * m->geom_hulladr[g] : NULL;
  o->nhv = o->type == RMBX_GEOM_MESH ? m->geom_hullnum[g] : 0;
  o->margin = margin;
}

/* mjc_Convex: one contact from MPR (normal from A to B) */
static int col_convex(const Data* d, int ga, int gb, double margin, Contact* out) {
  ConvexObj a, b;
  convex_obj(d, ga, margin, &a);
  convex_obj(d, gb, margin, &b);
  double depth, dir[3], pos[3];
  if (!mpr_penetration(&a, &b, &depth, dir, pos)) return 0;
  if (dir[0] == 0 && dir[1] == 0 && dir[2] == 0) return 0; /* touching: normal undefined */
  double dist = margin - depth;
  if (dist >= margin) return 0;
  memcpy(out->n, dir, sizeof(dir));
  memcpy(out->pos, pos, sizeof(pos));
  out->dist = dist;
  return 1;
}

/* stable top-4 of a candidate stream by contact_deeper (earlier candidates win ties) */
static void top4_insert(Contact* best, int* nb, const Contact* c) {
  int k = *nb < 4 ? *nb : 4;
  int at = k;
  while (at > 0 && contact_deeper(c, &best[at - 1])) at--;
  if (at >= 4) return;
  for (int i = (k < 4 ? k : 3); i > at; i--) best[i] = best[i - 1];
  best[at] = *c;
  if (*nb < 4) (*nb)++;
}

/* plane (A, normal = local z) vs a convex hull (B): every hull vertex below the margin is a
 * candidate, the 4 deepest are kept (mjc_PlaneConvex's vertex contacts) */
static int col_plane_mesh(const double* cp, const double* Rp, const double* cb, const double* Rb,
                          const double* hv, int nhv, double margin, Contact* out) {
  double n[3] = {Rp[2], Rp[5], Rp[8]};
  int nb = 0;
  for (int k = 0; k < nhv; k++) {
    double w[3], x[3];
    matvec3(Rb, hv + 3 * k, w);
    for (int i = 0; i < 3; i++) x[i] = cb[i] + w[i];
    double v[3] = {x[0] - cp[0], x[1] - cp[1], x[2] - cp[2]};
    Contact c;
    c.dist = dot3(v, n);
    if (c.dist >= margin) continue;
    for (int i = 0; i < 3; i++) {
      c.n[i] = n[i];
      c.pos[i] = x[i] - n[i] * (0.5 * c.dist);
    }
    top4_insert(out, &nb, &c);
  }
  return nb;
}

/* plane (A) vs cylinder (B), after mjc_PlaneCylinder: the deepest rim point of each disk and
 * two more rim points of the deeper disk forming an equilateral triangle with its deepest */
static int col_plane_cylinder(const double* cp, const double* Rp, const double* cb, const double* Rb,
                              const double* sb, double margin, Contact* out) {
  double n[3] = {Rp[2], Rp[5], Rp[8]}, ax[3] = {Rb[2], Rb[5], Rb[8]};
  double r = sb[0], h = sb[1];
  double prj = dot3(n, ax);
  double u[3] = {-(n[0] - prj * ax[0]), -(n[1] - prj * ax[1]), -(n[2] - prj * ax[2])};
  double lu = norm3(u), v[3];
  if (lu < 1e-12) { /* axis along the normal: the disk's own x / y axes */
    u[0] = Rb[0];
    u[1] = Rb[3];
    u[2] = Rb[6];
  } else {
    for (int i = 0; i < 3; i++) u[i] /= lu;
  }
  cross3(ax, u, v);
  /* the deeper disk is the one whose centre lies further along -n */
  double sgn = prj > 0 ? -1.0 : 1.0; /* cap at c + sgn h ax is the deeper one */
  double cd[3], cs[3];
  for (int i = 0; i < 3; i++) {
    cd[i] = cb[i] + sgn * h * ax[i];
    cs[i] = cb[i] - sgn * h * ax[i];
  }
  double pts[4][3];
  const double s3 = 0.86602540378443864676;
  for (int i = 0; i < 3; i++) {
    pts[0][i] = cd[i] + r * u[i];
    pts[1][i] = cs[i] + r * u[i];
    pts[2][i] = cd[i] - 0.5 * r * u[i] + s3 * r * v[i];
    pts[3][i] = cd[i] - 0.5 * r * u[i] - s3 * r * v[i];
  }
  int nb = 0;
  for (int k = 0; k < 4; k++) {
    double w[3] = {pts[k][0] - cp[0], pts[k][1] - cp[1], pts[k][2] - cp[2]};
    Contact c;
    c.dist = dot3(w, n);
    if (c.dist >= margin) continue;
    for (int i = 0; i < 3; i++) {
      c.n[i] = n[i];
      c.pos[i] = pts[k][i] - n[i] * (0.5 * c.dist);
    }
    top4_insert(out, &nb, &c);
  }
  return nb;
}

static int narrowphase(Data* d, int g1, int g2, double margin, Contact* out) {
  const rmbx_model* m = d->m;
  int t1 = m->geom_ctype[g1], t2 = m->geom_ctype[g2];
  int flip = 0;
  if (t1 > t2) {
    int t = t1;
    t1 = t2;
    t2 = t;
    int g = g1;
    g1 = g2;
    g2 = g;
    flip = 1;
  }
  const double *c1 = d->gxpos + 3 * g1, *R1 = d->gxmat + 9 * g1, *s1 = m->geom_csize + 3 * g1;
  const double *c2 = d->gxpos + 3 * g2, *R2 = d->gxmat + 9 * g2, *s2 = m->geom_csize + 3 * g2;
  int n = 0;
  if (t1 == RMBX_GEOM_PLANE && t2 == RMBX_GEOM_MESH) {
    n = col_plane_mesh(c1, R1, c2, R2, m->hull_vert + 3 * m->geom_hulladr[g2], m->geom_hullnum[g2], margin, out);
  } else if (t1 == RMBX_GEOM_PLANE && t2 == RMBX_GEOM_CYLINDER) {
    n = col_plane_cylinder(c1, R1, c2, R2, s2, margin, out);
  } else if (t1 == RMBX_GEOM_PLANE) {
    n = col_plane(c1, R1, t2, c2, R2, s2, margin, out);
  } else if (t2 == RMBX_GEOM_MESH || t2 == RMBX_GEOM_CYLINDER) {
    n = col_convex(d, g1, g2, margin, out);
  } else if (t1 == RMBX_GEOM_SPHERE && t2 == RMBX_GEOM_SPHERE) {
    n = col_sphere_sphere(c1, s1[0], c2, s2[0], margin, out);
  } else if (t1 == RMBX_GEOM_SPHERE && t2 == RMBX_GEOM_CAPSULE) {
    double p[3], q[3], c[3], cc[3];
    capsule_ends(c2, R2, s2[1], p, q);
    closest_seg_seg(c1, c1, p, q, cc, c);
    n = col_sphere_sphere(c1, s1[0], c, s2[0], margin, out);
  } else if (t1 == RMBX_GEOM_SPHERE && t2 == RMBX_GEOM_BOX) {
    n = col_sphere_box(c1, s1[0], c2, R2, s2, margin, out);
  } else if (t1 == RMBX_GEOM_CAPSULE && t2 == RMBX_GEOM_CAPSULE) {
    n = col_capsule_capsule(c1, R1, s1, c2, R2, s2, margin, out);
  } else if (t1 == RMBX_GEOM_CAPSULE && t2 == RMBX_GEOM_BOX) {
    n = col_capsule_box(c1, R1, s1, c2, R2, s2, margin, out);
  } else if (t1 == RMBX_GEOM_BOX && t2 == RMBX_GEOM_BOX) {
    n = col_box_box(c1, R1, s1, c2, R2, s2, margin, out);
  }
  if (flip)
    for (int i = 0; i < n; i++)
      for (int k = 0; k < 3; k++) out[i].n[k] = -out[i].n[k];
  return n;
}

static void geom_aabb(const Data* d, int g, double* lo, double* hi) {
  const rmbx_model* m = d->m;
  const double *c = d->gxpos + 3 * g, *R = d->gxmat + 9 * g, *s = m->geom_csize + 3 * g;
  int t = m->geom_ctype[g];
  for (int i = 0; i < 3; i++) {
    double e;
    if (t == RMBX_GEOM_SPHERE)
      e = s[0];
    else if (t == RMBX_GEOM_CAPSULE || t == RMBX_GEOM_CYLINDER)
      e = fabs(R[3 * i + 2]) * s[1] + s[0];
    else
      e = fabs(R[3 * i]) * s[0] + fabs(R[3 * i + 1]) * s[1] + fabs(R[3 * i + 2]) * s[2];
    lo[i] = c[i] - e;
    hi[i] = c[i] + e;
  }
}

static void make_frame(const double* n, double* F) {
  F[0] = n[0];
  F[1] = n[1];
  F[2] = n[2];
  double a[3] = {0, 0, 0};
  if (fabs(n[0]) < 0.5)
    a[0] = 1;
  else
    a[1] = 1;
  double t = dot3(a, n);
  double t1[3] = {a[0] - t * n[0], a[1] - t * n[1], a[2] - t * n[2]};
  double l = norm3(t1);
  t1[0] /= l;
  t1[1] /= l;
  t1[2] /= l;
  double t2[3];
  cross3(n, t1, t2);
  memcpy(F + 3, t1, sizeof(t1));
  memcpy(F + 6, t2, sizeof(t2));
}

/* broadphase survivors taken into the narrow phase: at most this many, in pair order (the
 * engine's LDS survivor list has the same cap) */
#define MAX_CANDIDATES 2048

static void collision(Data* d) {
  const rmbx_model* m = d->m;
  d->ncon = 0;
  int cap = m->npair < MAX_CANDIDATES ? m->npair : MAX_CANDIDATES, nsurv = 0;
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p];
    double margin = m->pair_margin[p];
    int t1 = m->geom_ctype[g1], t2 = m->geom_ctype[g2];
    if (t1 == RMBX_GEOM_PLANE || t2 == RMBX_GEOM_PLANE) {
      int gp = t1 == RMBX_GEOM_PLANE ? g1 : g2, go = gp == g1 ? g2 : g1;
      const double* R = d->gxmat + 9 * gp;
      double n[3] = {R[2], R[5], R[8]};
      double v[3] = {d->gxpos[3 * go] - d->gxpos[3 * gp], d->gxpos[3 * go + 1] - d->gxpos[3 * gp + 1],
                     d->gxpos[3 * go + 2] - d->gxpos[3 * gp + 2]};
      if (dot3(v, n) - m->geom_rbound[go] > margin) continue;
    } else {
      double lo1[3], hi1[3], lo2[3], hi2[3];
      geom_aabb(d, g1, lo1, hi1);
      geom_aabb(d, g2, lo2, hi2);
      int sep = 0;
      for (int i = 0; i < 3; i++)
        if (lo1[i] > hi2[i] + margin || lo2[i] > hi1[i] + margin) sep = 1;
      if (sep) continue;
    }
    if (nsurv >= cap) break;
    nsurv++;
    Contact c[MAXCON_PAIR];
    int n = narrowphase(d, g1, g2, margin, c);
    for (int i = 0; i < n && d->ncon < m->max_contacts; i++) {
      int k = d->ncon++;
      memcpy(d->con_pos + 3 * k, c[i].pos, sizeof(double) * 3);
      make_frame(c[i].n, d->con_frame + 9 * k);
      d->con_dist[k] = c[i].dist;
      d->con_b1[k] = m->geom_body[g1];
      d->con_b2[k] = m->geom_body[g2];
      d->con_condim[k] = m->pair_condim[p];
      d->con_mu[k] = m->pair_friction[3 * p];
      d->con_pair[k] = p;
    }
  }
}

/* ------------------------------------------------------------------------------------------
 * Jacobians and constraint rows
 * ---------------------------------------------------------------------------------------- */
static int last_dof(const rmbx_model* m, int b) {
  int w = m->body_weldid[b];
  if (w == 0) return -1;
  return m->body_dofadr[w] + m->body_dofnum[w] - 1;
}
/* accumulate sgn * (translational Jacobian of point p on body b) projected on dir (3) into row */
static void jac_point_dir(Data* d, int b, const double* p, const double* dir, double sgn, double* row) {
  const rmbx_model* m = d->m;
  for (int k = last_dof(m, b); k >= 0; k = m->dof_parent[k]) {
    const double* S = d->cdof + 6 * k;
    double wxp[3];
    cross3(S, p, wxp);
    double v[3] = {S[3] + wxp[0], S[4] + wxp[1], S[5] + wxp[2]};
    row[k] += sgn * dot3(v, dir);
  }
}
static void jac_rot_dir(Data* d, int b, const double* dir, double sgn, double* row) {
  const rmbx_model* m = d->m;
  for (int k = last_dof(m, b); k >= 0; k = m->dof_parent[k]) row[k] += sgn * dot3(d->cdof + 6 * k, dir);
}

static double impedance(const double* solimp, double x) {
  double dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (dmin < 0.0001) dmin = 0.0001;
  if (dmin > 0.9999) dmin = 0.9999;
  if (dmax < 0.0001) dmax = 0.0001;
  if (dmax > 0.9999) dmax = 0.9999;
  x = fabs(x);
  if (width <= MINVAL || x >= width) return dmax;
  x = x / width;
  double y;
  if (power == 1)
    y = x;
  else if (x <= mid)
    y = pow(x, power) / pow(mid, power - 1);
  else
    y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  return dmin + y * (dmax - dmin);
}

static int add_row(Data* d, int type, double pos, double diag, const double* solref, const double* solimp,
                   double impx) {
  int r = d->nefc;
  if (r >= d->nefc_max) return -1;
  d->nefc++;
  d->efc_type[r] = type;
  d->efc_pos[r] = pos;
  double dmax = solimp[1] < 0.0001 ? 0.0001 : (solimp[1] > 0.9999 ? 0.9999 : solimp[1]);
  double tc = solref[0], dr = solref[1];
  double h2 = 2 * d->m->timestep;
  if (tc < h2) tc = h2;
  double k = 1 / (dmax * dmax * tc * tc * dr * dr);
  double bdamp = 2 / (dmax * tc);
  double imp = impedance(solimp, impx);
  d->efc_aref[r] = bdamp; /* temporarily store b; k*imp*pos folded below */
  d->efc_D[r] = k * imp * pos;
  double R = (1 - imp) / imp * diag;
  if (R < MINVAL) R = MINVAL;
  d->efc_R[r] = R;
  return r;
}

static void make_constraints(Data* d) {
  const rmbx_model* m = d->m;
  int nv = m->nv;
  d->nefc = 0;
  memset(d->J, 0, sizeof(double) * (size_t)d->nefc_max * nv);
  /* equality constraints */
  for (int e = 0; e < m->neq; e++) {
    const double* data = m->eq_data + RMBX_EQ_DATA * e;
    const double *sr = m->eq_solref + 2 * e, *si = m->eq_solimp + 5 * e;
    int o1 = m->eq_obj1[e], o2 = m->eq_obj2[e];
    if (m->eq_type[e] == RMBX_EQ_CONNECT || m->eq_type[e] == RMBX_EQ_WELD) {
      double p1[3], p2[3], t[3];
      double err[6];
      int nr = m->eq_type[e] == RMBX_EQ_CONNECT ? 3 : 6;
      if (m->eq_type[e] == RMBX_EQ_CONNECT) {
        matvec3(d->xmat + 9 * o1, data, t);
        for (int i = 0; i < 3; i++) p1[i] = d->xpos[3 * o1 + i] + t[i];
        matvec3(d->xmat + 9 * o2, data + 3, t);
        for (int i = 0; i < 3; i++) p2[i] = d->xpos[3 * o2 + i] + t[i];
      } else {
        double Rr[9], ra[3], u[3];
        quat2mat(data + 6, Rr);
        matvec3(Rr, data, ra);
        for (int i = 0; i < 3; i++) u[i] = data[3 + i] + ra[i];
        matvec3(d->xmat + 9 * o1, u, t);
        for (int i = 0; i < 3; i++) p1[i] = d->xpos[3 * o1 + i] + t[i];
        matvec3(d->xmat + 9 * o2, data, t);
        for (int i = 0; i < 3; i++) p2[i] = d->xpos[3 * o2 + i] + t[i];
      }
      for (int i = 0; i < 3; i++) err[i] = p1[i] - p2[i];
      double q1r[4], qe[4], cq1[4];
      if (nr == 6) {
        quatmul(d->xquat + 4 * o1, data + 6, q1r);
        cq1[0] = q1r[0];
        cq1[1] = -q1r[1];
        cq1[2] = -q1r[2];
        cq1[3] = -q1r[3];
        quatmul(cq1, d->xquat + 4 * o2, qe);
        for (int i = 0; i < 3; i++) err[3 + i] = qe[1 + i] * data[10];
      }
      double nrm = 0;
      for (int i = 0; i < nr; i++) nrm += err[i] * err[i];
      nrm = sqrt(nrm);
      for (int i = 0; i < 3; i++) {
        double dir[3] = {0, 0, 0};
        dir[i] = 1;
        double diag = m->body_invweight0[2 * o1] + m->body_invweight0[2 * o2];
        int r = add_row(d, 0, err[i], diag, sr, si, nrm);
        if (r < 0) return;
        jac_point_dir(d, o1, p1, dir, 1.0, d->J + (size_t)r * nv);
        jac_point_dir(d, o2, p2, dir, -1.0, d->J + (size_t)r * nv);
      }
      if (nr == 6) {
        /* rotational rows: Im(0.5 conj(q1r) [0, Jr2 - Jr1] q2) * torquescale */
        double diag = m->body_invweight0[2 * o1 + 1] + m->body_invweight0[2 * o2 + 1];
        int r0 = d->nefc;
        for (int i = 0; i < 3; i++)
          if (add_row(d, 0, err[3 + i], diag, sr, si, nrm) < 0) return;
        double jr[3 * 128];
        (void)jr;
        for (int k = 0; k < nv; k++) {
          double w[3] = {0, 0, 0};
          /* rotational Jacobian column k of body o2 minus o1 */
          int in2 = 0, in1 = 0;
          for (int kk = last_dof(m, o2); kk >= 0; kk = m->dof_parent[kk])
            if (kk == k) in2 = 1;
          for (int kk = last_dof(m, o1); kk >= 0; kk = m->dof_parent[kk])
            if (kk == k) in1 = 1;
          if (!in1 && !in2) continue;
          for (int i = 0; i < 3; i++) w[i] = (in2 ? d->cdof[6 * k + i] : 0) - (in1 ? d->cdof[6 * k + i] : 0);
          double wq[4] = {0, w[0], w[1], w[2]}, t1[4], t2[4];
          quatmul(cq1, wq, t1);
          quatmul(t1, d->xquat + 4 * o2, t2);
          for (int i = 0; i < 3; i++) d->J[(size_t)(r0 + i) * nv + k] = 0.5 * t2[1 + i] * data[10];
        }
      }
    } else if (m->eq_type[e] == RMBX_EQ_JOINT) {
      int j1 = o1, j2 = o2;
      double q1 = d->qpos[m->jnt_qposadr[j1]] - m->qpos0[m->jnt_qposadr[j1]];
      double q2 = d->qpos[m->jnt_qposadr[j2]] - m->qpos0[m->jnt_qposadr[j2]];
      const double* c = data;
      double poly = c[0] + q2 * (c[1] + q2 * (c[2] + q2 * (c[3] + q2 * c[4])));
      double dpoly = c[1] + q2 * (2 * c[2] + q2 * (3 * c[3] + q2 * 4 * c[4]));
      double err = q1 - poly;
      int d1 = m->jnt_dofadr[j1], d2 = m->jnt_dofadr[j2];
      int r = add_row(d, 0, err, m->dof_invweight0[d1] + m->dof_invweight0[d2], sr, si, err);
      if (r < 0) return;
      d->J[(size_t)r * nv + d1] += 1;
      d->J[(size_t)r * nv + d2] -= dpoly;
    }
  }
  d->ne = d->nefc;
  /* joint limits */
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j]) continue;
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    double q = d->qpos[qa];
    for (int side = 0; side < 2; side++) {
      double dist = side == 0 ? q - m->jnt_range[2 * j] : m->jnt_range[2 * j + 1] - q;
      if (dist < 0) {
        int r = add_row(d, 1, dist, m->dof_invweight0[da], m->jnt_solref + 2 * j, m->jnt_solimp + 5 * j, dist);
        if (r < 0) return;
        d->J[(size_t)r * nv + da] = side == 0 ? 1.0 : -1.0;
      }
    }
  }
  /* contacts: pyramidal */
  for (int c = 0; c < d->ncon; c++) {
    int p = d->con_pair[c];
    int b1 = d->con_b1[c], b2 = d->con_b2[c];
    const double* F = d->con_frame + 9 * c;
    const double* pos = d->con_pos + 3 * c;
    double tran = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
    double dist = d->con_dist[c] - m->pair_margin[p];
    const double *sr = m->pair_solref + 2 * p, *si = m->pair_solimp + 5 * p;
    d->con_efcadr[c] = d->nefc;
    if (d->con_condim[c] == 1) {
      int r = add_row(d, 1, dist, tran, sr, si, dist);
      if (r < 0) return;
      jac_point_dir(d, b2, pos, F, 1.0, d->J + (size_t)r * nv);
      jac_point_dir(d, b1, pos, F, -1.0, d->J + (size_t)r * nv);
    } else {
      double mu = d->con_mu[c];
      for (int t = 0; t < 2; t++)
        for (int sgn = 0; sgn < 2; sgn++) {
          double dir[3];
          double s = sgn == 0 ? mu : -mu;
          for (int i = 0; i < 3; i++) dir[i] = F[i] + s * F[3 * (1 + t) + i];
          int r = add_row(d, 1, dist, tran * (1 + mu * mu), sr, si, dist);
          if (r < 0) return;
          jac_point_dir(d, b2, pos, dir, 1.0, d->J + (size_t)r * nv);
          jac_point_dir(d, b1, pos, dir, -1.0, d->J + (size_t)r * nv);
        }
    }
  }
  /* aref = -b * (J qvel) - k * imp * pos ; D = 1 / R */
  for (int r = 0; r < d->nefc; r++) {
    const double* Jr = d->J + (size_t)r * nv;
    double v = 0;
    for (int k = 0; k < nv; k++) v += Jr[k] * d->qvel[k];
    d->efc_vel[r] = v;
    double b = d->efc_aref[r];
    d->efc_aref[r] = -b * v - d->efc_D[r];
    d->efc_D[r] = 1.0 / d->efc_R[r];
  }
}

/* ------------------------------------------------------------------------------------------
 * primal Newton solver (mj_solNewton) with exact line search
 * ---------------------------------------------------------------------------------------- */
static void matvec_sym(const double* A, const double* x, double* y, int n) {
  for (int i = 0; i < n; i++) {
    double s = 0;
    for (int k = 0; k < n; k++) s += A[i * n + k] * x[k];
    y[i] = s;
  }
}

/* cost at qacc a; fills efc_jar; returns total */
static double eval_cost(Data* d, const double* a) {
  const rmbx_model* m = d->m;
  int nv = m->nv;
  for (int k = 0; k < nv; k++) d->res[k] = a[k] - d->qacc_smooth[k];
  matvec_sym(d->M, d->res, d->tmpv2, nv);
  double cost = 0;
  for (int k = 0; k < nv; k++) cost += d->res[k] * d->tmpv2[k];
  cost *= 0.5;
  for (int r = 0; r < d->nefc; r++) {
    const double* Jr = d->J + (size_t)r * nv;
    double s = 0;
    for (int k = 0; k < nv; k++) s += Jr[k] * a[k];
    double jar = s - d->efc_aref[r];
    d->efc_jar[r] = jar;
    if (d->efc_type[r] == 0 || jar < 0) cost += 0.5 * d->efc_D[r] * jar * jar;
  }
  return cost;
}

static void solve(Data* d) {
  const rmbx_model* m = d->m;
  int nv = m->nv, nefc = d->nefc;
  double* a = d->qacc;
  /* qacc_smooth = M^-1 qfrc_smooth */
  memcpy(d->L, d->M, sizeof(double) * nv * nv);
  cholesky(d->L, nv);
  chol_solve(d->L, nv, d->qfrc_smooth, d->qacc_smooth);
  /* warmstart: pick the lower-cost start (cost of qacc_smooth: res = 0, only the rows) */
  double c_ws = eval_cost(d, d->qacc_ws);
  memcpy(d->tmpv3, d->tmpv2, sizeof(double) * nv); /* M res of the warm start */
  memcpy(d->efc_tmp, d->efc_jar, sizeof(double) * nefc);
  double c_sm = 0;
  for (int r = 0; r < nefc; r++) {
    const double* Jr = d->J + (size_t)r * nv;
    double s = 0;
    for (int k = 0; k < nv; k++) s += Jr[k] * d->qacc_smooth[k];
    double jar = s - d->efc_aref[r];
    d->efc_jar[r] = jar;
    if (d->efc_type[r] == 0 || jar < 0) c_sm += 0.5 * d->efc_D[r] * jar * jar;
  }
  double cost;
  if (c_ws < c_sm) {
    memcpy(a, d->qacc_ws, sizeof(double) * nv);
    for (int k = 0; k < nv; k++) d->res[k] = a[k] - d->qacc_smooth[k];
    memcpy(d->tmpv2, d->tmpv3, sizeof(double) * nv);
    memcpy(d->efc_jar, d->efc_tmp, sizeof(double) * nefc);
    cost = c_ws;
  } else {
    memcpy(a, d->qacc_smooth, sizeof(double) * nv);
    for (int k = 0; k < nv; k++) d->res[k] = d->tmpv2[k] = 0;
    cost = c_sm;
  }
  double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  int it;
  for (int k = 0; k < 128; k++) d->trace_grad[k] = d->trace_impr[k] = d->trace_kink[k] = -1.0;
  for (it = 0; it < m->solver_iterations; it++) {
    /* gradient: M (a - a0) - J^T f, f = -D jar on active rows (res/tmpv2 set by eval_cost) */
    for (int k = 0; k < nv; k++) d->grad[k] = d->tmpv2[k];
    for (int r = 0; r < nefc; r++) {
      double jar = d->efc_jar[r];
      if (d->efc_type[r] == 0 || jar < 0) {
        double f = d->efc_D[r] * jar;
        const double* Jr = d->J + (size_t)r * nv;
        for (int k = 0; k < nv; k++) d->grad[k] += Jr[k] * f;
      }
    }
    double gn = 0;
    for (int k = 0; k < nv; k++) gn += d->grad[k] * d->grad[k];
    if (it < 128) {
      d->trace_grad[it] = scale * sqrt(gn);
      /* nearest inequality row to its kink (jar = 0), relative to the largest |jar|: an exact line
         search often stops at a kink, where the row's side is decided by rounding */
      double mn = 1e300, mx = 0;
      for (int r = d->ne; r < nefc; r++) {
        const double x = fabs(d->efc_jar[r]);
        if (x > 0) mn = x < mn ? x : mn;  /* (an exact 0 is no rounding question) */
        mx = x > mx ? x : mx;
      }
      d->trace_kink[it] = mx > 0 ? mn / mx : 1.0;
    }
    if (scale * sqrt(gn) < m->solver_tolerance) break;
    /* Hessian H = M + J^T D_active J */
    memcpy(d->H, d->M, sizeof(double) * nv * nv);
    for (int r = 0; r < nefc; r++) {
      double jar = d->efc_jar[r];
      if (!(d->efc_type[r] == 0 || jar < 0)) continue;
      const double* Jr = d->J + (size_t)r * nv;
      double D = d->efc_D[r];
      for (int i = 0; i < nv; i++) {
        if (Jr[i] == 0) continue;
        double t = D * Jr[i];
        for (int k = 0; k <= i; k++) d->H[i * nv + k] += t * Jr[k];
      }
    }
    for (int i = 0; i < nv; i++)
      for (int k = 0; k < i; k++) d->H[k * nv + i] = d->H[i * nv + k];
    cholesky(d->H, nv);
    chol_solve(d->H, nv, d->grad, d->search);
    for (int k = 0; k < nv; k++) d->search[k] = -d->search[k];
    /* exact line search on the piecewise quadratic */
    matvec_sym(d->M, d->search, d->Ms, nv);
    double qg = 0, lg = 0;
    for (int k = 0; k < nv; k++) {
      qg += d->search[k] * d->Ms[k];
      lg += d->res[k] * d->Ms[k];
    }
    for (int r = 0; r < nefc; r++) {
      const double* Jr = d->J + (size_t)r * nv;
      double s = 0;
      for (int k = 0; k < nv; k++) s += Jr[k] * d->search[k];
      d->efc_Js[r] = s;
    }
    double alpha = 0, lo = 0, hi = 1e300;
    for (int ls = 0; ls < m->ls_iterations; ls++) {
      double d1 = alpha * qg + lg, d2 = qg;
      for (int r = 0; r < nefc; r++) {
        double x = d->efc_jar[r] + alpha * d->efc_Js[r];
        if (d->efc_type[r] == 0 || x < 0) {
          d1 += d->efc_D[r] * x * d->efc_Js[r];
          d2 += d->efc_D[r] * d->efc_Js[r] * d->efc_Js[r];
        }
      }
      if (d1 == 0) break;
      if (d1 < 0)
        lo = alpha;
      else
        hi = alpha;
      double an = alpha - d1 / d2;
      if (!(an > lo && an < hi)) an = hi < 1e300 ? 0.5 * (lo + hi) : (an > lo ? an : lo);
      /* exact if the active set is unchanged between alpha and an */
      int same = 1;
      for (int r = d->ne; r < nefc; r++) {
        double x0 = d->efc_jar[r] + alpha * d->efc_Js[r], x1 = d->efc_jar[r] + an * d->efc_Js[r];
        if ((x0 < 0) != (x1 < 0)) {
          same = 0;
          break;
        }
      }
      alpha = an;
      if (same) break;
    }
    /* move along the search direction; res, M res and jar are updated incrementally
       (mj_solNewton's qacc / Ma / efc_Jaref updates) */
    for (int k = 0; k < nv; k++) {
      a[k] += alpha * d->search[k];
      d->res[k] += alpha * d->search[k];
      d->tmpv2[k] += alpha * d->Ms[k];
    }
    double newcost = 0;
    for (int k = 0; k < nv; k++) newcost += d->res[k] * d->tmpv2[k];
    newcost *= 0.5;
    for (int r = 0; r < nefc; r++) {
      double jar = d->efc_jar[r] + alpha * d->efc_Js[r];
      d->efc_jar[r] = jar;
      if (d->efc_type[r] == 0 || jar < 0) newcost += 0.5 * d->efc_D[r] * jar * jar;
    }
    double improvement = scale * (cost - newcost);
    if (it < 128) d->trace_impr[it] = improvement;
    cost = newcost;
    if (improvement < m->solver_tolerance) {
      it++;
      break;
    }
  }
  d->solver_iter = it;
  /* final forces with the last eval_cost's jar */
  memset(d->qfrc_constraint, 0, sizeof(double) * nv);
  for (int r = 0; r < nefc; r++) {
    double jar = d->efc_jar[r];
    double f = (d->efc_type[r] == 0 || jar < 0) ? -d->efc_D[r] * jar : 0.0;
    d->efc_force[r] = f;
    const double* Jr = d->J + (size_t)r * nv;
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] += Jr[k] * f;
  }
}

/* ------------------------------------------------------------------------------------------
 * sensors: mj_rnePostConstraint -> cfrc_int -> force/torque in site frame
 * ---------------------------------------------------------------------------------------- */
static void sensors(Data* d) {
  const rmbx_model* m = d->m;
  if (m->nsensor == 0) return;
  rne(d, d->qacc, NULL);
  /* subtract external contact forces */
  for (int c = 0; c < d->ncon; c++) {
    int r0 = d->con_efcadr[c];
    const double* F = d->con_frame + 9 * c;
    double fn, f1 = 0, f2 = 0;
    if (d->con_condim[c] == 1) {
      fn = d->efc_force[r0];
    } else {
      double mu = d->con_mu[c];
      const double* f = d->efc_force + r0;
      fn = f[0] + f[1] + f[2] + f[3];
      f1 = mu * (f[0] - f[1]);
      f2 = mu * (f[2] - f[3]);
    }
    double Fw[3], pxF[3];
    for (int i = 0; i < 3; i++) Fw[i] = fn * F[i] + f1 * F[3 + i] + f2 * F[6 + i];
    cross3(d->con_pos + 3 * c, Fw, pxF);
    int b2 = d->con_b2[c], b1 = d->con_b1[c];
    for (int i = 0; i < 3; i++) {
      d->cfrc[6 * b2 + i] -= pxF[i];
      d->cfrc[6 * b2 + 3 + i] -= Fw[i];
      d->cfrc[6 * b1 + i] += pxF[i];
      d->cfrc[6 * b1 + 3 + i] += Fw[i];
    }
  }
  rne_backward(d, NULL);
  for (int s = 0; s < m->nsensor && s < 2; s++) {
    int site = m->sensor_site[s];
    int b = m->site_body[site];
    const double* f = d->cfrc + 6 * b;
    const double* p = d->sxpos + 3 * site;
    const double* R = d->sxmat + 9 * site;
    double out[3];
    if (m->sensor_type[s] == RMBX_SENS_FORCE) {
      mattvec3(R, f + 3, out);
    } else {
      double pxf[3], n[3];
      cross3(p, f + 3, pxf);
      for (int i = 0; i < 3; i++) n[i] = f[i] - pxf[i];
      mattvec3(R, n, out);
    }
    memcpy(d->sensordata + 3 * s, out, sizeof(out));
  }
}

/* ------------------------------------------------------------------------------------------
 * implicitfast integration + mj_step
 * ---------------------------------------------------------------------------------------- */
void orc_forward(void* p);

/* mj_step after mj_forward (MuJoCo 3.1.6 [ext]): mj_checkAcc on the forward (constraint-solver)
 * qacc -- a non-finite or |qacc| > 1e10 entry resets the data (mj_resetData: qpos0, zero velocity
 * / warm start / ctrl, time 0) and runs mj_forward on the reset state -- then the implicitfast
 * integration of this substep, from the reset state when there was one. */
static void integrate(Data* d) {
  for (int k = 0; k < d->m->nv; k++)
    if (!isfinite(d->qacc[k]) || fabs(d->qacc[k]) > 1e10) {
      memcpy(d->qpos, d->m->qpos0, sizeof(double) * d->m->nq);
      memset(d->qvel, 0, sizeof(double) * d->m->nv);
      memset(d->qacc_ws, 0, sizeof(double) * d->m->nv);
      memset(d->ctrl, 0, sizeof(double) * d->m->nu);
      d->time = 0;
      d->bad = d->substep;
      orc_forward(d);
      break;
    }
  const rmbx_model* m = d->m;
  int nv = m->nv;
  double h = m->timestep;
  /* A = M + h * Dv, Dv = damping + actuator velocity gains (-bias[2] * moment moment^T) */
  memcpy(d->A, d->M, sizeof(double) * nv * nv);
  for (int k = 0; k < nv; k++) d->A[k * nv + k] += h * m->dof_damping[k];
  for (int u = 0; u < m->nu; u++) {
    double kv = -m->act_bias[3 * u + 2];
    if (kv == 0) continue;
    int id = m->act_trnid[u];
    if (m->act_trntype[u] == RMBX_TRN_JOINT) {
      int k = m->jnt_dofadr[id];
      d->A[k * nv + k] += h * kv;
    } else {
      for (int w1 = m->ten_adr[id]; w1 < m->ten_adr[id] + m->ten_num[id]; w1++)
        for (int w2 = m->ten_adr[id]; w2 < m->ten_adr[id] + m->ten_num[id]; w2++) {
          int k1 = m->jnt_dofadr[m->wrap_jnt[w1]], k2 = m->jnt_dofadr[m->wrap_jnt[w2]];
          d->A[k1 * nv + k2] += h * kv * m->wrap_coef[w1] * m->wrap_coef[w2];
        }
    }
  }
  cholesky(d->A, nv);
  for (int k = 0; k < nv; k++) d->tmpv[k] = d->qfrc_smooth[k] + d->qfrc_constraint[k];
  chol_solve(d->A, nv, d->tmpv, d->qacc);
  for (int k = 0; k < nv; k++) d->qvel[k] += h * d->qacc[k];
  memcpy(d->qacc_ws, d->qacc, sizeof(double) * nv);
  for (int j = 0; j < m->njnt; j++) {
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (m->jnt_type[j] == RMBX_JNT_FREE) {
      for (int i = 0; i < 3; i++) d->qpos[qa + i] += h * d->qvel[da + i];
      const double* w = d->qvel + da + 3;
      double nw = norm3(w);
      if (nw > MINVAL) {
        double ax[3] = {w[0] / nw, w[1] / nw, w[2] / nw}, qr[4];
        axisangle_quat(ax, nw * h, qr);
        quatmul(d->qpos + qa + 3, qr, d->qpos + qa + 3);
      }
      quatnorm(d->qpos + qa + 3);
    } else {
      d->qpos[qa] += h * d->qvel[da];
    }
  }
  d->time += h;
}

void orc_forward(void* p) {
  Data* d = (Data*)p;
  kinematics(d);
  com_pos(d);
  crb(d);
  com_vel(d);
  rne(d, NULL, NULL);
  rne_backward(d, d->qfrc_bias);
  passive_actuation(d);
  for (int k = 0; k < d->m->nv; k++)
    d->qfrc_smooth[k] = d->qfrc_passive[k] + d->qfrc_actuator[k] - d->qfrc_bias[k];
  collision(d);
  make_constraints(d);
  solve(d);
  sensors(d);
}

/* returns the 1-based substep of the last divergence reset in this call (0: none), the
 * engine's stats[3] */
int orc_step(void* p, int nsub) {
  Data* d = (Data*)p;
  d->bad = 0;
  for (int s = 0; s < nsub; s++) {
    d->substep = s + 1;
    orc_forward(d);
    integrate(d);
  }
  return d->bad;
}

/* ------------------------------------------------------------------------------------------
 * accessors
 * ---------------------------------------------------------------------------------------- */
void orc_set_state(void* p, double time, const double* qpos, const double* qvel, const double* qacc_ws,
                   const double* ctrl) {
  Data* d = (Data*)p;
  const rmbx_model* m = d->m;
  d->time = time;
  if (qpos) memcpy(d->qpos, qpos, sizeof(double) * m->nq);
  if (qvel) memcpy(d->qvel, qvel, sizeof(double) * m->nv);
  if (qacc_ws) memcpy(d->qacc_ws, qacc_ws, sizeof(double) * m->nv);
  if (ctrl) memcpy(d->ctrl, ctrl, sizeof(double) * m->nu);
}
void orc_get_state(void* p, double* time, double* qpos, double* qvel, double* qacc_ws) {
  Data* d = (Data*)p;
  const rmbx_model* m = d->m;
  if (time) *time = d->time;
  if (qpos) memcpy(qpos, d->qpos, sizeof(double) * m->nq);
  if (qvel) memcpy(qvel, d->qvel, sizeof(double) * m->nv);
  if (qacc_ws) memcpy(qacc_ws, d->qacc_ws, sizeof(double) * m->nv);
}
void orc_set_body_pos(void* p, int body, const double* pos) {
  Data* d = (Data*)p;
  memcpy(d->body_pos_env + 3 * body, pos, 3 * sizeof(double));
}
void orc_get_xpos(void* p, double* xpos, double* xquat) {
  Data* d = (Data*)p;
  if (xpos) memcpy(xpos, d->xpos, sizeof(double) * 3 * d->m->nbody);
  if (xquat) memcpy(xquat, d->xquat, sizeof(double) * 4 * d->m->nbody);
}
void orc_get_geom(void* p, double* gxpos, double* gxmat) {
  Data* d = (Data*)p;
  if (gxpos) memcpy(gxpos, d->gxpos, sizeof(double) * 3 * d->m->ngeom);
  if (gxmat) memcpy(gxmat, d->gxmat, sizeof(double) * 9 * d->m->ngeom);
}
void orc_get_sensor(void* p, double* out6) { memcpy(out6, ((Data*)p)->sensordata, sizeof(double) * 6); }
void orc_get_M(void* p, double* M) {
  Data* d = (Data*)p;
  memcpy(M, d->M, sizeof(double) * d->m->nv * d->m->nv);
}
void orc_get_vecs(void* p, double* bias, double* passive, double* actuator, double* constraint, double* qacc) {
  Data* d = (Data*)p;
  size_t n = sizeof(double) * d->m->nv;
  if (bias) memcpy(bias, d->qfrc_bias, n);
  if (passive) memcpy(passive, d->qfrc_passive, n);
  if (actuator) memcpy(actuator, d->qfrc_actuator, n);
  if (constraint) memcpy(constraint, d->qfrc_constraint, n);
  if (qacc) memcpy(qacc, d->qacc, n);
}
/* constraint Jacobian (dense, nefc x nv) and row weights D of the last forward / step */
void orc_get_efc(void* p, double* J, double* D) {
  Data* d = (Data*)p;
  if (J) memcpy(J, d->J, sizeof(double) * (size_t)d->nefc * d->m->nv);
  if (D) memcpy(D, d->efc_D, sizeof(double) * (size_t)d->nefc);
}
/* constraint forces of the last forward / step (row order as orc_get_efc): the active set is the
   rows with a nonzero force */
void orc_get_efc_force(void* p, double* force) {
  Data* d = (Data*)p;
  memcpy(force, d->efc_force, sizeof(double) * (size_t)d->nefc);
}
int orc_ncon(void* p) { return ((Data*)p)->ncon; }
int orc_nefc(void* p) { return ((Data*)p)->nefc; }
int orc_solver_iter(void* p) { return ((Data*)p)->solver_iter; }
/* the last solve's per-iteration stopping quantities (scaled gradient norm, scaled cost
   improvement; -1 where the iteration did not reach that test), 128 entries each */
void orc_get_solver_trace(void* p, double* grad, double* impr, double* kink) {
  Data* d = (Data*)p;
  memcpy(grad, d->trace_grad, sizeof(d->trace_grad));
  memcpy(impr, d->trace_impr, sizeof(d->trace_impr));
  if (kink) memcpy(kink, d->trace_kink, sizeof(d->trace_kink));
}
void orc_get_contacts(void* p, double* pos, double* frame, double* dist, int* pair) {
  Data* d = (Data*)p;
  int n = d->ncon;
  if (pos) memcpy(pos, d->con_pos, sizeof(double) * 3 * n);
  if (frame) memcpy(frame, d->con_frame, sizeof(double) * 9 * n);
  if (dist) memcpy(dist, d->con_dist, sizeof(double) * n);
  if (pair) memcpy(pair, d->con_pair, sizeof(int) * n);
}
