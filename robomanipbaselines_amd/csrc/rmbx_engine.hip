// Batched MuJoCo-subset physics for the rollout hot path (gfx950).
//
// Replaces the reference's per-env env.step -> gymnasium do_simulation -> mujoco.mj_step x 8
// (envs/mujoco/MujocoEnvBase.py:82-97, :12-13) for thousands of envs in lockstep.
//
// Execution model, per substep: front_kernel (ONE WAVEFRONT per env; lanes split the
// data-parallel stages -- bodies for the tree passes (pointer-jumping prefixes, DFS subtree
// ranges), geoms, pairs, contacts, constraint rows) then solver_kernel (256 threads per env: the
// nv x nv Newton Hessian / mass-matrix factorisations as 4x4 register blocks, one per thread of
// the lower triangle).  Between the two, per-env data lives in a workspace slice (mass matrix
// as packed lower 4x4 blocks, dof axes, contacts, row data); the constraint Jacobian is never
// materialised (see the ROW_* comment below).  Algorithm, stage for stage, is the one restated
// serially in oracle/dyn_oracle.c (see that header for the MuJoCo mapping).

#include <cstring>
#include <string>
#include <vector>

#include "rmbx_common.h"

#include <cstdlib>
#include "rmbx_math.h"
#include "rmbx_model.h"

namespace rmbx {

#define MAXCON_PAIR 8

// ------------------------------------------------------------------------------------------
// workspace layout (offsets in doubles within one env slice; ints stored in a trailing region)
// ------------------------------------------------------------------------------------------
struct Layout {
  size_t stride;  // doubles per env
  size_t xmat, xipos, xanchor, xaxis, sxpos, sxmat, cdof, cdofdot, cinert, crb, cvel, cacc, cfrc;
  size_t Mblk;  // mass matrix as packed lower-triangle 4x4 blocks (block t = bi(bi+1)/2 + bj)
  size_t qfrc_bias, qfrc_passive, qfrc_actuator, qfrc_smooth, qacc_smooth, qfrc_constraint, qacc,
      res, Mres, grad, search, Ms, tmp;
  size_t ten_len, ten_vel;
  size_t con_pos, con_frame, con_dist, con_mu;
  size_t con_tmp;  // collision stage: 4 candidate contacts (pos, normal, dist) per survivor
  size_t hsave;    // solver: Hessian blocks of the substep's full build (net-change updates)
  size_t efc_pos, efc_aref, efc_D, efc_sqD, efc_R, efc_force, efc_jar, efc_Js, efc_vel, efc_tmp;
  size_t efc_rho;  // contact rows: (p x dir, dir), J_r = efc_rho . (V_b2 - V_b1)
  size_t eqr_rho, eqr_coef;  // equality rows: 2 body-side 6-vectors, 2 dof coefficients
  size_t ints;  // start of the int32 region (in doubles)
  // int32 offsets relative to the int region
  size_t con_b1, con_b2, con_condim, con_pair, con_efcadr, efc_type, efc_act, efc_hact, efc_kind,
      efc_obj, eqr_body, eqr_dof, scal;
  size_t istride;  // int32 count
  int nefc_max;
  int neqr_max;  // equality rows (6 per weld)
};

// Constraint rows are never materialised as a dense Jacobian.  Row r is described by
// (efc_kind[r] = kind | sub << 3, efc_obj[r]):
//   ROW_CONTACT  obj = contact c, sub = pyramid edge t (0..3) or 4 (frictionless normal):
//                J_r = dir_t . (v_b2(p) - v_b1(p)), the relative velocity at the contact point,
//                = efc_rho . (V_b2 - V_b1) with efc_rho = (p x dir_t, dir_t)
//   ROW_LIMIT    obj = dof, sub = 0 (+1) / 1 (-1)
//   ROW_EQ       obj = equality-row slot s: J_r = sum over the two sides of
//                [dof on chain(eqr_body)] cdof . eqr_rho + the dof terms (eqr_dof, eqr_coef)
// so J x is a tree pass (body velocities of x) plus one 6-dot per row, J^T w a pass of body
// wrenches summed over subtrees, and a Hessian chunk is computed from cdof in LDS.
enum { ROW_CONTACT = 0, ROW_LIMIT = 1, ROW_EQ = 2 };

struct rmbx_engine_impl;

}  // namespace rmbx

struct rmbx_engine {
  rmbx_model host;       // copy of scalars (pointers unused)
  rmbx_model dev;        // device pointers
  const int32_t* subtree_end;  // device [nbody]: DFS subtree ranges for the tree passes
  int tree_rounds;             // ceil(log2(max body depth + 1)) (solver pointer jumping)
  const double* hBblk;         // device: h * (damping + actuator velocity gains), packed 4x4 blocks
  // two-level broadphase (models with long runs of same-body-pair geom pairs, e.g. the Pick
  // scene's convex-hull meshes): nprun = 0 disables it
  int nprun;
  const int32_t* prun_start;   // device [nprun + 1]: pair range of each run
  const int32_t* prun_body;    // device [nprun][2]: the run's two bodies
  const double* prun_margin;   // device [nprun]: largest pair margin of the run
  const int32_t* body_cgeom;   // device [nbody][2]: first collision geom, count
  std::vector<void*> allocations;
  rmbx::Layout L;
  int n_env;
  rmbx_env_buffers bufs;
  bool bound;
  size_t front_lds;  // dynamic LDS of a front-kernel launch (front_launch_lds)
  int solver_minb;   // solver blocks per CU of this batch size (solver_minb_for)
};

namespace rmbx {

struct Env {
  const rmbx_model* m;
  double* ws;
  int32_t* iw;
  const Layout* L;
  double* qpos;
  double* qvel;
  double* qacc_ws;
  double* ctrl;
  double* body_pos;
  double* xpos;
  double* xquat;
  double* gxpos;
  double* gxmat;
  double* sensordata;
  double* time;
  int32_t* stats;
  double* sh;  // front-kernel LDS: xpos, xquat, xmat, cvel, cacc, cfrc, cdofdot
  const int32_t* subtree_end;  // DFS subtree ranges (tree passes, chain membership)
};

#define W(name) (e.ws + e.L->name)
#define WI(name) (e.iw + e.L->name)

__device__ __forceinline__ void sync() { __syncthreads(); }
// Block barrier for LDS traffic only (the CK block_sync_lds idiom): waits for this wave's LDS
// and scalar-memory operations, then s_barrier.  __syncthreads() is a workgroup fence as well and
// drains every outstanding global load and store (vmcnt(0)) -- ~1-2k cycles after a global store
// -- so it stays only where threads hand data to each other through global memory.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ unsigned long long stamp() { return __builtin_readcyclecounter(); }
// diagnostic cycle slots per env: 0-7 stages, 8-15 solver, 16-19 collision, 20-23 constraints,
// 24-27 J^T w passes, 28-31 J x / M x passes
#define RMBX_PROF_SLOTS 32
#define SUBPROF(k)                                \
  if (prof) {                                     \
    __syncthreads();                              \
    const unsigned long long t_ = stamp();        \
    if (threadIdx.x == 0) prof[k] += t_ - tp;     \
    tp = t_;                                      \
  }

// ------------------------------------------------------------------------------------------
// Tree passes, lane = body (nbody <= 64).  Bodies are in DFS preorder, so a subtree is the id
// range [b, subtree_end[b]).  Root-to-leaf accumulations (frames, velocities, accelerations) are
// parallel prefix passes by pointer jumping (log2(depth) rounds instead of a depth-long serial
// chain); leaf-to-root accumulations are per-lane sums over the subtree range.  Every thread of
// the block calls these (barriers are block-wide); lanes >= nbody idle.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void anc_init(const rmbx_model& m, int* s_anc, int lane) {
  if (lane < m.nbody) s_anc[lane] = lane == 0 ? -1 : m.body_parent[lane];
  sync();
}

// X[6b..] <- sum of the increments X over the path world .. b (6-vectors in LDS)
__device__ void tree_prefix6(const rmbx_model& m, double* X, int* s_anc, int lane) {
  anc_init(m, s_anc, lane);
  const int b = lane;
  while (true) {
    const int a = b < m.nbody ? s_anc[b] : -1;
    const bool act = a >= 0;
    if (!__syncthreads_or(act)) break;
    double v[6];
    int an = -1;
    if (act) {
      for (int i = 0; i < 6; i++) v[i] = X[6 * a + i] + X[6 * b + i];
      an = s_anc[a];
    }
    sync();
    if (act) {
      for (int i = 0; i < 6; i++) X[6 * b + i] = v[i];
      s_anc[b] = an;
    }
    sync();
  }
}

// frames (P, Q) relative to the ancestor in s_anc -> world frames: T_b <- T_a o T_b
__device__ void tree_compose(const rmbx_model& m, double* P, double* Q, int* s_anc, int lane) {
  anc_init(m, s_anc, lane);
  const int b = lane;
  while (true) {
    const int a = b < m.nbody ? s_anc[b] : -1;
    const bool act = a >= 0;
    if (!__syncthreads_or(act)) break;
    double q[4], p[3];
    int an = -1;
    if (act) {
      double R[9], t[3];
      quatmul(Q + 4 * a, Q + 4 * b, q);
      quat2mat(Q + 4 * a, R);
      matvec3(R, P + 3 * b, t);
      for (int i = 0; i < 3; i++) p[i] = P[3 * a + i] + t[i];
      an = s_anc[a];
    }
    sync();
    if (act) {
      for (int i = 0; i < 4; i++) Q[4 * b + i] = q[i];
      for (int i = 0; i < 3; i++) P[3 * b + i] = p[i];
      s_anc[b] = an;
    }
    sync();
  }
}

// ------------------------------------------------------------------------------------------
// kinematics (mj_kinematics): each lane builds its body's frame in the parent frame (body offset
// and its joints, the hinge sin/cos included), one prefix pass composes the world frames, then
// joint anchors/axes, inertial frames, geoms and sites in parallel
// ------------------------------------------------------------------------------------------
__device__ void kinematics(Env& e, int lane, int* s_anc) {
  const rmbx_model& m = *e.m;
  const int nb = m.nbody;
  double* sx = e.sh;            // xpos  [3 nb]
  double* sq = sx + 3 * nb;     // xquat [4 nb]
  double* sm = sq + 4 * nb;     // xmat  [9 nb]
  double* xipos = W(xipos);
  double* xanchor = W(xanchor);
  double* xaxis = W(xaxis);
  const int b = lane;
  bool free_body = false;
  if (b < nb) {
    double P[3] = {0, 0, 0}, Q[4] = {1, 0, 0, 0};
    if (b > 0) {
      const int ja = m.body_jntadr[b], jn = m.body_jntnum[b];
      if (jn > 0 && m.jnt_type[ja] == RMBX_JNT_FREE) {
        free_body = true;  // child of the world: local frame = world frame
        const int a = m.jnt_qposadr[ja];
        for (int i = 0; i < 3; i++) P[i] = e.qpos[a + i];
        for (int i = 0; i < 4; i++) Q[i] = e.qpos[a + 3 + i];
        quatnorm(Q);
        for (int i = 0; i < 3; i++) xanchor[3 * ja + i] = P[i];
        xaxis[3 * ja] = 0;
        xaxis[3 * ja + 1] = 0;
        xaxis[3 * ja + 2] = 1;
      } else {
        for (int i = 0; i < 3; i++) P[i] = e.body_pos[3 * b + i];
        for (int i = 0; i < 4; i++) Q[i] = m.body_quat[4 * b + i];
        for (int j = ja; j < ja + jn; j++) {
          double R[9], t[3], anc[3], ax[3];
          quat2mat(Q, R);
          matvec3(R, m.jnt_pos + 3 * j, t);
          for (int i = 0; i < 3; i++) anc[i] = P[i] + t[i];
          matvec3(R, m.jnt_axis + 3 * j, ax);
          for (int i = 0; i < 3; i++) {  // parent-frame anchor/axis; made world below
            xanchor[3 * j + i] = anc[i];
            xaxis[3 * j + i] = ax[i];
          }
          const int qa = m.jnt_qposadr[j];
          const double qd = e.qpos[qa] - m.qpos0[qa];
          if (m.jnt_type[j] == RMBX_JNT_HINGE) {
            double qr[4];
            axisangle_quat(m.jnt_axis + 3 * j, qd, qr);
            quatmul(Q, qr, Q);
            quatnorm(Q);
            quat2mat(Q, R);
            matvec3(R, m.jnt_pos + 3 * j, t);
            for (int i = 0; i < 3; i++) P[i] = anc[i] - t[i];
          } else if (m.jnt_type[j] == RMBX_JNT_SLIDE) {
            for (int i = 0; i < 3; i++) P[i] += ax[i] * qd;
          }
        }
      }
    }
    for (int i = 0; i < 3; i++) sx[3 * b + i] = P[i];
    for (int i = 0; i < 4; i++) sq[4 * b + i] = Q[i];
  }
  sync();
  tree_compose(m, sx, sq, s_anc, lane);
  if (b < nb) quat2mat(sq + 4 * b, sm + 9 * b);
  sync();
  if (b > 0 && b < nb) {
    const int p = m.body_parent[b];
    if (!free_body) {
      for (int j = m.body_jntadr[b]; j < m.body_jntadr[b] + m.body_jntnum[b]; j++) {
        double t[3], ax[3];
        matvec3(sm + 9 * p, xanchor + 3 * j, t);
        matvec3(sm + 9 * p, xaxis + 3 * j, ax);
        for (int i = 0; i < 3; i++) {
          xanchor[3 * j + i] = sx[3 * p + i] + t[i];
          xaxis[3 * j + i] = ax[i];
        }
      }
    }
    double t[3];
    matvec3(sm + 9 * b, m.body_ipos + 3 * b, t);
    for (int i = 0; i < 3; i++) xipos[3 * b + i] = sx[3 * b + i] + t[i];
  }
  sync();
  for (int k = lane; k < 3 * nb; k += 64) e.xpos[k] = sx[k];
  for (int k = lane; k < 4 * nb; k += 64) e.xquat[k] = sq[k];
  for (int k = lane; k < 9 * nb; k += 64) W(xmat)[k] = sm[k];
  const double* xmat = sm;
  sync();
  for (int g = lane; g < m.ngeom; g += 64) {
    const int b = m.geom_body[g];
    const bool col = m.geom_ctype[g] >= 0;
    const double* gp = col ? m.geom_cpos + 3 * g : m.geom_pos + 3 * g;
    const double* gq = col ? m.geom_cquat + 4 * g : m.geom_quat + 4 * g;
    double t[3], R[9];
    matvec3(xmat + 9 * b, gp, t);
    for (int i = 0; i < 3; i++) e.gxpos[3 * g + i] = sx[3 * b + i] + t[i];
    quat2mat(gq, R);
    matmul3(xmat + 9 * b, R, e.gxmat + 9 * g);
  }
  for (int s = lane; s < m.nsite; s += 64) {
    const int b = m.site_body[s];
    double t[3], R[9];
    matvec3(xmat + 9 * b, m.site_pos + 3 * s, t);
    for (int i = 0; i < 3; i++) W(sxpos)[3 * s + i] = sx[3 * b + i] + t[i];
    quat2mat(m.site_quat + 4 * s, R);
    matmul3(xmat + 9 * b, R, W(sxmat) + 9 * s);
  }
}

// ------------------------------------------------------------------------------------------
// mj_comPos + mj_crb
// ------------------------------------------------------------------------------------------
// front-kernel LDS map (doubles): xpos 3nb | xquat 4nb | xmat 9nb | cvel 6nb | cacc 6nb |
// cfrc 6nb | cdofdot 6nv | cinert 10nb | cdof 6nv | crb 10nb
__host__ __device__ __forceinline__ size_t front_lds_doubles(int nb, int nv) { return 54 * (size_t)nb + 12 * (size_t)nv; }
// front kernel LDS: [0, 16 nb) xpos / xquat / xmat (live to the end); [16 nb, 34 nb + 6 nv) cvel,
// cacc, cfrc, cdofdot; cinert [10 nb]; crb [10 nb] (dead once the mass matrix is written); cdof
// [6 nv] -- all of [16 nb, ...) dead after the velocity stage and reused by the collision stage
#define LDS_CINERT(e) ((e).sh + 34 * (e).m->nbody + 6 * (e).m->nv)
#define LDS_CRB(e) (LDS_CINERT(e) + 10 * (e).m->nbody)
#define LDS_CDOF(e) (LDS_CRB(e) + 10 * (e).m->nbody)

__device__ void com_pos_crb(Env& e, int lane, const int32_t* subtree_end) {
  const rmbx_model& m = *e.m;
  const int nv = m.nv, nb = m.nbody;
  double* cinert = LDS_CINERT(e);
  double* cdof = LDS_CDOF(e);
  double* crb = LDS_CRB(e);
  for (int b = lane; b < nb; b += 64) {
    double* I = cinert + 10 * b;
    if (b == 0) {
      for (int k = 0; k < 10; k++) I[k] = 0;
      continue;
    }
    const double mass = m.body_mass[b];
    const double* c = W(xipos) + 3 * b;
    const double* R = e.sh + 7 * nb + 9 * b;  // xmat (LDS)
    const double* Ib = m.body_inertia + 9 * b;
    double T[9], Iw[9], Rt[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) Rt[3 * i + j] = R[3 * j + i];
    matmul3(R, Ib, T);
    matmul3(T, Rt, Iw);
    const double cc = dot3(c, c);
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
  for (int j = lane; j < m.njnt; j += 64) {
    const int b = m.jnt_body[j], da = m.jnt_dofadr[j];
    const double* ax = W(xaxis) + 3 * j;
    const double* anc = W(xanchor) + 3 * j;
    double* S = cdof + 6 * da;
    const int t = m.jnt_type[j];
    if (t == RMBX_JNT_HINGE) {
      S[0] = ax[0];
      S[1] = ax[1];
      S[2] = ax[2];
      cross3(anc, ax, S + 3);
    } else if (t == RMBX_JNT_SLIDE) {
      S[0] = S[1] = S[2] = 0;
      S[3] = ax[0];
      S[4] = ax[1];
      S[5] = ax[2];
    } else if (t == RMBX_JNT_FREE) {
      for (int k = 0; k < 36; k++) S[k] = 0;
      S[3] = 1;
      S[10] = 1;
      S[17] = 1;
      const double* R = e.sh + 7 * nb + 9 * b;
      const double* x = e.sh + 3 * b;
      for (int k = 0; k < 3; k++) {
        double* Sk = S + 6 * (3 + k);
        const double a[3] = {R[k], R[3 + k], R[6 + k]};
        Sk[0] = a[0];
        Sk[1] = a[1];
        Sk[2] = a[2];
        cross3(x, a, Sk + 3);
      }
    }
  }
  sync();
  // composite rigid-body inertia = subtree sums (DFS ranges), copies for the solver kernel
  // (exact range sums: a prefix-difference scan would cost ~1e-12 relative on the light links)
  for (int b = lane; b < nb; b += 64) {
    double acc[10];
    for (int k = 0; k < 10; k++) acc[k] = cinert[10 * b + k];
    if (b > 0)
      for (int d = b + 1; d < subtree_end[b]; d++)
        for (int k = 0; k < 10; k++) acc[k] += cinert[10 * d + k];
    for (int k = 0; k < 10; k++) crb[10 * b + k] = acc[k];
  }
  for (int k = lane; k < 10 * nb; k += 64) W(cinert)[k] = cinert[k];
  for (int k = lane; k < 6 * nv; k += 64) W(cdof)[k] = cdof[k];
  sync();
  // lower triangle, lane = row i: M_ij = cdof_j . (crb_body(i) cdof_i) for dofs j on i's chain,
  // written straight into the packed 4x4 blocks the solver loads (zeros off the chain; the
  // upper half of a diagonal block is never read; padding rows get the identity)
  // (lane per row: F_i = crb_body(i) cdof_i into the velocity stage's not yet used LDS; then
  // lane per block, so the triangle's 153 blocks spread evenly over the lanes)
  double* Mb = W(Mblk);
  const int NB = (nv + 3) / 4;
  double* Fr = e.sh + 16 * nb;  // [6 nv] (cvel/cacc region: free until velocity_stage)
  for (int i = lane; i < nv; i += 64) inert_mul(crb + 10 * m.dof_body[i], cdof + 6 * i, Fr + 6 * i);
  sync();
  for (int t = lane; t < NB * (NB + 1) / 2; t += 64) {
    int bi, bj;
    {
      int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
      while ((r + 1) * (r + 2) / 2 <= t) r++;
      while (r * (r + 1) / 2 > t) r--;
      bi = r;
      bj = t - r * (r + 1) / 2;
    }
    double* dstb = Mb + 16 * (size_t)t;
#pragma unroll 1
    for (int p = 0; p < 4; p++) {
      double row[4];
      const int i = 4 * bi + p;
      const int bi_ = i < nv ? m.dof_body[i] : 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int c = 4 * bj + q;
        double v;
        if (i >= nv || c >= nv) {
          v = i == c ? 1.0 : 0.0;
        } else if (c > i) {
          v = 0.0;  // (upper half of a diagonal block: never read)
        } else {
          const int bc = m.dof_body[c];
          const bool anc = bc == bi_ || (bc < bi_ && bi_ < subtree_end[bc]);
          v = anc ? dot6(cdof + 6 * c, Fr + 6 * i) : 0.0;
          if (c == i) v += m.dof_armature[i];
        }
        row[q] = v;
      }
      double2* dst = reinterpret_cast<double2*>(dstb + 4 * p);
      dst[0] = make_double2(row[0], row[1]);
      dst[1] = make_double2(row[2], row[3]);
    }
  }
  sync();
}

// ------------------------------------------------------------------------------------------
// mj_comVel + mj_rne (bias) ; passive ; tendons ; actuation
// ------------------------------------------------------------------------------------------
// RNE forward pass, lane = body: cacc = prefix over the tree of the per-body increments
// (world: -gravity), cfrc = I cacc + cvel x* (I cvel).  cdof/cinert/cvel/cdofdot/qacc may be
// LDS or global; ca and cfrc are LDS [6 nb].
__device__ void rne_forward(const Env& e, const double* qacc, double* ca, double* cfrc, const double* cvel,
                            const double* cdofdot, const double* cdof, const double* cinert, int* s_anc,
                            int lane) {
  const rmbx_model& m = *e.m;
  const int b = lane;
  if (b == 0) {
    ca[0] = ca[1] = ca[2] = 0;
    ca[3] = -m.gravity[0];
    ca[4] = -m.gravity[1];
    ca[5] = -m.gravity[2];
  } else if (b < m.nbody) {
    double a[6] = {0, 0, 0, 0, 0, 0};
    const int da = m.body_dofadr[b], dn = m.body_dofnum[b];
    for (int k = da; k < da + dn; k++) {
      for (int i = 0; i < 6; i++) a[i] += cdofdot[6 * k + i] * e.qvel[k];
      if (qacc)
        for (int i = 0; i < 6; i++) a[i] += cdof[6 * k + i] * qacc[k];
    }
    for (int i = 0; i < 6; i++) ca[6 * b + i] = a[i];
  }
  sync();
  tree_prefix6(m, ca, s_anc, lane);
  if (b > 0 && b < m.nbody) {
    double Ia[6], Iv[6], vxIv[6];
    const double* I = cinert + 10 * b;
    const double* v = cvel + 6 * b;
    inert_mul(I, ca + 6 * b, Ia);
    inert_mul(I, v, Iv);
    cross_force(v, Iv, vxIv);
    for (int i = 0; i < 6; i++) cfrc[6 * b + i] = Ia[i] + vxIv[i];
  }
  sync();
}

// RNE backward pass: cfrc[b] <- sum over the subtree of b (b > 0), lane = body
__device__ void rne_backward(const rmbx_model& m, double* cfrc, const int32_t* subtree_end, int lane) {
  const int b = lane;
  double acc[6];
  const bool act = b > 0 && b < m.nbody;
  if (act) {
    for (int i = 0; i < 6; i++) acc[i] = cfrc[6 * b + i];
    for (int d = b + 1; d < subtree_end[b]; d++)
      for (int i = 0; i < 6; i++) acc[i] += cfrc[6 * d + i];
  }
  sync();
  if (act)
    for (int i = 0; i < 6; i++) cfrc[6 * b + i] = acc[i];
  sync();
}

__device__ void velocity_stage(Env& e, int lane, int* s_anc, const int32_t* subtree_end) {
  const rmbx_model& m = *e.m;
  const int nv = m.nv, nb = m.nbody;
  double* cvel = e.sh + 16 * nb;   // LDS
  double* scacc = cvel + 6 * nb;   // LDS
  double* scfrc = scacc + 6 * nb;  // LDS
  double* cdofdot = scfrc + 6 * nb;  // LDS [6 nv]
  const double* cdof = LDS_CDOF(e);
  const int b = lane;
  // body velocity increments, then the prefix over the tree
  if (b < nb) {
    double v[6] = {0, 0, 0, 0, 0, 0};
    if (b > 0)
      for (int k = m.body_dofadr[b]; k < m.body_dofadr[b] + m.body_dofnum[b]; k++)
        for (int i = 0; i < 6; i++) v[i] += cdof[6 * k + i] * e.qvel[k];
    for (int i = 0; i < 6; i++) cvel[6 * b + i] = v[i];
  }
  sync();
  tree_prefix6(m, cvel, s_anc, lane);
  // cdof_dot = (velocity before the dof) x cdof, per body in joint order
  if (b > 0 && b < nb) {
    double cv[6];
    for (int i = 0; i < 6; i++) cv[i] = cvel[6 * m.body_parent[b] + i];
    for (int j = m.body_jntadr[b]; j < m.body_jntadr[b] + m.body_jntnum[b]; j++) {
      const int da = m.jnt_dofadr[j];
      if (m.jnt_type[j] == RMBX_JNT_FREE) {
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) cdofdot[6 * (da + k) + i] = 0;
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) cv[i] += cdof[6 * (da + k) + i] * e.qvel[da + k];
        for (int k = 3; k < 6; k++) cross_motion(cv, cdof + 6 * (da + k), cdofdot + 6 * (da + k));
        for (int k = 3; k < 6; k++)
          for (int i = 0; i < 6; i++) cv[i] += cdof[6 * (da + k) + i] * e.qvel[da + k];
      } else {
        cross_motion(cv, cdof + 6 * da, cdofdot + 6 * da);
        for (int i = 0; i < 6; i++) cv[i] += cdof[6 * da + i] * e.qvel[da];
      }
    }
  }
  sync();
  rne_forward(e, nullptr, scacc, scfrc, cvel, cdofdot, cdof, LDS_CINERT(e), s_anc, lane);
  rne_backward(m, scfrc, subtree_end, lane);
  for (int k = lane; k < 6 * nb; k += 64) W(cvel)[k] = cvel[k];
  for (int k = lane; k < 6 * nv; k += 64) W(cdofdot)[k] = cdofdot[k];
  double* bias = W(qfrc_bias);
  double* passive = W(qfrc_passive);
  for (int k = lane; k < nv; k += 64) {
    bias[k] = dot6(cdof + 6 * k, scfrc + 6 * m.dof_body[k]);
    passive[k] = -m.dof_damping[k] * e.qvel[k];
  }
  sync();
  for (int j = lane; j < m.njnt; j += 64) {
    if (m.jnt_stiffness[j] != 0 &&
        (m.jnt_type[j] == RMBX_JNT_HINGE || m.jnt_type[j] == RMBX_JNT_SLIDE)) {
      passive[m.jnt_dofadr[j]] -= m.jnt_stiffness[j] * (e.qpos[m.jnt_qposadr[j]] - m.jnt_springref[j]);
    }
  }
  double* act = W(qfrc_actuator);
  for (int k = lane; k < nv; k += 64) act[k] = 0;
  sync();
  if (lane == 0) {
    double* tl = W(ten_len);
    double* tv = W(ten_vel);
    for (int t = 0; t < m.ntendon; t++) {
      double L = 0, V = 0;
      for (int w = m.ten_adr[t]; w < m.ten_adr[t] + m.ten_num[t]; w++) {
        const int j = m.wrap_jnt[w];
        L += m.wrap_coef[w] * e.qpos[m.jnt_qposadr[j]];
        V += m.wrap_coef[w] * e.qvel[m.jnt_dofadr[j]];
      }
      tl[t] = L;
      tv[t] = V;
    }
    for (int u = 0; u < m.nu; u++) {
      double c = e.ctrl[u];
      if (m.act_ctrllimited[u]) {
        c = c < m.act_ctrlrange[2 * u] ? m.act_ctrlrange[2 * u] : c;
        c = c > m.act_ctrlrange[2 * u + 1] ? m.act_ctrlrange[2 * u + 1] : c;
      }
      const int id = m.act_trnid[u];
      double len, vel;
      if (m.act_trntype[u] == RMBX_TRN_JOINT) {
        len = e.qpos[m.jnt_qposadr[id]];
        vel = e.qvel[m.jnt_dofadr[id]];
      } else {
        len = tl[id];
        vel = tv[id];
      }
      const double* bp = m.act_bias + 3 * u;
      double f = m.act_gain[u] * c + bp[0] + bp[1] * len + bp[2] * vel;
      if (m.act_forcelimited[u]) {
        f = f < m.act_forcerange[2 * u] ? m.act_forcerange[2 * u] : f;
        f = f > m.act_forcerange[2 * u + 1] ? m.act_forcerange[2 * u + 1] : f;
      }
      if (m.act_trntype[u] == RMBX_TRN_JOINT) {
        act[m.jnt_dofadr[id]] += f;
      } else {
        for (int w = m.ten_adr[id]; w < m.ten_adr[id] + m.ten_num[id]; w++)
          act[m.jnt_dofadr[m.wrap_jnt[w]]] += m.wrap_coef[w] * f;
      }
    }
  }
  sync();
  double* sm = W(qfrc_smooth);
  for (int k = lane; k < nv; k += 64) sm[k] = passive[k] + act[k] - bias[k];
  sync();
}

// ------------------------------------------------------------------------------------------
// collision: lanes over candidate pairs, deterministic wave-scan compaction (pair order)
// ------------------------------------------------------------------------------------------
struct Contact {
  double pos[3], n[3], dist;
};

__device__ void closest_seg_seg(const double* p1, const double* q1, const double* p2,
                                const double* q2, double* c1, double* c2) {
  double d1[3], d2[3], r[3];
  for (int i = 0; i < 3; i++) {
    d1[i] = q1[i] - p1[i];
    d2[i] = q2[i] - p2[i];
    r[i] = p1[i] - p2[i];
  }
  const double a = dot3(d1, d1), ee = dot3(d2, d2), f = dot3(d2, r);
  double s, t;
  if (a <= RMBX_MINVAL && ee <= RMBX_MINVAL) {
    s = t = 0;
  } else if (a <= RMBX_MINVAL) {
    s = 0;
    t = fmin(fmax(f / ee, 0.0), 1.0);
  } else {
    const double c = dot3(d1, r);
    if (ee <= RMBX_MINVAL) {
      t = 0;
      s = fmin(fmax(-c / a, 0.0), 1.0);
    } else {
      const double b = dot3(d1, d2);
      const double den = a * ee - b * b;
      s = den > RMBX_MINVAL ? fmin(fmax((b * f - c * ee) / den, 0.0), 1.0) : 0.0;
      t = (b * s + f) / ee;
      if (t < 0) {
        t = 0;
        s = fmin(fmax(-c / a, 0.0), 1.0);
      } else if (t > 1) {
        t = 1;
        s = fmin(fmax((b - c) / a, 0.0), 1.0);
      }
    }
  }
  for (int i = 0; i < 3; i++) {
    c1[i] = p1[i] + d1[i] * s;
    c2[i] = p2[i] + d2[i] * t;
  }
}

__device__ int col_sphere_sphere(const double* ca, double ra, const double* cb, double rb,
                                 double margin, Contact* out) {
  const double v[3] = {cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2]};
  const double l = norm3(v);
  const double dist = l - ra - rb;
  if (dist >= margin) return 0;
  double n[3];
  if (l < RMBX_MINVAL) {
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

__device__ __forceinline__ void capsule_ends(const double* c, const double* R, double h, double* p,
                                             double* q) {
  for (int i = 0; i < 3; i++) {
    p[i] = c[i] - R[3 * i + 2] * h;
    q[i] = c[i] + R[3 * i + 2] * h;
  }
}

__device__ double point_box(const double* p, const double* cb, const double* Rb, const double* hb,
                            double* n, double* surf) {
  const double dlt[3] = {p[0] - cb[0], p[1] - cb[1], p[2] - cb[2]};
  double l[3], q[3];
  mattvec3(Rb, dlt, l);
  bool inside = true;
  for (int i = 0; i < 3; i++) {
    q[i] = l[i] < -hb[i] ? -hb[i] : (l[i] > hb[i] ? hb[i] : l[i]);
    if (q[i] != l[i]) inside = false;
  }
  double nl[3], dist;
  if (!inside) {
    const double v[3] = {l[0] - q[0], l[1] - q[1], l[2] - q[2]};
    dist = norm3(v);
    nl[0] = v[0] / dist;
    nl[1] = v[1] / dist;
    nl[2] = v[2] / dist;
  } else {
    int k = 0;
    double best = hb[0] - fabs(l[0]);
    for (int i = 1; i < 3; i++) {
      const double pen = hb[i] - fabs(l[i]);
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

__device__ int col_sphere_box(const double* cs, double r, const double* cb, const double* Rb,
                              const double* hb, double margin, Contact* out) {
  double n[3], surf[3];
  const double dist = point_box(cs, cb, Rb, hb, n, surf) - r;
  if (dist >= margin) return 0;
  for (int i = 0; i < 3; i++) {
    out->n[i] = -n[i];
    out->pos[i] = surf[i] + n[i] * (0.5 * dist);
  }
  out->dist = dist;
  return 1;
}

__device__ int col_capsule_box(const double* ca, const double* Ra, const double* sa,
                               const double* cb, const double* Rb, const double* hb, double margin,
                               Contact* out) {
  double p[3], q[3];
  capsule_ends(ca, Ra, sa[1], p, q);
  Contact c0, c1, cm;
  const int h0 = col_sphere_box(p, sa[0], cb, Rb, hb, margin, &c0);
  const int h1 = col_sphere_box(q, sa[0], cb, Rb, hb, margin, &c1);
  double lo = 0, hi = 1;
  for (int it = 0; it < 40; it++) {
    const double t1 = lo + (hi - lo) / 3, t2 = hi - (hi - lo) / 3;
    double x1[3], x2[3], nn[3], ss[3];
    for (int i = 0; i < 3; i++) {
      x1[i] = p[i] + (q[i] - p[i]) * t1;
      x2[i] = p[i] + (q[i] - p[i]) * t2;
    }
    const double f1 = point_box(x1, cb, Rb, hb, nn, ss), f2 = point_box(x2, cb, Rb, hb, nn, ss);
    if (f1 < f2)
      hi = t2;
    else
      lo = t1;
  }
  const double tm = 0.5 * (lo + hi);
  double xm[3];
  for (int i = 0; i < 3; i++) xm[i] = p[i] + (q[i] - p[i]) * tm;
  const int hm = col_sphere_box(xm, sa[0], cb, Rb, hb, margin, &cm);
  if (h0 && h1) {
    out[0] = c0;
    out[1] = c1;
    return 2;
  }
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

// Candidate order for the multi-point contact routines: depth quantised to 1 nm, so candidates of
// a face-face configuration (equal depth up to rounding) keep their generation order and the
// selected points do not jump under last-bit changes of the geometry.
__device__ __forceinline__ bool contact_deeper(const Contact* a, const Contact* b) {
  return floor(a->dist * 1e9) < floor(b->dist * 1e9);
}

constexpr double BOX_INSIDE_TOL = 1e-9;  // m

__device__ int col_box_box(const double* ca, const double* Ra, const double* ha, const double* cb,
                           const double* Rb, const double* hb, double margin, Contact* out) {
  // the 15 separating-axis candidates, each formed when it is needed (a [15][3] table here, with
  // the 16-contact table below, was most of the front kernel's 1,920 B of private scratch per
  // lane): A's and B's face axes, then the normalised edge cross products (zero when parallel)
  auto axis = [&](int k, double* a) {
    if (k < 6) {
      const double* R = k < 3 ? Ra : Rb;
      const int c = k < 3 ? k : k - 3;
      a[0] = R[c];
      a[1] = R[3 + c];
      a[2] = R[6 + c];
      return;
    }
    const int i = (k - 6) / 3, j = (k - 6) - 3 * i;
    const double ai[3] = {Ra[i], Ra[3 + i], Ra[6 + i]}, bj[3] = {Rb[j], Rb[3 + j], Rb[6 + j]};
    double c[3];
    cross3(ai, bj, c);
    const double l = norm3(c);
    if (l < 1e-6) {
      a[0] = a[1] = a[2] = 0;
    } else {
      a[0] = c[0] / l;
      a[1] = c[1] / l;
      a[2] = c[2] / l;
    }
  };
  const double dc[3] = {cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2]};
  double best = -1e300;
  int bk = -1;
  for (int k = 0; k < 15; k++) {
    double a[3];
    axis(k, a);
    if (a[0] == 0 && a[1] == 0 && a[2] == 0) continue;
    double ra = 0, rb = 0;
    for (int i = 0; i < 3; i++) {
      const double ua[3] = {Ra[i], Ra[3 + i], Ra[6 + i]}, ub[3] = {Rb[i], Rb[3 + i], Rb[6 + i]};
      ra += ha[i] * fabs(dot3(a, ua));
      rb += hb[i] * fabs(dot3(a, ub));
    }
    const double sep = fabs(dot3(dc, a)) - ra - rb;
    if (sep >= margin) return 0;
    // B's face axes yield to A's within 1e-12 m (parallel faces tie up to rounding), edge axes
    // to faces within 1 um
    const double score = k < 3 ? sep : (k < 6 ? sep - 1e-12 : sep - 1e-6);
    if (score > best) {
      best = score;
      bk = k;
    }
  }
  if (bk < 0) return 0; /* non-finite geometry (a diverged env): no axis scored */
  double n[3];
  axis(bk, n);
  if (dot3(n, dc) < 0) {
    n[0] = -n[0];
    n[1] = -n[1];
    n[2] = -n[2];
  }
  // contact candidates: each vertex of one box inside the other, kept as (depth, side << 3 | vertex);
  // the four deepest are rebuilt from their vertex by the same arithmetic below
  double cdist[16];
  uint8_t ccode[16];
  int nc = 0;
  for (int side = 0; side < 2; side++) {
    const double* c = side == 0 ? cb : ca;
    const double* R = side == 0 ? Rb : Ra;
    const double* h = side == 0 ? hb : ha;
    const double* co = side == 0 ? ca : cb;
    const double* Ro = side == 0 ? Ra : Rb;
    const double* ho = side == 0 ? ha : hb;
    for (int v = 0; v < 8; v++) {
      const double l[3] = {(v & 1) ? h[0] : -h[0], (v & 2) ? h[1] : -h[1], (v & 4) ? h[2] : -h[2]};
      double w[3];
      matvec3(R, l, w);
      const double x[3] = {c[0] + w[0], c[1] + w[1], c[2] + w[2]};
      const double dl[3] = {x[0] - co[0], x[1] - co[1], x[2] - co[2]};
      double lo[3];
      mattvec3(Ro, dl, lo);
      // a vertex within BOX_INSIDE_TOL of a face plane counts as inside (aligned equal faces, e.g.
      // the gripper pads closing on each other, keep one manifold whatever their last bits)
      const double tol = margin + BOX_INSIDE_TOL;
      if (fabs(lo[0]) > ho[0] + tol || fabs(lo[1]) > ho[1] + tol || fabs(lo[2]) > ho[2] + tol)
        continue;
      double sup = 0;
      for (int i = 0; i < 3; i++) {
        const double u[3] = {Ro[i], Ro[3 + i], Ro[6 + i]};
        sup += ho[i] * fabs(dot3(n, u));
      }
      const double dist = side == 0 ? (dot3(dl, n) - sup) : (-dot3(dl, n) - sup);
      if (dist >= margin) continue;
      if (nc < 16) {
        cdist[nc] = dist;
        ccode[nc] = (uint8_t)(side << 3 | v);
        ++nc;
      }
    }
  }
  if (nc == 0) {
    double pa[3], pb[3];
    const double neg[3] = {-n[0], -n[1], -n[2]};
    for (int i = 0; i < 3; i++) {
      pa[i] = ca[i];
      pb[i] = cb[i];
    }
    int fa = -1, fb = -1, nfa = 0, nfb = 0;  // the box axes parallel to the contact plane
    for (int k = 0; k < 3; k++) {
      const double ua[3] = {Ra[k], Ra[3 + k], Ra[6 + k]}, ub[3] = {Rb[k], Rb[3 + k], Rb[6 + k]};
      // support coordinate along each box axis: the extent's end facing the other box, or its
      // centre when the axis is perpendicular to n within 1e-9 (a face or edge parallel to the
      // contact plane: every point along it is a support point, and the sign of a ~1e-17 dot
      // product would pick an end by rounding -- the engine and the oracle then put the contact
      // a half extent apart)
      const double da = dot3(ua, n), db = dot3(ub, neg);
      const bool pa_free = fabs(da) < 1e-9, pb_free = fabs(db) < 1e-9;
      const double sa2 = pa_free ? 0.0 : (da > 0 ? ha[k] : -ha[k]);
      const double sb2 = pb_free ? 0.0 : (db > 0 ? hb[k] : -hb[k]);
      if (pa_free) { fa = k; ++nfa; }
      if (pb_free) { fb = k; ++nfb; }
      for (int i = 0; i < 3; i++) {
        pa[i] += ua[i] * sa2;
        pb[i] += ub[i] * sb2;
      }
    }
    const double dist = dot3(n, pb) - dot3(n, pa);
    if (dist >= margin) return 0;
    if (nfa == 1 && nfb == 1) {
      // edge against edge: the closest points of the two support edges (segments pa + s ua,
      // |s| <= ha, and pb + t ub, |t| <= hb; both lie in planes normal to n), clamped to the
      // segments -- for crossed edges the contact sits where they cross, not at their centres
      const double ua[3] = {Ra[fa], Ra[3 + fa], Ra[6 + fa]}, ub[3] = {Rb[fb], Rb[3 + fb], Rb[6 + fb]};
      const double w[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
      const double b = dot3(ua, ub), d = dot3(ua, w), e = dot3(ub, w);
      const double den = 1.0 - b * b;
      if (den > 1e-12) {  // (parallel edges keep the centres)
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
  // the exchange sort by quantised depth (contact_deeper) of the oracle, on (depth, code) pairs
  for (int i = 0; i < nc; i++)
    for (int j = i + 1; j < nc; j++)
      if (floor(cdist[j] * 1e9) < floor(cdist[i] * 1e9)) {
        const double t = cdist[i];
        cdist[i] = cdist[j];
        cdist[j] = t;
        const uint8_t tc = ccode[i];
        ccode[i] = ccode[j];
        ccode[j] = tc;
      }
  const int k = nc < 4 ? nc : 4;
  for (int q = 0; q < k; q++) {
    const int side = ccode[q] >> 3, v = ccode[q] & 7;
    const double* c = side == 0 ? cb : ca;
    const double* R = side == 0 ? Rb : Ra;
    const double* h = side == 0 ? hb : ha;
    const double l[3] = {(v & 1) ? h[0] : -h[0], (v & 2) ? h[1] : -h[1], (v & 4) ? h[2] : -h[2]};
    double w[3];
    matvec3(R, l, w);
    const double x[3] = {c[0] + w[0], c[1] + w[1], c[2] + w[2]};
    const double sgn = side == 0 ? 1.0 : -1.0;
    const double dist = cdist[q];
    out[q].dist = dist;
    for (int i = 0; i < 3; i++) {
      out[q].n[i] = n[i];
      out[q].pos[i] = x[i] - sgn * n[i] * (0.5 * dist);
    }
  }
  return k;
}

__device__ int col_plane(const double* cp, const double* Rp, int tb, const double* cb,
                         const double* Rb, const double* sb, double margin, Contact* out) {
  const double n[3] = {Rp[2], Rp[5], Rp[8]};
  double rad = 0;
  int np = 0;
  if (tb == RMBX_GEOM_SPHERE) {
    np = 1;
    rad = sb[0];
  } else if (tb == RMBX_GEOM_CAPSULE) {
    np = 2;
    rad = sb[0];
  } else if (tb == RMBX_GEOM_BOX) {
    np = 8;
  }
  // point k of the geom (the sphere's centre, the capsule's segment ends, the box's vertices),
  // formed where it is needed instead of held in a table (private scratch)
  auto point = [&](int k, double* p) {
    if (tb == RMBX_GEOM_SPHERE) {
      p[0] = cb[0];
      p[1] = cb[1];
      p[2] = cb[2];
    } else if (tb == RMBX_GEOM_CAPSULE) {
      double e0[3], e1[3];
      capsule_ends(cb, Rb, sb[1], e0, e1);
      for (int i = 0; i < 3; i++) p[i] = k == 0 ? e0[i] : e1[i];
    } else {
      const double l[3] = {(k & 1) ? sb[0] : -sb[0], (k & 2) ? sb[1] : -sb[1], (k & 4) ? sb[2] : -sb[2]};
      double w[3];
      matvec3(Rb, l, w);
      for (int i = 0; i < 3; i++) p[i] = cb[i] + w[i];
    }
  };
  double cdist[8];
  uint8_t ccode[8];
  int nc = 0;
  for (int k = 0; k < np; k++) {
    double p[3];
    point(k, p);
    const double v[3] = {p[0] - cp[0], p[1] - cp[1], p[2] - cp[2]};
    const double dist = dot3(v, n) - rad;
    if (dist >= margin) continue;
    cdist[nc] = dist;
    ccode[nc] = (uint8_t)k;
    ++nc;
  }
  for (int i = 0; i < nc; i++)
    for (int j = i + 1; j < nc; j++)
      if (floor(cdist[j] * 1e9) < floor(cdist[i] * 1e9)) {  // contact_deeper
        const double t = cdist[i];
        cdist[i] = cdist[j];
        cdist[j] = t;
        const uint8_t tc = ccode[i];
        ccode[i] = ccode[j];
        ccode[j] = tc;
      }
  const int k = nc < 4 ? nc : 4;
  for (int q = 0; q < k; q++) {
    double p[3];
    point(ccode[q], p);
    const double dist = cdist[q];
    out[q].dist = dist;
    for (int i = 0; i < 3; i++) {
      out[q].n[i] = n[i];
      out[q].pos[i] = p[i] - n[i] * (rad + 0.5 * dist);
    }
  }
  return k;
}

// Convex narrow phase: MPR (libccd's ccdMPRPenetration as MuJoCo 3.1.6's mjc_Convex calls it,
// [ext]) for pairs with a convex-hull mesh or a cylinder; the same algorithm and operation
// order as oracle/dyn_oracle.c (tolerance 1e-6, at most 50 refinement iterations, supports
// inflated by margin / 2, one contact: dist = margin - depth, normal from geom 1 to geom 2,
// position = the witness points' midpoint).  One lane per pair; the hull support is a serial
// scan of the hull's vertices (<= 64 for the scanned objects).
#define CCD_EPS 2.2204460492503131e-16
#define MPR_TOLERANCE 1e-6
#define MPR_ITERATIONS 50

struct ConvexObj {
  const double *c, *R, *s, *hv;
  int type, nhv;
  double margin;
};
struct SupportPt {
  double v[3], v1[3], v2[3];
};

__device__ __forceinline__ bool ccd_is_zero(double x) { return fabs(x) < CCD_EPS; }
__device__ __forceinline__ bool ccd_eq(double a, double b) {
  const double ab = fabs(a - b);
  if (ab < CCD_EPS) return true;
  const double fa = fabs(a), fb = fabs(b);
  return fb > fa ? ab < CCD_EPS * fb : ab < CCD_EPS * fa;
}
__device__ __forceinline__ bool vec_eq0(const double* a) {
  return ccd_eq(a[0], 0.0) && ccd_eq(a[1], 0.0) && ccd_eq(a[2], 0.0);
}
__device__ __forceinline__ void vec_normalize(double* v) {
  const double k = 1.0 / sqrt(dot3(v, v));
  v[0] *= k;
  v[1] *= k;
  v[2] *= k;
}
__device__ __forceinline__ double sgn0(double x) { return x < 0 ? -1.0 : (x > 0 ? 1.0 : 0.0); }

__device__ void convex_support(const ConvexObj& o, const double* dir, double* out) {
  double ld[3], res[3] = {0, 0, 0};
  mattvec3(o.R, dir, ld);
  const double* s = o.s;
  if (o.type == RMBX_GEOM_SPHERE || o.type == RMBX_GEOM_CAPSULE) {
    const double n = norm3(ld);
    if (n > RMBX_MINVAL)
      for (int i = 0; i < 3; i++) res[i] = ld[i] * (s[0] / n);
    if (o.type == RMBX_GEOM_CAPSULE) res[2] += sgn0(ld[2]) * s[1];
  } else if (o.type == RMBX_GEOM_CYLINDER) {
    const double n = sqrt(ld[0] * ld[0] + ld[1] * ld[1]);
    if (n > RMBX_MINVAL) {
      res[0] = ld[0] * (s[0] / n);
      res[1] = ld[1] * (s[0] / n);
    }
    res[2] = sgn0(ld[2]) * s[1];
  } else if (o.type == RMBX_GEOM_BOX) {
    for (int i = 0; i < 3; i++) res[i] = sgn0(ld[i]) * s[i];
  } else {
    int best = 0;
    double bd = -1e300;
    for (int k = 0; k < o.nhv; k++) {
      const double dd = dot3(o.hv + 3 * k, ld);
      if (dd > bd) {
        bd = dd;
        best = k;
      }
    }
    for (int i = 0; i < 3; i++) res[i] = o.hv[3 * best + i];
  }
  if (o.margin > 0) {
    const double n = norm3(ld);
    if (n > RMBX_MINVAL)
      for (int i = 0; i < 3; i++) res[i] += ld[i] * (0.5 * o.margin / n);
  }
  double w[3];
  matvec3(o.R, res, w);
  for (int i = 0; i < 3; i++) out[i] = o.c[i] + w[i];
}

__device__ void mpr_support(const ConvexObj& a, const ConvexObj& b, const double* dir, SupportPt& p) {
  const double nd[3] = {-dir[0], -dir[1], -dir[2]};
  convex_support(a, dir, p.v1);
  convex_support(b, nd, p.v2);
  for (int i = 0; i < 3; i++) p.v[i] = p.v1[i] - p.v2[i];
}

__device__ double point_segment_dist2(const double* P, const double* x0, const double* b, double* witness) {
  const double d[3] = {b[0] - x0[0], b[1] - x0[1], b[2] - x0[2]};
  const double a[3] = {x0[0] - P[0], x0[1] - P[1], x0[2] - P[2]};
  double t = -1.0 * dot3(a, d);
  t /= dot3(d, d);
  if (t < 0 || ccd_is_zero(t)) {
    for (int i = 0; i < 3; i++) witness[i] = x0[i];
  } else if (t > 1 || ccd_eq(t, 1.0)) {
    for (int i = 0; i < 3; i++) witness[i] = b[i];
  } else {
    for (int i = 0; i < 3; i++) witness[i] = d[i] * t + x0[i];
  }
  const double w[3] = {witness[0] - P[0], witness[1] - P[1], witness[2] - P[2]};
  return dot3(w, w);
}

__device__ double point_tri_dist2(const double* P, const double* x0, const double* B, const double* C,
                                  double* witness) {
  double d1[3], d2[3], a[3];
  for (int i = 0; i < 3; i++) {
    d1[i] = B[i] - x0[i];
    d2[i] = C[i] - x0[i];
    a[i] = x0[i] - P[i];
  }
  const double v = dot3(d1, d1), w = dot3(d2, d2), p = dot3(a, d1), q = dot3(a, d2), r = dot3(d1, d2);
  const double dd = w * v - r * r;
  double s, t;
  if (ccd_is_zero(dd)) {
    s = t = -1.0;
  } else {
    s = (q * r - w * p) / dd;
    t = (-s * r - q) / w;
  }
  if ((ccd_is_zero(s) || s > 0) && (ccd_eq(s, 1.0) || s < 1) && (ccd_is_zero(t) || t > 0) &&
      (ccd_eq(t, 1.0) || t < 1) && (ccd_eq(t + s, 1.0) || t + s < 1)) {
    for (int i = 0; i < 3; i++) witness[i] = x0[i] + d1[i] * s + d2[i] * t;
    const double e3[3] = {witness[0] - P[0], witness[1] - P[1], witness[2] - P[2]};
    return dot3(e3, e3);
  }
  double w2[3];
  double dist = point_segment_dist2(P, x0, B, witness);
  double dist2 = point_segment_dist2(P, x0, C, w2);
  if (dist2 < dist) {
    dist = dist2;
    for (int i = 0; i < 3; i++) witness[i] = w2[i];
  }
  dist2 = point_segment_dist2(P, B, C, w2);
  if (dist2 < dist) {
    dist = dist2;
    for (int i = 0; i < 3; i++) witness[i] = w2[i];
  }
  return dist;
}

__device__ void portal_dir(const SupportPt* pt, double* dir) {
  double v2v1[3], v3v1[3];
  for (int i = 0; i < 3; i++) {
    v2v1[i] = pt[2].v[i] - pt[1].v[i];
    v3v1[i] = pt[3].v[i] - pt[1].v[i];
  }
  cross3(v2v1, v3v1, dir);
  vec_normalize(dir);
}

__device__ bool portal_reach_tolerance(const SupportPt* pt, const SupportPt& v4, const double* dir) {
  const double dv1 = dot3(pt[1].v, dir), dv2 = dot3(pt[2].v, dir), dv3 = dot3(pt[3].v, dir), dv4 = dot3(v4.v, dir);
  double d1 = dv4 - dv1;
  const double d2 = dv4 - dv2, d3 = dv4 - dv3;
  d1 = d1 < d2 ? d1 : d2;
  d1 = d1 < d3 ? d1 : d3;
  return ccd_eq(d1, MPR_TOLERANCE) || d1 < MPR_TOLERANCE;
}

__device__ void expand_portal(SupportPt* pt, const SupportPt& v4) {
  double v4v0[3];
  cross3(v4.v, pt[0].v, v4v0);
  double dot = dot3(pt[1].v, v4v0);
  if (dot > 0) {
    dot = dot3(pt[2].v, v4v0);
    if (dot > 0)
      pt[1] = v4;
    else
      pt[3] = v4;
  } else {
    dot = dot3(pt[3].v, v4v0);
    if (dot > 0)
      pt[2] = v4;
    else
      pt[1] = v4;
  }
}

__device__ int discover_portal(const ConvexObj& a, const ConvexObj& b, SupportPt* pt) {
  double dir[3], va[3], vb[3];
  for (int i = 0; i < 3; i++) {
    pt[0].v1[i] = a.c[i];
    pt[0].v2[i] = b.c[i];
    pt[0].v[i] = pt[0].v1[i] - pt[0].v2[i];
  }
  if (vec_eq0(pt[0].v)) pt[0].v[0] += CCD_EPS * 10.0;
  for (int i = 0; i < 3; i++) dir[i] = -pt[0].v[i];
  vec_normalize(dir);
  mpr_support(a, b, dir, pt[1]);
  double dot = dot3(pt[1].v, dir);
  if (ccd_is_zero(dot) || dot < 0) return -1;
  cross3(pt[0].v, pt[1].v, dir);
  if (ccd_is_zero(dot3(dir, dir))) return vec_eq0(pt[1].v) ? 1 : 2;
  vec_normalize(dir);
  mpr_support(a, b, dir, pt[2]);
  dot = dot3(pt[2].v, dir);
  if (ccd_is_zero(dot) || dot < 0) return -1;
  for (int i = 0; i < 3; i++) {
    va[i] = pt[1].v[i] - pt[0].v[i];
    vb[i] = pt[2].v[i] - pt[0].v[i];
  }
  cross3(va, vb, dir);
  vec_normalize(dir);
  if (dot3(dir, pt[0].v) > 0) {
    const SupportPt t = pt[1];
    pt[1] = pt[2];
    pt[2] = t;
    for (int i = 0; i < 3; i++) dir[i] = -dir[i];
  }
  for (int guard = 0; guard < 1000; guard++) {
    mpr_support(a, b, dir, pt[3]);
    dot = dot3(pt[3].v, dir);
    if (ccd_is_zero(dot) || dot < 0) return -1;
    bool cont = false;
    cross3(pt[1].v, pt[3].v, va);
    dot = dot3(va, pt[0].v);
    if (dot < 0 && !ccd_is_zero(dot)) {
      pt[2] = pt[3];
      cont = true;
    }
    if (!cont) {
      cross3(pt[3].v, pt[2].v, va);
      dot = dot3(va, pt[0].v);
      if (dot < 0 && !ccd_is_zero(dot)) {
        pt[1] = pt[3];
        cont = true;
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

__device__ int refine_portal(const ConvexObj& a, const ConvexObj& b, SupportPt* pt) {
  double dir[3];
  SupportPt v4;
  for (int guard = 0; guard < 1000; guard++) {
    portal_dir(pt, dir);
    double dot = dot3(pt[1].v, dir);
    if (ccd_is_zero(dot) || dot > 0) return 0;
    mpr_support(a, b, dir, v4);
    dot = dot3(v4.v, dir);
    if (!(ccd_is_zero(dot) || dot > 0) || portal_reach_tolerance(pt, v4, dir)) return -1;
    expand_portal(pt, v4);
  }
  return -1;
}

__device__ void find_pos(const SupportPt* pt, double* pos) {
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
  const double inv = 1.0 / sum;
  double p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < 3; i++) {
      p1[i] += pt[k].v1[i] * bc[k];
      p2[i] += pt[k].v2[i] * bc[k];
    }
  for (int i = 0; i < 3; i++) pos[i] = (p1[i] * inv + p2[i] * inv) * 0.5;
}

__device__ bool mpr_penetration(const ConvexObj& a, const ConvexObj& b, double* depth, double* dir, double* pos) {
  SupportPt pt[4];
  const int res = discover_portal(a, b, pt);
  if (res < 0) return false;
  if (res == 1) {
    *depth = 0;
    dir[0] = dir[1] = dir[2] = 0;
    for (int i = 0; i < 3; i++) pos[i] = (pt[1].v1[i] + pt[1].v2[i]) * 0.5;
    return true;
  }
  if (res == 2) {
    for (int i = 0; i < 3; i++) {
      pos[i] = (pt[1].v1[i] + pt[1].v2[i]) * 0.5;
      dir[i] = pt[1].v[i];
    }
    *depth = sqrt(dot3(dir, dir));
    vec_normalize(dir);
    return true;
  }
  if (refine_portal(a, b, pt) < 0) return false;
  SupportPt v4;
  for (int it = 0;; it++) {
    double pd[3];
    portal_dir(pt, pd);
    mpr_support(a, b, pd, v4);
    if (portal_reach_tolerance(pt, v4, pd) || it > MPR_ITERATIONS) {
      const double zero[3] = {0, 0, 0};
      *depth = sqrt(point_tri_dist2(zero, pt[1].v, pt[2].v, pt[3].v, dir));
      if (ccd_is_zero(*depth))
        dir[0] = dir[1] = dir[2] = 0;
      else
        vec_normalize(dir);
      find_pos(pt, pos);
      return true;
    }
    expand_portal(pt, v4);
  }
}

__device__ void convex_obj(const Env& e, int g, double margin, ConvexObj& o) {
  const rmbx_model& m = *e.m;
  o.c = e.gxpos + 3 * g;
  o.R = e.gxmat + 9 * g;
  o.s = m.geom_csize + 3 * g;
  o.type = m.geom_ctype[g];
  o.hv = o.type == RMBX_GEOM_MESH ? m.hull_vert + 3 * m.geom_hulladr[g] : nullptr;
  o.nhv = o.type == RMBX_GEOM_MESH ? m.geom_hullnum[g] : 0;
  o.margin = margin;
}

__device__ int col_convex(const Env& e, int ga, int gb, double margin, Contact* out) {
  ConvexObj a, b;
  convex_obj(e, ga, margin, a);
  convex_obj(e, gb, margin, b);
  double depth, dir[3], pos[3];
  if (!mpr_penetration(a, b, &depth, dir, pos)) return 0;
  if (dir[0] == 0 && dir[1] == 0 && dir[2] == 0) return 0;
  const double dist = margin - depth;
  if (dist >= margin) return 0;
  for (int i = 0; i < 3; i++) {
    out->n[i] = dir[i];
    out->pos[i] = pos[i];
  }
  out->dist = dist;
  return 1;
}

// stable top-4 of a candidate stream by contact_deeper (earlier candidates win ties)
__device__ void top4_insert(Contact* best, int* nb, const Contact& c) {
  const int k = *nb < 4 ? *nb : 4;
  int at = k;
  while (at > 0 && contact_deeper(&c, &best[at - 1])) at--;
  if (at >= 4) return;
  for (int i = (k < 4 ? k : 3); i > at; i--) best[i] = best[i - 1];
  best[at] = c;
  if (*nb < 4) (*nb)++;
}

__device__ int col_plane_mesh(const double* cp, const double* Rp, const double* cb, const double* Rb,
                              const double* hv, int nhv, double margin, Contact* out) {
  const double n[3] = {Rp[2], Rp[5], Rp[8]};
  int nb = 0;
  for (int k = 0; k < nhv; k++) {
    double w[3], x[3];
    matvec3(Rb, hv + 3 * k, w);
    for (int i = 0; i < 3; i++) x[i] = cb[i] + w[i];
    const double v[3] = {x[0] - cp[0], x[1] - cp[1], x[2] - cp[2]};
    Contact c;
    c.dist = dot3(v, n);
    if (c.dist >= margin) continue;
    for (int i = 0; i < 3; i++) {
      c.n[i] = n[i];
      c.pos[i] = x[i] - n[i] * (0.5 * c.dist);
    }
    top4_insert(out, &nb, c);
  }
  return nb;
}

__device__ int col_plane_cylinder(const double* cp, const double* Rp, const double* cb, const double* Rb,
                                  const double* sb, double margin, Contact* out) {
  const double n[3] = {Rp[2], Rp[5], Rp[8]}, ax[3] = {Rb[2], Rb[5], Rb[8]};
  const double r = sb[0], h = sb[1];
  const double prj = dot3(n, ax);
  double u[3] = {-(n[0] - prj * ax[0]), -(n[1] - prj * ax[1]), -(n[2] - prj * ax[2])};
  const double lu = norm3(u);
  double v[3];
  if (lu < 1e-12) {
    u[0] = Rb[0];
    u[1] = Rb[3];
    u[2] = Rb[6];
  } else {
    for (int i = 0; i < 3; i++) u[i] /= lu;
  }
  cross3(ax, u, v);
  const double sgn = prj > 0 ? -1.0 : 1.0;
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
    const double w[3] = {pts[k][0] - cp[0], pts[k][1] - cp[1], pts[k][2] - cp[2]};
    Contact c;
    c.dist = dot3(w, n);
    if (c.dist >= margin) continue;
    for (int i = 0; i < 3; i++) {
      c.n[i] = n[i];
      c.pos[i] = pts[k][i] - n[i] * (0.5 * c.dist);
    }
    top4_insert(out, &nb, c);
  }
  return nb;
}

// Narrow-phase classes.  The collision stage first classifies every pair (broadphase + type
// combination), then runs one collider at a time over the compacted survivors of its class, so a
// wave never executes the union of the colliders its 64 pairs happen to need.
enum { CLS_PLANE = 0, CLS_SPH_SPH, CLS_SPH_CAP, CLS_SPH_BOX, CLS_CAP_CAP, CLS_CAP_BOX, CLS_BOX_BOX, CLS_CONVEX, NCLS };

// Broadphase record of one geom in LDS (8 doubles): centre, AABB half-extent (a plane: its
// normal), bounding radius, type.
// broadphase record of geom g: center [3], half-extents (plane: normal) [3], rbound; the type goes to
// a byte array beside the records (gtype)
constexpr int GREC = 7;
__device__ void geom_record(const Env& e, int g, double* r, uint8_t* gtype) {
  const rmbx_model& m = *e.m;
  const double* c = e.gxpos + 3 * g;
  const double* R = e.gxmat + 9 * g;
  const double* s = m.geom_csize + 3 * g;
  const int t = m.geom_ctype[g];
  double x[GREC];
  for (int i = 0; i < 3; i++) {
    x[i] = c[i];
    if (t == RMBX_GEOM_PLANE)
      x[3 + i] = R[3 * i + 2];
    else if (t == RMBX_GEOM_SPHERE)
      x[3 + i] = s[0];
    else if (t == RMBX_GEOM_CAPSULE || t == RMBX_GEOM_CYLINDER)
      x[3 + i] = fabs(R[3 * i + 2]) * s[1] + s[0];
    else
      x[3 + i] = fabs(R[3 * i]) * s[0] + fabs(R[3 * i + 1]) * s[1] + fabs(R[3 * i + 2]) * s[2];
  }
  x[6] = m.geom_rbound[g];
  for (int i = 0; i < GREC; i++) r[i] = x[i];
  gtype[g] = (uint8_t)t;
}

// broadphase of pair p (geoms g1, g2, records in LDS); returns its narrow-phase class, or -1
// when it cannot touch (or the type combination has no collider: no contacts)
__device__ int pair_class(const double* grec, const uint8_t* gtype, int g1, int g2, double margin) {
  double r1[GREC], r2[GREC];
  for (int i = 0; i < GREC; i++) {
    r1[i] = grec[GREC * g1 + i];
    r2[i] = grec[GREC * g2 + i];
  }
  const int t1 = gtype[g1], t2 = gtype[g2];
  if (t1 == RMBX_GEOM_PLANE || t2 == RMBX_GEOM_PLANE) {
    const double* rp = t1 == RMBX_GEOM_PLANE ? r1 : r2;
    const double* ro = t1 == RMBX_GEOM_PLANE ? r2 : r1;
    const double v[3] = {ro[0] - rp[0], ro[1] - rp[1], ro[2] - rp[2]};
    if (dot3(v, rp + 3) - ro[6] > margin) return -1;
    return CLS_PLANE;
  }
  for (int i = 0; i < 3; i++) {
    const double lo1 = r1[i] - r1[3 + i], hi1 = r1[i] + r1[3 + i];
    const double lo2 = r2[i] - r2[3 + i], hi2 = r2[i] + r2[3 + i];
    if (lo1 > hi2 + margin || lo2 > hi1 + margin) return -1;
  }
  const int a = t1 < t2 ? t1 : t2, b = t1 < t2 ? t2 : t1;
  if (b == RMBX_GEOM_MESH || b == RMBX_GEOM_CYLINDER) return CLS_CONVEX;
  if (a == RMBX_GEOM_SPHERE) {
    if (b == RMBX_GEOM_SPHERE) return CLS_SPH_SPH;
    if (b == RMBX_GEOM_CAPSULE) return CLS_SPH_CAP;
    if (b == RMBX_GEOM_BOX) return CLS_SPH_BOX;
  } else if (a == RMBX_GEOM_CAPSULE) {
    if (b == RMBX_GEOM_CAPSULE) return CLS_CAP_CAP;
    if (b == RMBX_GEOM_BOX) return CLS_CAP_BOX;
  } else if (a == RMBX_GEOM_BOX && b == RMBX_GEOM_BOX) {
    return CLS_BOX_BOX;
  }
  return -1;
}

// narrow phase of a pair that passed pair_class (cls uniform across the wave)
__device__ int pair_narrow(const Env& e, int p, int cls, Contact* out) {
  const rmbx_model& m = *e.m;
  int g1 = m.pair_geom1[p], g2 = m.pair_geom2[p];
  const double margin = m.pair_margin[p];
  const int t1 = m.geom_ctype[g1], t2 = m.geom_ctype[g2];
  const bool flip = t1 > t2;
  if (flip) {
    const int t = g1;
    g1 = g2;
    g2 = t;
  }
  const double *c1 = e.gxpos + 3 * g1, *R1 = e.gxmat + 9 * g1, *s1 = m.geom_csize + 3 * g1;
  const double *c2 = e.gxpos + 3 * g2, *R2 = e.gxmat + 9 * g2, *s2 = m.geom_csize + 3 * g2;
  int n = 0;
  switch (cls) {
    case CLS_PLANE: {
      const int to = flip ? t1 : t2;
      if (to == RMBX_GEOM_MESH)
        n = col_plane_mesh(c1, R1, c2, R2, m.hull_vert + 3 * m.geom_hulladr[g2], m.geom_hullnum[g2], margin, out);
      else if (to == RMBX_GEOM_CYLINDER)
        n = col_plane_cylinder(c1, R1, c2, R2, s2, margin, out);
      else
        n = col_plane(c1, R1, to, c2, R2, s2, margin, out);
      break;
    }
    case CLS_CONVEX:
      n = col_convex(e, g1, g2, margin, out);
      break;
    case CLS_SPH_SPH:
      n = col_sphere_sphere(c1, s1[0], c2, s2[0], margin, out);
      break;
    case CLS_SPH_CAP: {
      double pp[3], qq[3], c[3], cc[3];
      capsule_ends(c2, R2, s2[1], pp, qq);
      closest_seg_seg(c1, c1, pp, qq, cc, c);
      n = col_sphere_sphere(c1, s1[0], c, s2[0], margin, out);
      break;
    }
    case CLS_SPH_BOX:
      n = col_sphere_box(c1, s1[0], c2, R2, s2, margin, out);
      break;
    case CLS_CAP_CAP: {
      double p1[3], q1[3], p2[3], q2[3], cc1[3], cc2[3];
      capsule_ends(c1, R1, s1[1], p1, q1);
      capsule_ends(c2, R2, s2[1], p2, q2);
      closest_seg_seg(p1, q1, p2, q2, cc1, cc2);
      n = col_sphere_sphere(cc1, s1[0], cc2, s2[0], margin, out);
      break;
    }
    case CLS_CAP_BOX:
      n = col_capsule_box(c1, R1, s1, c2, R2, s2, margin, out);
      break;
    default:
      n = col_box_box(c1, R1, s1, c2, R2, s2, margin, out);
      break;
  }
  if (flip)
    for (int i = 0; i < n; i++)
      for (int k = 0; k < 3; k++) out[i].n[k] = -out[i].n[k];
  return n;
}

__device__ void make_frame(const double* n, double* F) {
  F[0] = n[0];
  F[1] = n[1];
  F[2] = n[2];
  double a[3] = {0, 0, 0};
  if (fabs(n[0]) < 0.5)
    a[0] = 1;
  else
    a[1] = 1;
  const double t = dot3(a, n);
  double t1[3] = {a[0] - t * n[0], a[1] - t * n[1], a[2] - t * n[2]};
  const double l = norm3(t1);
  t1[0] /= l;
  t1[1] /= l;
  t1[2] /= l;
  double t2[3];
  cross3(n, t1, t2);
  F[3] = t1[0];
  F[4] = t1[1];
  F[5] = t1[2];
  F[6] = t2[0];
  F[7] = t2[1];
  F[8] = t2[2];
}

// LDS scratch of the collision stage.  It lives in the front kernel's velocity/RNE arrays, dead
// once velocity_stage has copied them out (extra dynamic LDS only for models where that region
// is too small): geom broadphase records; the survivors of the broadphase in pair order (pair
// index, narrow-phase class, contact count; at most collision_cap(npair), the same cap as the
// oracle's) and the class-major list of survivor indices.
#define RMBX_MAX_CANDIDATES 2048
// Two-level broadphase (models whose candidate pairs come in long runs with the same two bodies,
// e.g. the Pick scene's 32-hull meshes: 35,591 pairs in 1,301 runs): a run is tested first on its
// bodies' AABBs (the union of their collision geoms' broadphase boxes, a plane geom making it
// infinite) grown by the run's largest margin, and only the pairs of the runs that pass are
// classified.  Every pair pair_class accepts lies in a run that passes (its geoms' boxes lie in
// their bodies' boxes, its margin is at most the run's, and rounding is monotone), so the
// survivors -- and with them the contacts and their order -- are exactly the one-level pass's.
struct PairRuns {
  int n;                      // runs; 0: one-level broadphase
  const int32_t* start;       // [n + 1] pair range of each run
  const int32_t* body;        // [n][2] the run's two bodies
  const double* margin;       // [n] largest pair margin of the run
  const int32_t* body_cgeom;  // [nbody][2] first collision geom of the body, count
};
struct CollisionLds {
  double* geom;      // [ngeom][GREC] broadphase records
  uint8_t* gtype;    // [ngeom] geom types
  uint16_t* spair;   // survivors' pair indices (npair <= 65535, checked at engine creation)
  int16_t* list;
  uint8_t* count;
  uint8_t* scls;
  double* bbox;      // [nbody][6] body AABB (two-level only)
  int32_t* run_pre;  // [65] flat pair offsets of the kept runs of a 64-run chunk (two-level only)
  int32_t* run_id;   // [64] kept runs of the chunk, in order (two-level only)
};
__host__ __device__ __forceinline__ int collision_cap(int npair) {
  return npair < RMBX_MAX_CANDIDATES ? npair : RMBX_MAX_CANDIDATES;
}
// doubles of the survivor arrays: spair (2 B), list (2 B), count (1 B), scls (1 B) per survivor
__host__ __device__ __forceinline__ size_t collision_surv_doubles(int cap) { return (6 * (size_t)cap + 7) / 8 + 1; }
__host__ __device__ __forceinline__ size_t collision_lds_doubles(int ngeom, int npair, int nbody, int nprun) {
  // GREC doubles + a type byte per geom; 6 bytes per survivor; two-level: 6 doubles per body + 129
  // int32 of run-chunk bookkeeping
  const size_t runs = nprun > 0 ? 6 * (size_t)nbody + 65 : 0;
  return GREC * (size_t)ngeom + ((size_t)ngeom + 7) / 8 + collision_surv_doubles(collision_cap(npair)) + runs;
}
// The collision scratch starts at 16 nb: everything above the body frames (cvel, cacc, cfrc,
// cdofdot, cinert, crb, cdof) is dead once the velocity stage has copied it out, and a model whose
// scratch is larger runs past the end of that region.  The cable scene's 1,891 doubles fit in
// the 2,906 there: 29.6 KiB of LDS per env instead of 48.1, so four envs per CU and all 1,024 in
// one round of blocks; the Pick scene's 4,276 take it to 38.8 KiB (four envs per CU, was 61.5: two)
__host__ __device__ __forceinline__ size_t front_kernel_lds_doubles(int nb, int nv, size_t need) {
  const size_t front = front_lds_doubles(nb, nv), coll = 16 * (size_t)nb + need;
  return front > coll ? front : coll;
}
static inline size_t front_kernel_lds_bytes(const rmbx_model& h, int nprun) {
  const size_t need = collision_lds_doubles(h.ngeom, h.npair, h.nbody, nprun);
  return front_kernel_lds_doubles(h.nbody, h.nv, need) * sizeof(double);
}
__device__ __forceinline__ CollisionLds collision_lds(const Env& e, const PairRuns& pr) {
  const rmbx_model& m = *e.m;
  CollisionLds cl;
  const int cap = collision_cap(m.npair);
  cl.geom = e.sh + 16 * m.nbody;  // (front_kernel_lds_bytes sized the LDS for it)
  cl.gtype = reinterpret_cast<uint8_t*>(cl.geom + GREC * m.ngeom);
  double* sv = cl.geom + GREC * m.ngeom + (m.ngeom + 7) / 8;
  cl.spair = reinterpret_cast<uint16_t*>(sv);
  cl.list = reinterpret_cast<int16_t*>(cl.spair + cap);
  cl.count = reinterpret_cast<uint8_t*>(cl.list + cap);
  cl.scls = cl.count + cap;
  cl.bbox = sv + collision_surv_doubles(cap);
  cl.run_pre = reinterpret_cast<int32_t*>(cl.bbox + 6 * m.nbody);
  cl.run_id = cl.run_pre + 65;
  return cl;
}

// the two-level broadphase (PairRuns): survivors in pair order, at most cap (inlined: an
// out-of-line call made the front kernel save its live registers around it, +1.5 KiB of scratch)
__device__ __forceinline__ int broadphase_runs(const Env& e, int lane, const CollisionLds& cl,
                                                         const PairRuns& pr, int cap) {
  const rmbx_model& m = *e.m;
  const unsigned long long below = (1ull << lane) - 1;
  int nsurv = 0;
  // level 1: body AABBs (lane per body), then the runs on them, kept runs compacted in order
  // with the flat offsets of their pairs
  for (int b = lane; b < m.nbody; b += 64) {
    double lx = 1e300, ly = 1e300, lz = 1e300, hx = -1e300, hy = -1e300, hz = -1e300;
    bool inf = false;
    const int g0 = pr.body_cgeom[2 * b], gn = pr.body_cgeom[2 * b + 1];
    for (int g = g0; g < g0 + gn; g++) {
      const double* r = cl.geom + GREC * g;
      if (m.geom_ctype[g] < 0) continue;  // visual only
      if (cl.gtype[g] == RMBX_GEOM_PLANE) {
        inf = true;
        continue;
      }
      lx = fmin(lx, r[0] - r[3]);
      ly = fmin(ly, r[1] - r[4]);
      lz = fmin(lz, r[2] - r[5]);
      hx = fmax(hx, r[0] + r[3]);
      hy = fmax(hy, r[1] + r[4]);
      hz = fmax(hz, r[2] + r[5]);
    }
    double* bb = cl.bbox + 6 * b;
    bb[0] = inf ? -1e300 : lx;
    bb[1] = inf ? -1e300 : ly;
    bb[2] = inf ? -1e300 : lz;
    bb[3] = inf ? 1e300 : hx;
    bb[4] = inf ? 1e300 : hy;
    bb[5] = inf ? 1e300 : hz;
  }
  sync();
  // runs in chunks of 64: the chunk's kept runs are compacted in order with the flat offsets
  // of their pairs, then those pairs are classified (level 2), lane i of a pair chunk finding
  // its run by binary search over the kept runs' offsets -- survivors stay in pair order
  for (int rbase = 0; rbase < pr.n && nsurv < cap; rbase += 64) {
    const int r = rbase + lane;
    bool ok = false;
    int size = 0;
    if (r < pr.n) {
      const double* b1 = cl.bbox + 6 * pr.body[2 * r];
      const double* b2 = cl.bbox + 6 * pr.body[2 * r + 1];
      const double mg = pr.margin[r];
      ok = true;
      for (int i = 0; i < 3; i++)
        if (b1[i] > b2[3 + i] + mg || b2[i] > b1[3 + i] + mg) ok = false;
      size = ok ? pr.start[r + 1] - pr.start[r] : 0;
    }
    int total;
    const int off = wave_excl_scan(size, lane, &total);
    const unsigned long long rk = __ballot(ok);
    const int nkeep = __popcll(rk);
    if (ok) {
      const int k = __popcll(rk & below);
      cl.run_id[k] = r;
      cl.run_pre[k] = off;
    }
    if (lane == 0) cl.run_pre[nkeep] = total;
    sync();
    for (int base = 0; base < total && nsurv < cap; base += 64) {
      const int i = base + lane;
      int c = -1, p = 0;
      if (i < total) {
        int lo = 0, hi = nkeep;  // run_pre[lo] <= i < run_pre[hi]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (cl.run_pre[mid] <= i)
            lo = mid;
          else
            hi = mid;
        }
        p = pr.start[cl.run_id[lo]] + (i - cl.run_pre[lo]);
        c = pair_class(cl.geom, cl.gtype, m.pair_geom1[p], m.pair_geom2[p], m.pair_margin[p]);
      }
      const unsigned long long mk = __ballot(c >= 0);
      const int idx = nsurv + __popcll(mk & below);
      if (c >= 0 && idx < cap) {
        cl.spair[idx] = (uint16_t)p;
        cl.scls[idx] = (uint8_t)c;
      }
      nsurv += __popcll(mk);
    }
    sync();
  }
  return nsurv;
}

// Contacts in pair order, at most max_contacts (the serial per-pair loop's result, bit for bit):
// 1. broadphase + class of every pair (geom records staged in LDS); survivors appended in pair
//    order (at most collision_cap(npair): the scan stops there, as the oracle's loop does)
// 2. survivors listed class-major
// 3. one collider at a time over its class's survivors, contacts into con_tmp[survivor]
// 4. pair-order scan of the survivors' counts, contacts copied to their final slots
template <bool RUNS>
__device__ int collision(Env& e, int lane, const CollisionLds& cl, const PairRuns& pr, unsigned long long* prof) {
  const rmbx_model& m = *e.m;
  unsigned long long tp = prof ? stamp() : 0;
  const int np = m.npair;
  const int cap = collision_cap(np);
  const unsigned long long below = (1ull << lane) - 1;
  for (int g = lane; g < m.ngeom; g += 64) geom_record(e, g, cl.geom + GREC * g, cl.gtype);
  sync();
  SUBPROF(16)
  int nsurv = 0;
  if constexpr (RUNS) {
    nsurv = broadphase_runs(e, lane, cl, pr, cap);
  } else {
    // pair indices and margins of the next chunk are loaded before this chunk's tests
    int g1n = 0, g2n = 0;
    double mn = 0;
    if (lane < np) {
      g1n = m.pair_geom1[lane];
      g2n = m.pair_geom2[lane];
      mn = m.pair_margin[lane];
    }
    for (int base = 0; base < np && nsurv < cap; base += 64) {
      const int p = base + lane;
      const int g1 = g1n, g2 = g2n;
      const double mg = mn;
      if (p + 64 < np) {
        g1n = m.pair_geom1[p + 64];
        g2n = m.pair_geom2[p + 64];
        mn = m.pair_margin[p + 64];
      }
      const int c = p < np ? pair_class(cl.geom, cl.gtype, g1, g2, mg) : -1;
      const unsigned long long mk = __ballot(c >= 0);
      const int idx = nsurv + __popcll(mk & below);
      if (c >= 0 && idx < cap) {
        cl.spair[idx] = (uint16_t)p;
        cl.scls[idx] = (uint8_t)c;
      }
      nsurv += __popcll(mk);
    }
  }
  nsurv = nsurv < cap ? nsurv : cap;
  if (nsurv == 0) return 0;
  sync();
  int cnt[NCLS], off[NCLS], run[NCLS];
#pragma unroll
  for (int k = 0; k < NCLS; k++) cnt[k] = 0;
  for (int base = 0; base < nsurv; base += 64) {
    const int i = base + lane;
    const int c = i < nsurv ? cl.scls[i] : -1;
#pragma unroll
    for (int k = 0; k < NCLS; k++) cnt[k] += __popcll(__ballot(c == k));
  }
  int acc = 0;
#pragma unroll
  for (int k = 0; k < NCLS; k++) {
    off[k] = run[k] = acc;
    acc += cnt[k];
  }
  for (int base = 0; base < nsurv; base += 64) {
    const int i = base + lane;
    const int c = i < nsurv ? cl.scls[i] : -1;
#pragma unroll
    for (int k = 0; k < NCLS; k++) {
      const unsigned long long mk = __ballot(c == k);
      if (c == k) cl.list[run[k] + __popcll(mk & below)] = (int16_t)i;
      run[k] += __popcll(mk);
    }
  }
  sync();
  SUBPROF(17)
  double* tmp = W(con_tmp);
#pragma unroll 1
  for (int k = 0; k < NCLS; k++) {
    const int end = off[k] + cnt[k];
    for (int i0 = off[k]; i0 < end; i0 += 64) {
      const int i = i0 + lane;
      if (i < end) {
        const int sv = cl.list[i];
        Contact c[4];
        const int n = pair_narrow(e, cl.spair[sv], k, c);
        cl.count[sv] = (uint8_t)n;
        double* t = tmp + 28 * (size_t)sv;
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (j < n) {
            for (int d = 0; d < 3; d++) {
              t[7 * j + d] = c[j].pos[d];
              t[7 * j + 3 + d] = c[j].n[d];
            }
            t[7 * j + 6] = c[j].dist;
          }
      }
    }
  }
  sync();
  SUBPROF(18)
  int ncon = 0;
  for (int base = 0; base < nsurv && ncon < m.max_contacts; base += 64) {
    const int sv = base + lane;
    const int n = sv < nsurv ? cl.count[sv] : 0;
    const int p = sv < nsurv ? cl.spair[sv] : 0;
    int total;
    const int o = wave_excl_scan(n, lane, &total);
    const double* t = tmp + 28 * (size_t)(sv < nsurv ? sv : 0);
    for (int i = 0; i < n; i++) {
      const int k = ncon + o + i;
      if (k >= m.max_contacts) break;
      for (int j = 0; j < 3; j++) W(con_pos)[3 * k + j] = t[7 * i + j];
      make_frame(t + 7 * i + 3, W(con_frame) + 9 * k);
      W(con_dist)[k] = t[7 * i + 6];
      W(con_mu)[k] = m.pair_friction[3 * p];
      WI(con_b1)[k] = m.geom_body[m.pair_geom1[p]];
      WI(con_b2)[k] = m.geom_body[m.pair_geom2[p]];
      WI(con_condim)[k] = m.pair_condim[p];
      WI(con_pair)[k] = p;
    }
    ncon += total;
  }
  return ncon < m.max_contacts ? ncon : m.max_contacts;
}


// ------------------------------------------------------------------------------------------
// constraint rows
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int last_dof(const rmbx_model& m, int b) {
  const int w = m.body_weldid[b];
  if (w == 0) return -1;
  return m.body_dofadr[w] + m.body_dofnum[w] - 1;
}

// dof k moves body b (its body is b or an ancestor of b: DFS subtree range test)
__device__ __forceinline__ bool dof_on_chain(const Env& e, int k, int b) {
  const int a = e.m->dof_body[k];
  return a <= b && b < e.subtree_end[a];
}

__device__ double impedance(const double* solimp, double x) {
  double dmin = fmin(fmax(solimp[0], 0.0001), 0.9999);
  double dmax = fmin(fmax(solimp[1], 0.0001), 0.9999);
  const double width = solimp[2], mid = solimp[3], power = solimp[4];
  x = fabs(x);
  if (width <= RMBX_MINVAL || x >= width) return dmax;
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

// stores b in efc_tmp, k*imp*pos in efc_D, R in efc_R (finalised after J is complete)
__device__ __forceinline__ void set_row(Env& e, int r, int type, double pos, double diag, const double* solref,
                        const double* solimp, double impx) {
  const double dmax = fmin(fmax(solimp[1], 0.0001), 0.9999);
  double tc = solref[0];
  const double dr = solref[1];
  const double h2 = 2 * e.m->timestep;
  if (tc < h2) tc = h2;
  const double k = 1 / (dmax * dmax * tc * tc * dr * dr);
  const double b = 2 / (dmax * tc);
  const double imp = impedance(solimp, impx);
  WI(efc_type)[r] = type;
  W(efc_pos)[r] = pos;
  W(efc_tmp)[r] = b;
  W(efc_D)[r] = k * imp * pos;
  double R = (1 - imp) / imp * diag;
  W(efc_R)[r] = R < RMBX_MINVAL ? RMBX_MINVAL : R;
}

// pyramid edge t of a contact (t = 4: the normal of a frictionless contact), the row directions
// of mj_instantiateContact: normal +- mu * tangent_(t/2)
__device__ __forceinline__ void contact_dir(const double* F, double mu, int t, double* dir) {
  if (t == 4) {
    dir[0] = F[0];
    dir[1] = F[1];
    dir[2] = F[2];
    return;
  }
  const double s = (t & 1) ? -mu : mu;
  const double* T = F + 3 * (1 + (t >> 1));
#pragma unroll
  for (int i = 0; i < 3; i++) dir[i] = F[i] + s * T[i];
}

// 6-dot with a depth-3 dependency tree (three products, two pair sums, one final sum) instead
// of the 6-long FMA chain of dot6: each dependent f64 op costs ~32 cycles on a wave
__device__ __forceinline__ double dot6t(const double* a, const double* b) {
  const double p0 = fma(a[0], b[0], a[1] * b[1]);
  const double p1 = fma(a[2], b[2], a[3] * b[3]);
  const double p2 = fma(a[4], b[4], a[5] * b[5]);
  return (p0 + p1) + p2;
}

// velocity of point p on body b2 relative to body b1, from per-body spatial velocities V
// (6 per body: angular, linear at the world origin; V of the world body is zero)
__device__ __forceinline__ void rel_point_vel(const double* V, int b1, int b2, const double* p, double* u) {
  double d[6];
#pragma unroll
  for (int i = 0; i < 6; i++) d[i] = V[6 * b2 + i] - V[6 * b1 + i];
  double wxp[3];
  cross3(d, p, wxp);
#pragma unroll
  for (int i = 0; i < 3; i++) u[i] = d[3 + i] + wxp[i];
}

// returns nefc; equality rows first (count in *ne).  Rows are described, not materialised (see
// the ROW_* comment at the top): each row gets its kind/object, the equality rows their two
// body-side 6-vectors, and efc_vel = J qvel is evaluated from the body velocities cvel.
__device__ int make_constraints(Env& e, int lane, int ncon, int* ne_out, int* nlim_out, unsigned long long* prof) {
  const rmbx_model& m = *e.m;
  unsigned long long tp = prof ? stamp() : 0;
  const int nefc_max = e.L->nefc_max;
  const double* cvel = W(cvel);  // (the LDS copy is collision scratch by now)
  int32_t* kind = WI(efc_kind);
  int32_t* obj = WI(efc_obj);
  double* vel = W(efc_vel);
  // count rows: equality
  int ne = 0;
  for (int q = 0; q < m.neq; q++) ne += m.eq_type[q] == RMBX_EQ_CONNECT ? 3 : (m.eq_type[q] == RMBX_EQ_WELD ? 6 : 1);
  // limits: ballot compaction in joint order
  int nlim = 0;
  for (int base = 0; base < m.njnt; base += 64) {
    const int j = base + lane;
    int cnt = 0;
    if (j < m.njnt && m.jnt_limited[j]) {
      const double q = e.qpos[m.jnt_qposadr[j]];
      cnt = (q - m.jnt_range[2 * j] < 0) + (m.jnt_range[2 * j + 1] - q < 0);
    }
    nlim += wave_sum_i(cnt);
  }
  // contacts rows (wave-parallel count)
  int nconrow = 0;
  for (int base = 0; base < ncon; base += 64) {
    const int c = base + lane;
    nconrow += wave_sum_i(c < ncon ? (WI(con_condim)[c] == 1 ? 1 : 4) : 0);
  }
  int nefc = ne + nlim + nconrow;
  if (nefc > nefc_max) nefc = nefc_max;
  SUBPROF(20)
  // equality rows: every lane evaluates the constraint's anchors/errors (cheap, no broadcast),
  // lane i < nrows describes row i: connect/weld translation J = J_p1(o1) e_i - J_p2(o2) e_i,
  // i.e. body-side vectors (p1 x e_i, e_i) and -(p2 x e_i, e_i); weld rotation
  // J = 0.5 d10 Im(conj(q1 r) (0, w) q2)_i with w = +cdof_ang on chain(o2), -cdof_ang on chain(o1)
  int r = 0, s = 0;
  double* eq_rho = W(eqr_rho);
  double* eq_coef = W(eqr_coef);
  int32_t* eq_body = WI(eqr_body);
  int32_t* eq_dof = WI(eqr_dof);
  for (int q = 0; q < m.neq; q++) {
    const double* data = m.eq_data + RMBX_EQ_DATA * q;
    const double* sr = m.eq_solref + 2 * q;
    const double* si = m.eq_solimp + 5 * q;
    const int o1 = m.eq_obj1[q], o2 = m.eq_obj2[q];
    const int type = m.eq_type[q];
    if (type == RMBX_EQ_CONNECT || type == RMBX_EQ_WELD) {
      double p1[3], p2[3], t[3], err[6];
      const int nr = type == RMBX_EQ_CONNECT ? 3 : 6;
      const double* xm = e.sh + 7 * m.nbody;  // xmat (LDS)
      if (type == RMBX_EQ_CONNECT) {
        matvec3(xm + 9 * o1, data, t);
        for (int i = 0; i < 3; i++) p1[i] = e.sh[3 * o1 + i] + t[i];
        matvec3(xm + 9 * o2, data + 3, t);
        for (int i = 0; i < 3; i++) p2[i] = e.sh[3 * o2 + i] + t[i];
      } else {
        double Rr[9], ra[3], u[3];
        quat2mat(data + 6, Rr);
        matvec3(Rr, data, ra);
        for (int i = 0; i < 3; i++) u[i] = data[3 + i] + ra[i];
        matvec3(xm + 9 * o1, u, t);
        for (int i = 0; i < 3; i++) p1[i] = e.sh[3 * o1 + i] + t[i];
        matvec3(xm + 9 * o2, data, t);
        for (int i = 0; i < 3; i++) p2[i] = e.sh[3 * o2 + i] + t[i];
      }
      for (int i = 0; i < 3; i++) err[i] = p1[i] - p2[i];
      double q1r[4], qe[4], cq1[4];
      const double* xq1 = e.sh + 3 * m.nbody + 4 * o1;
      const double* xq2 = e.sh + 3 * m.nbody + 4 * o2;
      if (nr == 6) {
        quatmul(xq1, data + 6, q1r);
        cq1[0] = q1r[0];
        cq1[1] = -q1r[1];
        cq1[2] = -q1r[2];
        cq1[3] = -q1r[3];
        quatmul(cq1, xq2, qe);
        for (int i = 0; i < 3; i++) err[3 + i] = qe[1 + i] * data[10];
      }
      double nrm = 0;
      for (int i = 0; i < nr; i++) nrm += err[i] * err[i];
      nrm = sqrt(nrm);
      if (lane < nr) {
        double rho1[6], rho2[6];
        if (lane < 3) {
          const double diag_t = m.body_invweight0[2 * o1] + m.body_invweight0[2 * o2];
          set_row(e, r + lane, 0, err[lane], diag_t, sr, si, nrm);
          double ei[3] = {0, 0, 0}, c2[3];
          ei[lane] = 1;
          cross3(p1, ei, rho1);
          cross3(p2, ei, c2);
          for (int i = 0; i < 3; i++) {
            rho1[3 + i] = ei[i];
            rho2[i] = -c2[i];
            rho2[3 + i] = -ei[i];
          }
        } else {
          const double diag_r = m.body_invweight0[2 * o1 + 1] + m.body_invweight0[2 * o2 + 1];
          set_row(e, r + lane, 0, err[lane], diag_r, sr, si, nrm);
          const int i = lane - 3;
          for (int j = 0; j < 3; j++) {
            double wq[4] = {0, 0, 0, 0}, t1[4], t2[4];
            wq[1 + j] = 1;
            quatmul(cq1, wq, t1);
            quatmul(t1, xq2, t2);
            rho2[j] = 0.5 * t2[1 + i] * data[10];
            rho1[j] = -rho2[j];
            rho1[3 + j] = rho2[3 + j] = 0.0;
          }
        }
        const int sl = s + lane;
        for (int i = 0; i < 6; i++) {
          eq_rho[12 * sl + i] = rho1[i];
          eq_rho[12 * sl + 6 + i] = rho2[i];
        }
        eq_body[2 * sl] = o1;
        eq_body[2 * sl + 1] = o2;
        eq_dof[2 * sl] = eq_dof[2 * sl + 1] = -1;
        eq_coef[2 * sl] = eq_coef[2 * sl + 1] = 0.0;
        kind[r + lane] = ROW_EQ;
        obj[r + lane] = sl;
        vel[r + lane] = dot6(rho1, cvel + 6 * o1) + dot6(rho2, cvel + 6 * o2);
      }
      r += nr;
      s += nr;
    } else {
      if (lane == 0) {
        const int j1 = o1, j2 = o2;
        const double q1 = e.qpos[m.jnt_qposadr[j1]] - m.qpos0[m.jnt_qposadr[j1]];
        const double q2 = e.qpos[m.jnt_qposadr[j2]] - m.qpos0[m.jnt_qposadr[j2]];
        const double* c = data;
        const double poly = c[0] + q2 * (c[1] + q2 * (c[2] + q2 * (c[3] + q2 * c[4])));
        const double dpoly = c[1] + q2 * (2 * c[2] + q2 * (3 * c[3] + q2 * 4 * c[4]));
        const double err = q1 - poly;
        const int d1 = m.jnt_dofadr[j1], d2 = m.jnt_dofadr[j2];
        set_row(e, r, 0, err, m.dof_invweight0[d1] + m.dof_invweight0[d2], sr, si, err);
        for (int i = 0; i < 12; i++) eq_rho[12 * s + i] = 0.0;
        eq_body[2 * s] = eq_body[2 * s + 1] = 0;
        eq_dof[2 * s] = d1;
        eq_dof[2 * s + 1] = d2;
        eq_coef[2 * s] = 1.0;
        eq_coef[2 * s + 1] = -dpoly;
        kind[r] = ROW_EQ;
        obj[r] = s;
        vel[r] = e.qvel[d1] - dpoly * e.qvel[d2];
      }
      r++;
      s++;
    }
  }
  SUBPROF(21)
  // limit rows
  int rbase = ne;
  for (int base = 0; base < m.njnt; base += 64) {
    const int j = base + lane;
    int cnt = 0;
    double d0 = 0, d1 = 0;
    if (j < m.njnt && m.jnt_limited[j]) {
      const double q = e.qpos[m.jnt_qposadr[j]];
      d0 = q - m.jnt_range[2 * j];
      d1 = m.jnt_range[2 * j + 1] - q;
      cnt = (d0 < 0) + (d1 < 0);
    }
    int total;
    const int off = wave_excl_scan(cnt, lane, &total);
    int r = rbase + off;
    if (cnt) {
      const int da = m.jnt_dofadr[j];
      if (d0 < 0 && r < nefc) {
        set_row(e, r, 1, d0, m.dof_invweight0[da], m.jnt_solref + 2 * j, m.jnt_solimp + 5 * j, d0);
        kind[r] = ROW_LIMIT;
        obj[r] = da;
        vel[r] = e.qvel[da];
        r++;
      }
      if (d1 < 0 && r < nefc) {
        set_row(e, r, 1, d1, m.dof_invweight0[da], m.jnt_solref + 2 * j, m.jnt_solimp + 5 * j, d1);
        kind[r] = ROW_LIMIT | (1 << 3);
        obj[r] = da;
        vel[r] = -e.qvel[da];
      }
    }
    rbase += total;
  }
  // contact rows: row address = rbase + 4*c (condim 3) / running offset with condim 1
  for (int base = 0; base < ncon; base += 64) {
    const int c = base + lane;
    const int cnt = c < ncon ? (WI(con_condim)[c] == 1 ? 1 : 4) : 0;
    int total;
    const int off = wave_excl_scan(cnt, lane, &total);
    if (c < ncon) {
      const int r0 = rbase + off;
      WI(con_efcadr)[c] = r0;
      const int p = WI(con_pair)[c];
      const int b1 = WI(con_b1)[c], b2 = WI(con_b2)[c];
      const double* F = W(con_frame) + 9 * c;
      const double* pos = W(con_pos) + 3 * c;
      const double tran = m.body_invweight0[2 * b1] + m.body_invweight0[2 * b2];
      const double dist = W(con_dist)[c] - m.pair_margin[p];
      const double* sr = m.pair_solref + 2 * p;
      const double* si = m.pair_solimp + 5 * p;
      const double mu = W(con_mu)[c];
      double dv[6];
      for (int i = 0; i < 6; i++) dv[i] = cvel[6 * b2 + i] - cvel[6 * b1 + i];
      for (int t = 0; t < cnt; t++) {
        const int rr = r0 + t;
        if (rr >= nefc) break;
        const int tt = cnt == 1 ? 4 : t;
        set_row(e, rr, 1, dist, cnt == 1 ? tran : tran * (1 + mu * mu), sr, si, dist);
        double rho[6];
        contact_dir(F, mu, tt, rho + 3);
        cross3(pos, rho + 3, rho);
        double* dst = W(efc_rho) + 6 * (size_t)rr;
        for (int i = 0; i < 6; i++) dst[i] = rho[i];
        kind[rr] = ROW_CONTACT | (tt << 3);
        obj[rr] = c;
        vel[rr] = dot6t(rho, dv);
      }
    }
    rbase += total;
  }
  sync();
  SUBPROF(22)
  // aref = -b (J qvel) - k imp pos ; D = 1/R
  for (int r = lane; r < nefc; r += 64) {
    W(efc_aref)[r] = -W(efc_tmp)[r] * vel[r] - W(efc_D)[r];
    const double D = 1.0 / W(efc_R)[r];
    W(efc_D)[r] = D;
    W(efc_sqD)[r] = sqrt(D);  // the Hessian's row weight
  }
  sync();
  SUBPROF(23)
  *ne_out = ne;
  *nlim_out = min(nlim, nefc - ne);
  return nefc;
}

// ------------------------------------------------------------------------------------------
// sensors (mj_rnePostConstraint -> force/torque at sites)
// ------------------------------------------------------------------------------------------
__device__ void sensors(Env& e, int ncon, int tid, double* cacc, double* cfrc, double* cw, int* s_anc,
                        const int32_t* subtree_end) {
  const rmbx_model& m = *e.m;
  if (m.nsensor == 0) return;
  const int nb = m.nbody;
  rne_forward(e, W(qacc), cacc, cfrc, W(cvel), W(cdofdot), W(cdof), W(cinert), s_anc, tid);
  // contact wrenches about the origin, lanes over contacts: cw[c] = (p x F, F)
  for (int c = tid; c < ncon; c += blockDim.x) {
    double* o = cw + 6 * c;
    const int r0 = WI(con_efcadr)[c];
    if (r0 + (WI(con_condim)[c] == 1 ? 1 : 4) > e.L->nefc_max) {
      for (int i = 0; i < 6; i++) o[i] = 0;
      continue;
    }
    const double* F = W(con_frame) + 9 * c;
    double fn, f1 = 0, f2 = 0;
    const double* f = W(efc_force) + r0;
    if (WI(con_condim)[c] == 1) {
      fn = f[0];
    } else {
      const double mu = W(con_mu)[c];
      fn = f[0] + f[1] + f[2] + f[3];
      f1 = mu * (f[0] - f[1]);
      f2 = mu * (f[2] - f[3]);
    }
    double Fw[3];
    for (int i = 0; i < 3; i++) Fw[i] = fn * F[i] + f1 * F[3 + i] + f2 * F[6 + i];
    cross3(W(con_pos) + 3 * c, Fw, o);
    for (int i = 0; i < 3; i++) o[3 + i] = Fw[i];
  }
  sync();
  // per body, in contact order (body 2 receives -w, body 1 +w)
  if (tid > 0 && tid < nb) {
    double acc[6];
    for (int i = 0; i < 6; i++) acc[i] = cfrc[6 * tid + i];
    for (int c = 0; c < ncon; c++) {
      if (WI(con_b2)[c] == tid)
        for (int i = 0; i < 6; i++) acc[i] -= cw[6 * c + i];
      if (WI(con_b1)[c] == tid)
        for (int i = 0; i < 6; i++) acc[i] += cw[6 * c + i];
    }
    for (int i = 0; i < 6; i++) cfrc[6 * tid + i] = acc[i];
  }
  sync();
  if (tid < m.nsensor && tid < 2) {
    const int s = tid;
    const int site = m.sensor_site[s];
    const int b = m.site_body[site];
    double f[6];
    for (int i = 0; i < 6; i++) f[i] = cfrc[6 * b + i];
    for (int d = b + 1; d < subtree_end[b]; d++)  // interaction force = subtree sum
      for (int i = 0; i < 6; i++) f[i] += cfrc[6 * d + i];
    const double* p = W(sxpos) + 3 * site;
    const double* R = W(sxmat) + 9 * site;
    double out[3];
    if (m.sensor_type[s] == RMBX_SENS_FORCE) {
      mattvec3(R, f + 3, out);
    } else {
      double pxf[3], n[3];
      cross3(p, f + 3, pxf);
      for (int i = 0; i < 3; i++) n[i] = f[i] - pxf[i];
      mattvec3(R, n, out);
    }
    for (int i = 0; i < 3; i++) e.sensordata[3 * s + i] = out[i];
  }
  sync();
}

// ------------------------------------------------------------------------------------------
// Solver kernel (256 threads per env): Newton solve of the constraint problem, constraint
// forces, site sensors and implicitfast integration.  Dense nv x nv matrices are held as 4x4
// f64 blocks in the registers of the threads that own the lower-triangle blocks (one block per
// thread, 153 threads at nv = 68); Cholesky, triangular solves and the Hessian J^T D J
// accumulation run on those register blocks with only one block column / vector staged in LDS.
// The constraint Jacobian streams from the workspace (HBM/L2) through a 16-row LDS chunk.
// ------------------------------------------------------------------------------------------
#define SOLVER_THREADS 256
#define MAX_NB 18  // nv <= 72
#define MAX_NVP (4 * MAX_NB)
#define RCHUNK 16
#define MAX_BODY 64
#define NEQR 24     // equality rows staged in LDS (6 per weld, 3 per connect, 1 per joint)
#define MAX_LIM 128 // limit rows staged in LDS (2 per limited joint)
#define MAX_CON 208  // contacts (J^T w: one wrench per contact in S.cw)
#define EQ_TAG 1024
static_assert(NEQR + MAX_LIM <= RCHUNK * 12, "J^T w stages the equality/limit row weights in S.jrho");
// capacity of the Hessian build's row-selection list: every constraint row can be selected once,
// and nefc_max = 4 max_contacts + 6 neq + 2 njnt + 8 (make_layout) with max_contacts <= MAX_CON,
// neq <= NEQR (each equality has >= 1 row) and 2 njnt <= MAX_LIM (checked at create)
#define HSEL_CAP (4 * MAX_CON + 6 * NEQR + MAX_LIM + 8)

struct SolverShared {
  double Lcol[MAX_NB][16];  // Cholesky: current block column, by block row
  double Ldiag[16];         // Cholesky: factor of the current diagonal block
  double Ldinv[4];          // Cholesky: reciprocals of its diagonal
  double a0[MAX_NVP];    // qacc_smooth
  double a[MAX_NVP];     // current qacc
  double res[MAX_NVP];   // a - a0
  double Mres[MAX_NVP];  // M res
  double grad[MAX_NVP];
  double srch[MAX_NVP];
  double Ms[MAX_NVP];
  double acc[MAX_NVP];
  double tmp[MAX_NVP];
  union {
    double jc[RCHUNK][MAX_NVP];  // Hessian: scaled Jacobian chunk
    double cw[6 * MAX_CON];      // J^T w: contact wrenches (sensors: the same)
  };
  double jrho[RCHUNK][12];     // chunk rows: the two body-side 6-vectors
  double jcoef[RCHUNK][2];     // chunk rows: dof-term coefficients
  double jw[RCHUNK];           // chunk row weights sqrt(D) (active rows)
  double jsg[RCHUNK];          // chunk row signs (incremental Hessian: +1 added, -1 removed)
  double bv[6 * MAX_BODY];     // body velocities of a dof vector / subtree sums (sensors: cacc)
  union {
    double bf[6 * MAX_BODY];     // body forces (sensors: cfrc)
    int16_t hsel[HSEL_CAP];      // Hessian build: the rows it adds / takes back, row order (bit 15: take back)
  };
  double cdof[6 * MAX_NVP];    // motion axes of the dofs (from the front kernel)
  double cinert[10 * MAX_BODY];
  double red[8];
  int ired[8];
  int jb[RCHUNK][2];           // chunk rows: the two bodies
  int jlist[RCHUNK];           // chunk rows with a nonzero weight, in row order
  int jn;
  int jd[RCHUNK][2];           // chunk rows: dof terms (-1: none)
  double eqrho[NEQR][12];      // equality rows: body-side 6-vectors, dof coefficients,
  double eqcoef[NEQR][2];      //   bodies, dofs (-1: none) -- staged once per launch
  int16_t eqb[NEQR][2];
  int16_t eqd[NEQR][2];
  int16_t ccb[MAX_CON][2];     // contact bodies (b1, b2)
  // per-body list of the wrenches J^T w collects, in contact order then equality-row order:
  // entry 2q (+, body = b2 of contact q), 2q + 1 (-, b1), EQ_TAG + 2s + side (equality row s)
  int16_t blist[2 * MAX_CON + 2 * NEQR];
  int16_t boff[MAX_BODY + 1];
  int16_t lim[MAX_LIM];        // limit rows: 2 * dof + (1 if the row's sign is -1)
  int anc[MAX_BODY];           // tree-pass ancestor pointers
  int16_t par[MAX_BODY];       // body parents
  int16_t send[MAX_BODY];      // end of each body's DFS subtree id range
  int16_t kb[MAX_NVP];         // dof -> body
};
static_assert(sizeof(int16_t) * HSEL_CAP <= sizeof(double) * 6 * MAX_BODY,
              "the Hessian row-selection list must fit inside its union partner bf");

// a value the compiler cannot see through (so addresses derived from it are not hoisted out of
// the loop it is read in); RMBX_SOLVER_HOIST restores the hoisting for the A/B
// (scripts/build_variant.py hoist)
__device__ __forceinline__ int opaque_int(int v) {
#ifndef RMBX_SOLVER_HOIST
  asm volatile("" : "+v"(v));
#endif
  return v;
}

// X[6b..] <- sum of the increments X over the path world .. b (solver block; parents from LDS)
__device__ void tree_prefix6_s(SolverShared& S, int nbody, int rounds, double* X, int b) {
  if (b < nbody) S.anc[b] = b == 0 ? -1 : S.par[b];
  lds_sync();
  for (int round = 0; round < rounds; round++) {  // ceil(log2(tree depth + 1)) pointer jumps
    const int a = b < nbody ? S.anc[b] : -1;
    const bool act = a >= 0;
    double v[6];
    int an = -1;
    if (act) {
      for (int i = 0; i < 6; i++) v[i] = X[6 * a + i] + X[6 * b + i];
      an = S.anc[a];
    }
    lds_sync();
    if (act) {
      for (int i = 0; i < 6; i++) X[6 * b + i] = v[i];
      S.anc[b] = an;
    }
    lds_sync();
  }
}

__device__ __forceinline__ void blk_coords(int t, int* bi, int* bj) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) i++;
  while (i * (i + 1) / 2 > t) i--;
  *bi = i;
  *bj = t - i * (i + 1) / 2;
}

__device__ __forceinline__ double block_sum(double v, SolverShared& S, int tid) {
  v = wave_sum(v);
  lds_sync();
  if ((tid & 63) == 0) S.red[tid >> 6] = v;
  lds_sync();
  return S.red[0] + S.red[1] + S.red[2] + S.red[3];
}
// two / three sums in one reduction (same summation order as block_sum: bit-identical)
__device__ __forceinline__ void block_sum2(double& a, double& b, SolverShared& S, int tid) {
  a = wave_sum(a);
  b = wave_sum(b);
  lds_sync();
  if ((tid & 63) == 0) {
    S.red[tid >> 6] = a;
    S.red[4 + (tid >> 6)] = b;
  }
  lds_sync();
  a = S.red[0] + S.red[1] + S.red[2] + S.red[3];
  b = S.red[4] + S.red[5] + S.red[6] + S.red[7];
}
__device__ __forceinline__ void block_sum3(double& a, double& b, int& c, SolverShared& S, int tid) {
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum_i(c);
  lds_sync();
  if ((tid & 63) == 0) {
    S.red[tid >> 6] = a;
    S.red[4 + (tid >> 6)] = b;
    S.ired[tid >> 6] = c;
  }
  lds_sync();
  a = S.red[0] + S.red[1] + S.red[2] + S.red[3];
  b = S.red[4] + S.red[5] + S.red[6] + S.red[7];
  c = S.ired[0] + S.ired[1] + S.ired[2] + S.ired[3];
}
__device__ __forceinline__ int block_sum_i(int v, SolverShared& S, int tid) {
  v = wave_sum_i(v);
  lds_sync();
  if ((tid & 63) == 0) S.ired[tid >> 6] = v;
  lds_sync();
  return S.ired[0] + S.ired[1] + S.ired[2] + S.ired[3];
}

// 4x4 in-place lower Cholesky (row-major)
// 4x4 Cholesky in place (lower); inv[j] = 1 / L_jj.  1/sqrt comes from v_rsq_f64 refined by
// two Newton steps (a shorter dependent chain than sqrt followed by a division, on the
// factorisation's critical path)
__device__ __forceinline__ void potrf4(double* a, double* inv) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    double s = a[4 * j + j];
#pragma unroll
    for (int k = 0; k < j; k++) s -= a[4 * j + k] * a[4 * j + k];
    const double sc = s > RMBX_MINVAL ? s : RMBX_MINVAL;
    double y = __builtin_amdgcn_rsq(sc);
    const double hs = 0.5 * sc;
    y = y * fma(-hs * y, y, 1.5);
    y = y * fma(-hs * y, y, 1.5);
    a[4 * j + j] = sc * y;
    inv[j] = y;
#pragma unroll
    for (int i = j + 1; i < 4; i++) {
      double t = a[4 * i + j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= a[4 * i + k] * a[4 * j + k];
      a[4 * i + j] = t * y;
    }
#pragma unroll
    for (int k = j + 1; k < 4; k++) a[4 * j + k] = 0;
  }
}
// a := a * L^-T  (L lower 4x4, inv = 1 / diag(L) from potrf4)
__device__ __forceinline__ void trsm4(double* a, const double* L, const double* inv) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      double t = a[4 * r + c];
#pragma unroll
      for (int k = 0; k < c; k++) t -= a[4 * r + k] * L[4 * c + k];
      a[4 * r + c] = t * inv[c];
    }
  }
}

// Distributed block Cholesky: thread t < nblk owns block (bi, bj) in a[16].  Lookahead: the
// owner of diagonal block k+1 factors it right after its own step-k update (every update of
// that block is its own), so a step costs two barriers and the potrf overlaps the other updates.
__device__ void blk_cholesky(double* a, int bi, int bj, bool own, int NB, SolverShared& S) {
  if (own && bi == 0 && bj == 0) {
    double inv[4];
    potrf4(a, inv);
#pragma unroll
    for (int q = 0; q < 16; q++) S.Ldiag[q] = a[q];
#pragma unroll
    for (int q = 0; q < 4; q++) S.Ldinv[q] = inv[q];
  }
  for (int k = 0; k < NB; k++) {
    lds_sync();
    if (own && bj == k && bi > k) {
      trsm4(a, S.Ldiag, S.Ldinv);
#pragma unroll
      for (int q = 0; q < 16; q++) S.Lcol[bi][q] = a[q];
    }
    lds_sync();
    if (own && bj > k) {
      const double* Li = S.Lcol[bi];
      const double* Lj = S.Lcol[bj];
#pragma unroll
      for (int p = 0; p < 4; p++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
          double t = a[4 * p + q];
#pragma unroll
          for (int r = 0; r < 4; r++) t -= Li[4 * p + r] * Lj[4 * q + r];
          a[4 * p + q] = t;
        }
      if (bi == k + 1 && bj == k + 1) {
        double inv[4];
        potrf4(a, inv);
#pragma unroll
        for (int q = 0; q < 16; q++) S.Ldiag[q] = a[q];  // read after the next barrier
#pragma unroll
        for (int q = 0; q < 4; q++) S.Ldinv[q] = inv[q];
      }
    }
  }
  lds_sync();
}

// y_k = L_kk^-1 S.acc[4k..4k+3] in place (inv = reciprocals of diag(L_kk) from potrf4)
__device__ __forceinline__ void fwd4(const double* a, const double* inv, double* y) {
  double v[4];
#pragma unroll
  for (int p = 0; p < 4; p++) {
    double t = y[p];
#pragma unroll
    for (int k = 0; k < p; k++) t -= a[4 * p + k] * v[k];
    v[p] = t * inv[p];
  }
#pragma unroll
  for (int p = 0; p < 4; p++) y[p] = v[p];
}

// blk_cholesky with the forward substitution of b folded in: on return the blocks hold L and
// S.acc holds y = L^-1 b (b: LDS, length NVP).  No extra barriers: in each step's trsm phase the
// owners of column k also eliminate y_k from their rows of the right-hand side, and the owner of
// the next diagonal block solves its block of y right after factoring it.
__device__ void blk_cholesky_fwd(double* a, int bi, int bj, bool own, int NB, const double* b, SolverShared& S,
                                 int tid) {
  for (int r = tid; r < 4 * NB; r += SOLVER_THREADS) S.acc[r] = b[r];
  lds_sync();
  if (own && bi == 0 && bj == 0) {
    double inv[4];
    potrf4(a, inv);
#pragma unroll
    for (int q = 0; q < 16; q++) S.Ldiag[q] = a[q];
#pragma unroll
    for (int q = 0; q < 4; q++) S.Ldinv[q] = inv[q];
    fwd4(a, inv, S.acc);
  }
  for (int k = 0; k < NB; k++) {
    lds_sync();
    if (own && bj == k && bi > k) {
      trsm4(a, S.Ldiag, S.Ldinv);
#pragma unroll
      for (int q = 0; q < 16; q++) S.Lcol[bi][q] = a[q];
      const double* y = S.acc + 4 * k;
#pragma unroll
      for (int p = 0; p < 4; p++)
        S.acc[4 * bi + p] -= a[4 * p] * y[0] + a[4 * p + 1] * y[1] + a[4 * p + 2] * y[2] + a[4 * p + 3] * y[3];
    }
    lds_sync();
    if (own && bj > k) {
      const double* Li = S.Lcol[bi];
      const double* Lj = S.Lcol[bj];
#pragma unroll
      for (int p = 0; p < 4; p++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
          double t = a[4 * p + q];
#pragma unroll
          for (int r = 0; r < 4; r++) t -= Li[4 * p + r] * Lj[4 * q + r];
          a[4 * p + q] = t;
        }
      if (bi == k + 1 && bj == k + 1) {
        double inv[4];
        potrf4(a, inv);
#pragma unroll
        for (int q = 0; q < 16; q++) S.Ldiag[q] = a[q];  // read after the next barrier
#pragma unroll
        for (int q = 0; q < 4; q++) S.Ldinv[q] = inv[q];
        fwd4(a, inv, S.acc + 4 * (k + 1));
      }
    }
  }
  lds_sync();
}

// x = L^-T S.acc (the backward half of blk_solve; S.acc = L^-1 b from blk_cholesky_fwd)
__device__ void blk_solve_back(const double* a, int bi, int bj, bool own, int NB, double* x, SolverShared& S,
                               int tid) {
  for (int i = NB - 1; i >= 0; i--) {
    if (own && bi == i && bj == i) {
      double xx[4], inv[4];
#pragma unroll
      for (int p = 0; p < 4; p++) inv[p] = 1.0 / a[4 * p + p];
#pragma unroll
      for (int p = 3; p >= 0; p--) {
        double t = S.acc[4 * i + p];
#pragma unroll
        for (int k = p + 1; k < 4; k++) t -= a[4 * k + p] * xx[k];
        xx[p] = t * inv[p];
      }
#pragma unroll
      for (int p = 0; p < 4; p++) S.acc[4 * i + p] = xx[p];
    }
    lds_sync();
    if (own && bi == i && bj < i) {
      const double* xi = S.acc + 4 * i;
#pragma unroll
      for (int q = 0; q < 4; q++)
        S.acc[4 * bj + q] -= a[q] * xi[0] + a[4 + q] * xi[1] + a[8 + q] * xi[2] + a[12 + q] * xi[3];
    }
    lds_sync();
  }
  for (int r = tid; r < 4 * NB; r += SOLVER_THREADS) x[r] = S.acc[r];
  lds_sync();
}

// x = (L L^T)^-1 b ; b, x in LDS (length NVP, may alias); uses S.acc
__device__ void blk_solve(const double* a, int bi, int bj, bool own, int NB, const double* b,
                          double* x, SolverShared& S, int tid) {
  const int NVP = 4 * NB;
  for (int r = tid; r < NVP; r += SOLVER_THREADS) S.acc[r] = b[r];
  lds_sync();
  // forward: y_j = L_jj^-1 (acc_j); acc_i -= L_ij y_j
  for (int j = 0; j < NB; j++) {
    if (own && bi == j && bj == j) {
      double y[4], inv[4];
#pragma unroll
      for (int p = 0; p < 4; p++) inv[p] = 1.0 / a[4 * p + p];
#pragma unroll
      for (int p = 0; p < 4; p++) {
        double t = S.acc[4 * j + p];
#pragma unroll
        for (int k = 0; k < p; k++) t -= a[4 * p + k] * y[k];
        y[p] = t * inv[p];
      }
#pragma unroll
      for (int p = 0; p < 4; p++) S.acc[4 * j + p] = y[p];
    }
    lds_sync();
    if (own && bj == j && bi > j) {
      const double* y = S.acc + 4 * j;
#pragma unroll
      for (int p = 0; p < 4; p++)
        S.acc[4 * bi + p] -= a[4 * p] * y[0] + a[4 * p + 1] * y[1] + a[4 * p + 2] * y[2] + a[4 * p + 3] * y[3];
    }
    lds_sync();
  }
  // backward: x_i = L_ii^-T acc_i ; acc_j -= L_ij^T x_i
  for (int i = NB - 1; i >= 0; i--) {
    if (own && bi == i && bj == i) {
      double xx[4], inv[4];
#pragma unroll
      for (int p = 0; p < 4; p++) inv[p] = 1.0 / a[4 * p + p];
#pragma unroll
      for (int p = 3; p >= 0; p--) {
        double t = S.acc[4 * i + p];
#pragma unroll
        for (int k = p + 1; k < 4; k++) t -= a[4 * k + p] * xx[k];
        xx[p] = t * inv[p];
      }
#pragma unroll
      for (int p = 0; p < 4; p++) S.acc[4 * i + p] = xx[p];
    }
    lds_sync();
    if (own && bi == i && bj < i) {
      const double* xi = S.acc + 4 * i;
#pragma unroll
      for (int q = 0; q < 4; q++)
        S.acc[4 * bj + q] -= a[q] * xi[0] + a[4 + q] * xi[1] + a[8 + q] * xi[2] + a[12 + q] * xi[3];
    }
    lds_sync();
  }
  for (int r = tid; r < NVP; r += SOLVER_THREADS) x[r] = S.acc[r];
  lds_sync();
}

// load this thread's block of the packed mass matrix (16 contiguous doubles)
__device__ __forceinline__ void load_blockp(const double* Mb, int t, double* a) {
  const double2* src = reinterpret_cast<const double2*>(Mb + 16 * (size_t)t);
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const double2 v = src[q];
    a[2 * q] = v.x;
    a[2 * q + 1] = v.y;
  }
}

struct SolverCtx {
  const rmbx_model* m;
  const double* aref;
  const double* D;
  const double* sqD;
  const double* rho;
  const int32_t* type;
  const int32_t* kind;
  const int32_t* obj;
  const double* cpos;
  const double* cframe;
  const double* cmu;
  const int32_t* cb1;
  const int32_t* cb2;
  const int32_t* ccondim;
  const int32_t* cefcadr;
  const double* eq_rho;
  const double* eq_coef;
  const int32_t* eq_body;
  const int32_t* eq_dof;
  double* jar;
  double* Js;
  double* force;
  double* wrow;  // per-row weights handed to jac_tmul
  unsigned long long* prof;  // diagnostic cycle slots (or NULL)
  int nefc, ne, nlim, ncon, nv, NB, tid, tree_rounds;
};
#define CPROF(k)                                  \
  if (c.prof) {                                   \
    lds_sync();                                   \
    const unsigned long long t_ = stamp();        \
    if (c.tid == 0) c.prof[k] += t_ - tp_;        \
    tp_ = t_;                                     \
  }

// body velocities of the dof vector x (LDS): S.bv[b] = sum over the dofs on b's chain of
// cdof_k x_k -- per-body increments, then the pointer-jumping prefix over the tree
__device__ void body_vel(const SolverCtx& c, const double* x, SolverShared& S) {
  const rmbx_model& m = *c.m;
  const int b = c.tid;
  unsigned long long tp_ = c.prof ? stamp() : 0;
  if (b < m.nbody) {
    double v[6] = {0, 0, 0, 0, 0, 0};
    if (b > 0)
      for (int k = m.body_dofadr[b]; k < m.body_dofadr[b] + m.body_dofnum[b]; k++) {
        const double xk = x[k];
#pragma unroll
        for (int i = 0; i < 6; i++) v[i] += S.cdof[6 * k + i] * xk;
      }
#pragma unroll
    for (int i = 0; i < 6; i++) S.bv[6 * b + i] = v[i];
  }
  lds_sync();
  CPROF(28)
  tree_prefix6_s(S, m.nbody, c.tree_rounds, S.bv, b);
  CPROF(29)
}

// (J x)_r from the body velocities of x (S.bv) and x itself
__device__ __forceinline__ double row_dot(const SolverCtx& c, int r, const SolverShared& S, const double* x) {
  const int kd = c.kind[r], k = kd & 7, sub = kd >> 3, o = c.obj[r];
  if (k == ROW_CONTACT) {
    const double* rho = c.rho + 6 * (size_t)r;
    const double* v2 = S.bv + 6 * S.ccb[o][1];
    const double* v1 = S.bv + 6 * S.ccb[o][0];
    double d[6];
#pragma unroll
    for (int i = 0; i < 6; i++) d[i] = v2[i] - v1[i];
    return dot6t(rho, d);
  }
  if (k == ROW_LIMIT) return sub ? -x[o] : x[o];
  const double* rho = S.eqrho[o];
  double v = dot6t(rho, S.bv + 6 * S.eqb[o][0]) + dot6t(rho + 6, S.bv + 6 * S.eqb[o][1]);
  const int d1 = S.eqd[o][0], d2 = S.eqd[o][1];
  if (d1 >= 0) v += S.eqcoef[o][0] * x[d1];
  if (d2 >= 0) v += S.eqcoef[o][1] * x[d2];
  return v;
}

// S.bv[b] <- sum of S.bf over b's subtree (b > 0; the world's entry is left alone).  Bodies are
// in DFS preorder, so a subtree is the id range [b, send[b]): wave 0 (lane = body) takes an
// inclusive prefix scan over the ids (6 shuffle rounds) and each subtree sum is the difference
// of two prefix values -- instead of a loop over up to nbody descendants per lane.
__device__ __forceinline__ void subtree_sums(const SolverCtx& c, SolverShared& S) {
  const int b = c.tid;
  const int nb = c.m->nbody;
  if (b < 64) {
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = (b > 0 && b < nb) ? S.bf[6 * b + i] : 0.0;  // (world: unused)
    // source lanes from an opaque copy of the lane index: __shfl_up's six lane-address
    // computations are otherwise hoisted to the kernel top and spilled at 128 registers
    const int lane = opaque_int(b);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int src = (lane - off) << 2;  // (b < off: a wrapped lane, discarded below)
#pragma unroll
      for (int i = 0; i < 6; i++) {
        const unsigned long long u = __double_as_longlong(x[i]);
        const int lo = __builtin_amdgcn_ds_bpermute(src, (int)u);
        const int hi = __builtin_amdgcn_ds_bpermute(src, (int)(u >> 32));
        const double y = __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
        if (b >= off) x[i] += y;
      }
    }
    if (b < nb)
#pragma unroll
      for (int i = 0; i < 6; i++) S.bf[6 * b + i] = x[i];
  }
  lds_sync();
  if (b > 0 && b < nb) {
    const double* hi = S.bf + 6 * (S.send[b] - 1);
    const double* lo = S.bf + 6 * (b - 1);
#pragma unroll
    for (int i = 0; i < 6; i++) S.bv[6 * b + i] = hi[i] - lo[i];
  }
  lds_sync();
}

// y = M x without M: body forces cinert_b V_b(x) summed over subtrees, projected on the dofs
// (plus armature).  Expects S.bv = body_vel(x); S.bv is consumed (holds the subtree sums after).
__device__ void mass_tail(const SolverCtx& c, const double* x, double* y, SolverShared& S) {
  const rmbx_model& m = *c.m;
  const int tid = c.tid;
  unsigned long long tp_ = c.prof ? stamp() : 0;
  if (tid > 0 && tid < m.nbody) {
    double f[6];
    inert_mul(S.cinert + 10 * tid, S.bv + 6 * tid, f);
#pragma unroll
    for (int i = 0; i < 6; i++) S.bf[6 * tid + i] = f[i];
  }
  lds_sync();
  subtree_sums(c, S);
  for (int k = tid; k < 4 * c.NB; k += SOLVER_THREADS)
    y[k] = k < c.nv ? dot6(S.cdof + 6 * k, S.bv + 6 * S.kb[k]) + m.dof_armature[k] * x[k] : 0.0;
  lds_sync();
  CPROF(30)
}

// out = J^T w (w: per-row weights in global, out: LDS dof vector).  Contact rows fold into one
// wrench per contact about the origin ((p x f, f), f = sum of w_r dir_r), bodies collect their
// contacts' (+ on b2, - on b1) and equality rows' wrenches in a fixed order, subtree sums carry
// them to the dofs, and the limit / joint-equality dof terms are added per dof.
__device__ void jac_tmul(const SolverCtx& c, const double* w, double* out, SolverShared& S) {
  const rmbx_model& m = *c.m;
  const int tid = c.tid;
  double* cw = S.cw;
  double* wst = &S.jrho[0][0];  // w of the equality and limit rows (NEQR + MAX_LIM <= 16 * 12)
  __syncthreads();  // w was written row-per-thread through global memory: full fence
  unsigned long long tp_ = c.prof ? stamp() : 0;
  // contact wrench about the origin = sum over the contact's rows of w_r (p x dir_r, dir_r)
  for (int q = tid; q < c.ncon; q += SOLVER_THREADS) {
    const int r0 = c.cefcadr[q];
    const int cnt = min(c.ccondim[q] == 1 ? 1 : 4, c.nefc - r0);
    double f[6] = {0, 0, 0, 0, 0, 0};
    for (int t = 0; t < cnt; t++) {
      const double wr = w[r0 + t];
      const double* rho = c.rho + 6 * (size_t)(r0 + t);
#pragma unroll
      for (int i = 0; i < 6; i++) f[i] += wr * rho[i];
    }
#pragma unroll
    for (int i = 0; i < 6; i++) cw[6 * q + i] = f[i];
  }
  for (int i = tid; i < c.ne + c.nlim; i += SOLVER_THREADS) wst[i] = w[i];
  lds_sync();
  CPROF(24)
  if (tid > 0 && tid < m.nbody) {
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int l = S.boff[tid]; l < S.boff[tid + 1]; l++) {
      const int en = S.blist[l];
      if (en < EQ_TAG) {
        const double* wq = cw + 6 * (en >> 1);
        const double sg = (en & 1) ? -1.0 : 1.0;
#pragma unroll
        for (int i = 0; i < 6; i++) acc[i] += sg * wq[i];
      } else {
        const int s = (en - EQ_TAG) >> 1;
        const double ws = wst[s];
        const double* rho = S.eqrho[s] + 6 * (en & 1);
#pragma unroll
        for (int i = 0; i < 6; i++) acc[i] += ws * rho[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) S.bf[6 * tid + i] = acc[i];
  }
  lds_sync();
  CPROF(25)
  subtree_sums(c, S);
  CPROF(26)
  for (int k = tid; k < 4 * c.NB; k += SOLVER_THREADS) {
    double v = 0.0;
    if (k < c.nv) {
      v = dot6(S.cdof + 6 * k, S.bv + 6 * S.kb[k]);
      for (int s = 0; s < c.ne; s++) {
        if (S.eqd[s][0] == k) v += S.eqcoef[s][0] * wst[s];
        if (S.eqd[s][1] == k) v += S.eqcoef[s][1] * wst[s];
      }
      for (int i = 0; i < c.nlim; i++) {
        const int l = S.lim[i];
        if ((l >> 1) == k) v += (l & 1) ? -wst[c.ne + i] : wst[c.ne + i];
      }
    }
    out[k] = v;
  }
  lds_sync();
  CPROF(27)
}

// cost at x: sets jar (J x - aref), S.res, S.Mres; returns cost
__device__ double solver_cost(const SolverCtx& c, const double* x, SolverShared& S) {
  const int tid = c.tid;
  for (int k = tid; k < 4 * c.NB; k += SOLVER_THREADS) S.res[k] = k < c.nv ? x[k] - S.a0[k] : 0.0;
  lds_sync();
  body_vel(c, S.res, S);
  mass_tail(c, S.res, S.Mres, S);
  double part = 0;
  for (int k = tid; k < c.nv; k += SOLVER_THREADS) part += S.res[k] * S.Mres[k];
  body_vel(c, x, S);
  double cpart = 0;
  for (int r = tid; r < c.nefc; r += SOLVER_THREADS) {
    const double jar = row_dot(c, r, S, x) - c.aref[r];
    c.jar[r] = jar;
    if (c.type[r] == 0 || jar < 0) cpart += 0.5 * c.D[r] * jar * jar;
  }
  block_sum2(part, cpart, S, tid);
  return 0.5 * part + cpart;
}

// constraint part of the cost at x: jar = J x - aref (c.jar), sum of 0.5 D jar^2 over active rows
__device__ double rows_cost(const SolverCtx& c, const double* x, SolverShared& S) {
  body_vel(c, x, S);
  double cpart = 0;
  for (int r = c.tid; r < c.nefc; r += SOLVER_THREADS) {
    const double jar = row_dot(c, r, S, x) - c.aref[r];
    c.jar[r] = jar;
    if (c.type[r] == 0 || jar < 0) cpart += 0.5 * c.D[r] * jar * jar;
  }
  return block_sum(cpart, S, c.tid);
}

// Gradient S.grad = M res + J^T (D_act jar) and the row activity flags; *changed = the active
// set differs from the one last factorised.  Returns |g|^2.
__device__ double solver_grad(const SolverCtx& c, int32_t* act_flags, SolverShared& S, bool* changed) {
  const int tid = c.tid, nv = c.nv, NVP = 4 * c.NB;
  int diff = 0;
  for (int r = tid; r < c.nefc; r += SOLVER_THREADS) {
    const double jar = c.jar[r];
    const int act = (c.type[r] == 0 || jar < 0) ? 1 : 0;
    c.wrow[r] = act ? c.D[r] * jar : 0.0;
    diff |= act != act_flags[r];
    act_flags[r] = act;
  }
  *changed = block_sum_i(diff, S, tid) != 0;  // (barrier inside)
  jac_tmul(c, c.wrow, S.acc, S);
  double gn = 0;
  if (tid < nv) {
    const double g = S.Mres[tid] + S.acc[tid];
    S.grad[tid] = g;
    gn = g * g;
  } else if (tid < NVP) {
    S.grad[tid] = 0;
  }
  return block_sum(gn, S, tid);
}

// Hessian blocks a = M + J^T D_act J (active rows only), in RCHUNK-row chunks of J computed in
// LDS from the row descriptions and cdof (scaled by sqrt(D)).  The first build of a substep
// starts from M and saves H with its row set (hsave, hess_flags); later ones start from that
// saved H and only add / subtract the rows whose active flag differs from that set (the net
// change; neither the copy nor the set is rewritten) -- MuJoCo's Newton solver likewise updates
// its Hessian incrementally instead of rebuilding it.

__device__ void solver_hessian(const SolverCtx& c, const double* Mb, const int32_t* act_flags, int32_t* hess_flags,
                               double* hsave, bool incremental, double* a, int bi, int bj, bool own,
                               SolverShared& S) {
  const int tid = c.tid, nv = c.nv, NVP = 4 * c.NB;
  __syncthreads();  // act_flags were written row-per-thread through global memory: full fence
  unsigned long long tp_ = c.prof ? stamp() : 0;
  if (own) {
    if (incremental) {
#pragma unroll
      for (int q = 0; q < 16; q++) a[q] = hsave[16 * tid + q];
    } else {
      load_blockp(Mb, tid, a);
    }
  }
  // select the rows this build adds (active now; an incremental build: newly active) or takes
  // back (an incremental build: no longer active) -- one pass over all rows, a block-wide ballot
  // scan into S.hsel in row order -- so the chunks below only describe and expand selected rows
  // (an incremental build after a small active-set change is one chunk, not nefc / RCHUNK)
  int nsel = 0;
  for (int base = 0; base < c.nefc; base += SOLVER_THREADS) {
    const int r = base + tid;
    bool sel = false, back = false;
    if (r < c.nefc) {
      const int act = act_flags[r];
      if (incremental) {
        sel = act != hess_flags[r];
        back = !act;
      } else {
        sel = act != 0;
      }
      if (!incremental) hess_flags[r] = act;
    }
    const unsigned long long bal = __ballot(sel);
    const int wv = tid >> 6;
    lds_sync();
    if ((tid & 63) == 0) S.ired[wv] = __popcll(bal);
    lds_sync();
    int off = nsel;
    for (int q = 0; q < wv; q++) off += S.ired[q];
    if (sel) S.hsel[off + __popcll(bal & ((1ull << (tid & 63)) - 1))] = (int16_t)(back ? (r | 0x8000) : r);
    nsel += S.ired[0] + S.ired[1] + S.ired[2] + S.ired[3];
  }
  for (int s0 = 0; s0 < nsel; s0 += RCHUNK) {
    const int nr = min(RCHUNK, nsel - s0);
    lds_sync();
    if (tid < RCHUNK) {
      double w = 0.0, sg = 1.0;
      if (tid < nr) {
        const int hs = (uint16_t)S.hsel[s0 + tid];
        const int r = hs & 0x7fff;
        const double Dr = c.sqD[r];
        const int kd = c.kind[r], o = c.obj[r];
        w = Dr;
        sg = (hs & 0x8000) ? -1.0 : 1.0;
        if (w != 0.0) {
          // describe row r: sides (body, 6-vector) and dof terms
          const int k = kd & 7, sub = kd >> 3;
          double* rho = S.jrho[tid];
          int b1 = 0, b2 = 0, d1 = -1, d2 = -1;
          double c1 = 0, c2 = 0;
          if (k == ROW_CONTACT) {
            const double* src = c.rho + 6 * (size_t)r;
            for (int i = 0; i < 6; i++) {
              const double v = src[i];
              rho[6 + i] = v;
              rho[i] = -v;
            }
            b1 = S.ccb[o][0];
            b2 = S.ccb[o][1];
          } else if (k == ROW_LIMIT) {
            for (int i = 0; i < 12; i++) rho[i] = 0.0;
            d1 = o;
            c1 = sub ? -1.0 : 1.0;
          } else {
            for (int i = 0; i < 12; i++) rho[i] = S.eqrho[o][i];
            b1 = S.eqb[o][0];
            b2 = S.eqb[o][1];
            d1 = S.eqd[o][0];
            d2 = S.eqd[o][1];
            c1 = S.eqcoef[o][0];
            c2 = S.eqcoef[o][1];
          }
          S.jb[tid][0] = b1;
          S.jb[tid][1] = b2;
          S.jd[tid][0] = d1;
          S.jd[tid][1] = d2;
          S.jcoef[tid][0] = c1;
          S.jcoef[tid][1] = c2;
        }
      }
      S.jw[tid] = w;
      S.jsg[tid] = sg;
      // compact the rows that update the Hessian (wave 0, lanes < RCHUNK)
      const unsigned long long nz = __ballot(w != 0.0) & ((1ull << RCHUNK) - 1);
      if (w != 0.0) S.jlist[__popcll(nz & ((1ull << tid) - 1))] = tid;
      if (tid == 0) S.jn = __popcll(nz);
    }
    lds_sync();
    CPROF(19)
    bool any = false;
#pragma unroll
    for (int k = 0; k < RCHUNK; k++) any |= S.jw[k] != 0.0;
    if (!any) continue;  // uniform: every thread read the same flags
    // J_rk = [k on chain(b1)] cdof_k . rho1 + [k on chain(b2)] cdof_k . rho2 + dof terms; a
    // contact's two sides are exact negatives, so dofs on both chains give exactly 0
    for (int e = tid; e < RCHUNK * NVP; e += SOLVER_THREADS) {
      const int rr = e / NVP, k = e - rr * NVP;
      double v = 0.0;
      const double w = S.jw[rr];
      if (rr < nr && k < nv && w != 0.0) {
        const int kb = S.kb[k], kend = S.send[kb];
        const int b1 = S.jb[rr][0], b2 = S.jb[rr][1];
        const double* Sk = S.cdof + 6 * k;
        if (kb <= b1 && b1 < kend) v += dot6t(Sk, S.jrho[rr]);
        if (kb <= b2 && b2 < kend) v += dot6t(Sk, S.jrho[rr] + 6);
        if (S.jd[rr][0] == k) v += S.jcoef[rr][0];
        if (S.jd[rr][1] == k) v += S.jcoef[rr][1];
        v *= w;
      }
      S.jc[rr][k] = v;
    }
    lds_sync();
    CPROF(31)
    if (own) {
      // rank-1 updates over the chunk's nonzero rows; the next row's slices are loaded before
      // this row's 16 FMAs so the LDS latency hides under them
      const int n = S.jn;
      int rr = n > 0 ? S.jlist[0] : 0;
      double2 ia = *reinterpret_cast<const double2*>(S.jc[rr] + 4 * bi);
      double2 ib = *reinterpret_cast<const double2*>(S.jc[rr] + 4 * bi + 2);
      double2 ja = *reinterpret_cast<const double2*>(S.jc[rr] + 4 * bj);
      double2 jb = *reinterpret_cast<const double2*>(S.jc[rr] + 4 * bj + 2);
      double sg = S.jsg[rr];  // -1: a row that left the active set is taken back out
      for (int l = 0; l < n; l++) {
        const int rn = S.jlist[l + 1 < n ? l + 1 : l];
        const double2 ia2 = *reinterpret_cast<const double2*>(S.jc[rn] + 4 * bi);
        const double2 ib2 = *reinterpret_cast<const double2*>(S.jc[rn] + 4 * bi + 2);
        const double2 ja2 = *reinterpret_cast<const double2*>(S.jc[rn] + 4 * bj);
        const double2 jb2 = *reinterpret_cast<const double2*>(S.jc[rn] + 4 * bj + 2);
        const double sg2 = S.jsg[rn];
        const double i0 = sg * ia.x, i1 = sg * ia.y, i2 = sg * ib.x, i3 = sg * ib.y;
        const double j0 = ja.x, j1 = ja.y, j2 = jb.x, j3 = jb.y;
        a[0] += i0 * j0; a[1] += i0 * j1; a[2] += i0 * j2; a[3] += i0 * j3;
        a[4] += i1 * j0; a[5] += i1 * j1; a[6] += i1 * j2; a[7] += i1 * j3;
        a[8] += i2 * j0; a[9] += i2 * j1; a[10] += i2 * j2; a[11] += i2 * j3;
        a[12] += i3 * j0; a[13] += i3 * j1; a[14] += i3 * j2; a[15] += i3 * j3;
        ia = ia2;
        ib = ib2;
        ja = ja2;
        jb = jb2;
        sg = sg2;
      }
    }
  }
  if (own && !incremental) {
#pragma unroll
    for (int q = 0; q < 16; q++) hsave[16 * tid + q] = a[q];
  }
  lds_sync();
}

#define SPROF(k)                                  \
  if (prof) {                                     \
    lds_sync();                                   \
    const unsigned long long t_ = stamp();        \
    if (tid == 0) prof[k] += t_ - tp;             \
    tp = t_;                                      \
  }

__device__ int solver_newton(Env& e, SolverShared& S, double* a, int bi, int bj, bool own,
                             int ncon, int nefc, int ne, int nlim, int tree_rounds, int tid_,
                             unsigned long long* prof) {
  const int tid = tid_;
  const rmbx_model& m = *e.m;
  unsigned long long tp = prof ? stamp() : 0;
  const int nv = m.nv, NB = (nv + 3) / 4, NVP = 4 * NB;
  const double* Mb = W(Mblk);
  SolverCtx c;
  c.m = e.m;
  c.aref = W(efc_aref);
  c.D = W(efc_D);
  c.sqD = W(efc_sqD);
  c.rho = W(efc_rho);
  c.type = WI(efc_type);
  c.kind = WI(efc_kind);
  c.obj = WI(efc_obj);
  c.cpos = W(con_pos);
  c.cframe = W(con_frame);
  c.cmu = W(con_mu);
  c.cb1 = WI(con_b1);
  c.cb2 = WI(con_b2);
  c.ccondim = WI(con_condim);
  c.cefcadr = WI(con_efcadr);
  c.eq_rho = W(eqr_rho);
  c.eq_coef = W(eqr_coef);
  c.eq_body = WI(eqr_body);
  c.eq_dof = WI(eqr_dof);
  c.jar = W(efc_jar);
  c.Js = W(efc_Js);
  c.force = W(efc_force);
  c.wrow = W(efc_tmp);
  c.prof = prof;
  c.tree_rounds = tree_rounds;
  c.nefc = nefc;
  c.ne = ne;
  c.nlim = nlim;
  c.ncon = ncon;
  c.nv = nv;
  c.NB = NB;
  c.tid = tid;
  // qacc_smooth = M^-1 qfrc_smooth
  if (own) load_blockp(Mb, tid, a);
  for (int k = tid; k < NVP; k += SOLVER_THREADS) S.tmp[k] = k < nv ? W(qfrc_smooth)[k] : 0.0;
  lds_sync();
  blk_cholesky_fwd(a, bi, bj, own, NB, S.tmp, S, tid);
  blk_solve_back(a, bi, bj, own, NB, S.a0, S, tid);
  SPROF(8)
  for (int k = tid; k < NVP; k += SOLVER_THREADS) S.tmp[k] = k < nv ? e.qacc_ws[k] : 0.0;
  lds_sync();
  // warm start vs smooth start (the smooth start has res = 0: only its rows cost anything)
  const double c_ws = solver_cost(c, S.tmp, S);
  double* jar_ws = W(efc_Js);  // (Js is dead until the first line search)
  for (int r = tid; r < nefc; r += SOLVER_THREADS) jar_ws[r] = c.jar[r];
  for (int k = tid; k < NVP; k += SOLVER_THREADS) S.Ms[k] = S.Mres[k];
  lds_sync();
  const double c_sm = rows_cost(c, S.a0, S);
  const bool use_ws = c_ws < c_sm;
  for (int k = tid; k < NVP; k += SOLVER_THREADS) {
    S.a[k] = use_ws ? S.tmp[k] : S.a0[k];
    S.res[k] = use_ws ? S.res[k] : 0.0;
    S.Mres[k] = use_ws ? S.Ms[k] : 0.0;
  }
  if (use_ws)
    for (int r = tid; r < nefc; r += SOLVER_THREADS) c.jar[r] = jar_ws[r];
  lds_sync();
  double cost = use_ws ? c_ws : c_sm;
  SPROF(9)
  const double scale = 1.0 / (m.meaninertia * (nv > 1 ? nv : 1));
  int it;
  int32_t* act_flags = WI(efc_act);
  bool have_factor = false;
  for (it = 0; it < m.solver_iterations; it++) {
    // the thread index, re-read opaquely each iteration: otherwise the compiler hoists ~20
    // per-lane 64-bit row/dof addresses (base + 8 tid) out of the loop and, at 128 registers,
    // spills them and reloads them every iteration (one add each to recompute)
    const int tid = opaque_int(tid_);
    c.tid = tid;
    bool changed;
    const double gn = solver_grad(c, act_flags, S, &changed);
    SPROF(10)
    if (scale * sqrt(gn) < m.solver_tolerance) break;
    // H = M + J^T D J over the active rows: built in full at the first iteration (saved with its
    // row set), later as that saved matrix +/- the rows whose activity differs from its set (the
    // net change: a row that came and went is never touched; with the usual two iterations the
    // same sums as a chain of increments). No copy of the factor is kept: when the active set did
    // not change (rare) the same net change is applied again -- a bit-identical matrix -- and
    // refactored, instead of a 19.6 KB factor write after every build that is almost never read.
    // (With one code path after the gradient the solver also compiles without spills at 128
    // registers: the separate reuse-the-factor solve was the last register peak.)
    (void)changed;
    solver_hessian(c, Mb, act_flags, WI(efc_hact), W(hsave), have_factor, a, bi, bj, own, S);
    SPROF(15)
    blk_cholesky_fwd(a, bi, bj, own, NB, S.grad, S, tid);
    blk_solve_back(a, bi, bj, own, NB, S.srch, S, tid);
    have_factor = true;
    SPROF(11)
    for (int k = tid; k < NVP; k += SOLVER_THREADS) S.srch[k] = -S.srch[k];
    lds_sync();
    // J search (rows) and M search from one pass of body velocities of the search direction
    body_vel(c, S.srch, S);
    for (int r = tid; r < nefc; r += SOLVER_THREADS) c.Js[r] = row_dot(c, r, S, S.srch);
    mass_tail(c, S.srch, S.Ms, S);
    double qp = 0, lp = 0;
    for (int k = tid; k < nv; k += SOLVER_THREADS) {
      qp += S.srch[k] * S.Ms[k];
      lp += S.res[k] * S.Ms[k];
    }
    block_sum2(qp, lp, S, tid);
    const double qg = qp, lg = lp;
    // exact line search on the piecewise quadratic (Newton steps on the derivative, bracketed);
    // the test "did any inequality row change side between the last two points" of step ls is
    // folded into the derivative reduction of step ls + 1 (one block reduction per step)
    double alpha = 0, prev = 0, lo = 0, hi = 1e300;
    for (int ls = 0; ls < m.ls_iterations; ls++) {
      double p1 = 0, p2 = 0;
      int changed = 0;
      for (int r = opaque_int(tid); r < nefc; r += SOLVER_THREADS) {
        const double js = c.Js[r], jr = c.jar[r];
        const double x = jr + alpha * js;
        if (c.type[r] == 0 || x < 0) {
          p1 += c.D[r] * x * js;
          p2 += c.D[r] * js * js;
        }
        if (r >= ne) changed |= ((jr + prev * js < 0) != (x < 0));
      }
      block_sum3(p1, p2, changed, S, tid);
      if (ls > 0 && changed == 0) break;
      const double d1 = alpha * qg + lg + p1;
      const double d2 = qg + p2;
      if (d1 == 0) break;
      if (d1 < 0)
        lo = alpha;
      else
        hi = alpha;
      double an = alpha - d1 / d2;
      if (!(an > lo && an < hi)) an = hi < 1e300 ? 0.5 * (lo + hi) : (an > lo ? an : lo);
      prev = alpha;
      alpha = an;
    }
    SPROF(12)
    // move along the search direction; res, M res and jar updated incrementally (as
    // mj_solNewton updates qacc, Ma and efc_Jaref)
    double part = 0, cpart = 0;
    for (int k = opaque_int(tid); k < NVP; k += SOLVER_THREADS) {
      S.a[k] += alpha * S.srch[k];
      S.res[k] += alpha * S.srch[k];
      S.Mres[k] += alpha * S.Ms[k];
      if (k < nv) part += S.res[k] * S.Mres[k];
    }
    for (int r = opaque_int(tid); r < nefc; r += SOLVER_THREADS) {
      const double jar = c.jar[r] + alpha * c.Js[r];
      c.jar[r] = jar;
      if (c.type[r] == 0 || jar < 0) cpart += 0.5 * c.D[r] * jar * jar;
    }
    block_sum2(part, cpart, S, tid);
    const double newcost = 0.5 * part + cpart;
    SPROF(13)
    const double improvement = scale * (cost - newcost);
    cost = newcost;
    if (improvement < m.solver_tolerance) {
      it++;
      break;
    }
  }
  // forces and qfrc_constraint = J^T f
  for (int r = tid; r < nefc; r += SOLVER_THREADS) {
    const double jar = c.jar[r];
    c.force[r] = (c.type[r] == 0 || jar < 0) ? -c.D[r] * jar : 0.0;
  }
  lds_sync();
  jac_tmul(c, c.force, S.acc, S);
  if (tid < nv) {
    W(qfrc_constraint)[tid] = S.acc[tid];
    W(qacc)[tid] = S.a[tid];
  }
  __syncthreads();  // the sensors read qacc body-per-thread: full fence
  SPROF(14)
  return it;
}
// Sensors (mj_rnePostConstraint -> force / torque at sites) in the solver block: body
// accelerations by the LDS tree prefix, contact wrenches (p x F, F) with F the contact's world force
// collected per body from the J^T w lists (body 2 receives -w, body 1 +w, contact order; equality
// rows do not enter), then each sensor site body's subtree sum.
__device__ void solver_sensors(Env& e, SolverShared& S, int ncon, int tree_rounds, int tid) {
  const rmbx_model& m = *e.m;
  if (m.nsensor == 0) return;
  const int nb = m.nbody;
  double* cacc = S.bv;
  double* cfrc = S.bf;
  double* cw = S.cw;
  const double* cvel = W(cvel);
  const double* cdofdot = W(cdofdot);
  if (tid == 0) {
    cacc[0] = cacc[1] = cacc[2] = 0;
    cacc[3] = -m.gravity[0];
    cacc[4] = -m.gravity[1];
    cacc[5] = -m.gravity[2];
  } else if (tid < nb) {
    double a[6] = {0, 0, 0, 0, 0, 0};
    const int da = m.body_dofadr[tid], dn = m.body_dofnum[tid];
    for (int k = da; k < da + dn; k++) {
      for (int i = 0; i < 6; i++) a[i] += cdofdot[6 * k + i] * e.qvel[k];
      for (int i = 0; i < 6; i++) a[i] += S.cdof[6 * k + i] * S.a[k];
    }
    for (int i = 0; i < 6; i++) cacc[6 * tid + i] = a[i];
  }
  lds_sync();
  tree_prefix6_s(S, nb, tree_rounds, cacc, tid);
  if (tid > 0 && tid < nb) {
    double Ia[6], Iv[6], vxIv[6];
    const double* I = S.cinert + 10 * tid;
    const double* v = cvel + 6 * tid;
    inert_mul(I, cacc + 6 * tid, Ia);
    inert_mul(I, v, Iv);
    cross_force(v, Iv, vxIv);
    for (int i = 0; i < 6; i++) cfrc[6 * tid + i] = Ia[i] + vxIv[i];
  }
  for (int c = tid; c < ncon; c += SOLVER_THREADS) {
    double* o = cw + 6 * c;
    const int r0 = WI(con_efcadr)[c];
    if (r0 + (WI(con_condim)[c] == 1 ? 1 : 4) > e.L->nefc_max) {
      for (int i = 0; i < 6; i++) o[i] = 0;
      continue;
    }
    const double* F = W(con_frame) + 9 * c;
    double fn, f1 = 0, f2 = 0;
    const double* f = W(efc_force) + r0;
    if (WI(con_condim)[c] == 1) {
      fn = f[0];
    } else {
      const double mu = W(con_mu)[c];
      fn = f[0] + f[1] + f[2] + f[3];
      f1 = mu * (f[0] - f[1]);
      f2 = mu * (f[2] - f[3]);
    }
    double Fw[3];
    for (int i = 0; i < 3; i++) Fw[i] = fn * F[i] + f1 * F[3 + i] + f2 * F[6 + i];
    cross3(W(con_pos) + 3 * c, Fw, o);
    for (int i = 0; i < 3; i++) o[3 + i] = Fw[i];
  }
  lds_sync();
  if (tid > 0 && tid < nb) {
    double acc[6];
    for (int i = 0; i < 6; i++) acc[i] = cfrc[6 * tid + i];
    for (int l = S.boff[tid]; l < S.boff[tid + 1]; l++) {
      const int en = S.blist[l];
      if (en >= EQ_TAG) continue;
      const double* wq = cw + 6 * (en >> 1);
      if (en & 1)
        for (int i = 0; i < 6; i++) acc[i] += wq[i];
      else
        for (int i = 0; i < 6; i++) acc[i] -= wq[i];
    }
    for (int i = 0; i < 6; i++) cfrc[6 * tid + i] = acc[i];
  }
  lds_sync();
  if (tid < m.nsensor && tid < 2) {
    const int s = tid;
    const int site = m.sensor_site[s];
    const int b = m.site_body[site];
    double f[6];
    for (int i = 0; i < 6; i++) f[i] = cfrc[6 * b + i];
    for (int d = b + 1; d < S.send[b]; d++)  // interaction force = subtree sum
      for (int i = 0; i < 6; i++) f[i] += cfrc[6 * d + i];
    const double* p = W(sxpos) + 3 * site;
    const double* R = W(sxmat) + 9 * site;
    double out[3];
    if (m.sensor_type[s] == RMBX_SENS_FORCE) {
      mattvec3(R, f + 3, out);
    } else {
      double pxf[3], n[3];
      cross3(p, f + 3, pxf);
      for (int i = 0; i < 3; i++) n[i] = f[i] - pxf[i];
      mattvec3(R, n, out);
    }
    for (int i = 0; i < 3; i++) e.sensordata[3 * s + i] = out[i];
  }
  lds_sync();
}

__device__ void solver_integrate(Env& e, SolverShared& S, double* a, int bi, int bj, bool own,
                                 int tid, int sub, const double* hB) {
  const rmbx_model& m = *e.m;
  const int nv = m.nv, NB = (nv + 3) / 4, NVP = 4 * NB;
  const double h = m.timestep;
  if (own) {
    // M + h * (damping + actuator velocity gains): the second term is a model constant built
    // once at create (rmbx_engine_create) in the same packed block order
    load_blockp(W(Mblk), threadIdx.x, a);
    double hb[16];
    load_blockp(hB, threadIdx.x, hb);
#pragma unroll
    for (int q = 0; q < 16; q++) a[q] += hb[q];
  }
  for (int k = tid; k < NVP; k += SOLVER_THREADS)
    S.tmp[k] = k < nv ? W(qfrc_smooth)[k] + W(qfrc_constraint)[k] : 0.0;
  lds_sync();
  // MuJoCo's divergence guard (mj_step -> mj_checkAcc) on the forward (constraint-solver) qacc
  bool bad = false;
  for (int k = tid; k < nv; k += SOLVER_THREADS) {
    const double acc = W(qacc)[k];
    if (!isfinite(acc) || fabs(acc) > 1e10) bad = true;
  }
  blk_cholesky_fwd(a, bi, bj, own, NB, S.tmp, S, tid);
  blk_solve_back(a, bi, bj, own, NB, S.a, S, tid);
  if (block_sum_i(bad ? 1 : 0, S, tid)) {
    // mj_resetData: the model's qpos0, zero velocity, warm start and ctrl, time 0 (ctrl stays 0
    // for the rest of the env-step, as in MuJoCo); stats[3] = the 1-based substep of the reset.
    // MuJoCo then runs mj_forward on the reset state and integrates this substep from it: here
    // the remaining substeps run from the reset state and the engine adds one masked substep
    // after the env-step (launch(): redo pass) for the envs that reset, so each env ends the
    // env-step with its full count of integrated substeps and MuJoCo's time.
    for (int k = tid; k < m.nq; k += SOLVER_THREADS) e.qpos[k] = m.qpos0[k];
    for (int k = tid; k < nv; k += SOLVER_THREADS) {
      e.qvel[k] = 0.0;
      e.qacc_ws[k] = 0.0;
    }
    for (int k = tid; k < m.nu; k += SOLVER_THREADS) e.ctrl[k] = 0.0;
    if (tid == 0) {
      e.time[0] = 0.0;
      e.stats[3] = sub;
    }
    __syncthreads();
    return;
  }
  for (int k = tid; k < nv; k += SOLVER_THREADS) {
    const double acc = S.a[k];
    e.qvel[k] += h * acc;
    e.qacc_ws[k] = acc;
  }
  __syncthreads();  // the joint loop reads qvel joint-per-thread: full fence
  for (int j = tid; j < m.njnt; j += SOLVER_THREADS) {
    const int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j];
    if (m.jnt_type[j] == RMBX_JNT_FREE) {
      for (int i = 0; i < 3; i++) e.qpos[qa + i] += h * e.qvel[da + i];
      const double* w = e.qvel + da + 3;
      const double nw = norm3(w);
      double* q = e.qpos + qa + 3;
      if (nw > RMBX_MINVAL) {
        const double ax[3] = {w[0] / nw, w[1] / nw, w[2] / nw};
        double qr[4];
        axisangle_quat(ax, nw * h, qr);
        quatmul(q, qr, q);
      }
      quatnorm(q);
    } else {
      e.qpos[qa] += h * e.qvel[da];
    }
  }
  if (tid == 0) e.time[0] += h;
  __syncthreads();
}

struct KArgs {
  rmbx_model m;
  Layout L;
  rmbx_env_buffers b;
  const uint8_t* active;
  int n_env;
  int nsub;
  int sub;  // 1-based substep index of this launch
  int integrate_flag;
  int redo;  // the extra substep after an env-step: only envs reset during it (stats[3] != 0) run
  unsigned long long* prof;  // optional [n_env][16] per-stage cycle sums (diagnostic)
  const int32_t* subtree_end;  // [nbody] end of each body's DFS subtree id range
  const double* hBblk;         // implicitfast: h * (damping + kv terms), packed like Mblk
  PairRuns runs;               // two-level broadphase (rmbx_engine::nprun > 0)
  int tree_rounds;             // pointer-jumping rounds covering the deepest body chain
};


__device__ __forceinline__ void make_env(const KArgs& args, int env, Env& e) {
  const rmbx_model& m = args.m;
  e.m = &args.m;
  e.L = &args.L;
  e.ws = reinterpret_cast<double*>(args.b.workspace) + (size_t)env * args.L.stride;
  e.iw = reinterpret_cast<int32_t*>(e.ws + args.L.ints);
  e.qpos = args.b.qpos + (size_t)env * m.nq;
  e.qvel = args.b.qvel + (size_t)env * m.nv;
  e.qacc_ws = args.b.qacc_ws + (size_t)env * m.nv;
  e.ctrl = args.b.ctrl + (size_t)env * m.nu;
  e.body_pos = args.b.body_pos + (size_t)env * m.nbody * 3;
  e.xpos = args.b.xpos + (size_t)env * m.nbody * 3;
  e.xquat = args.b.xquat + (size_t)env * m.nbody * 4;
  e.gxpos = args.b.gxpos + (size_t)env * m.ngeom * 3;
  e.gxmat = args.b.gxmat + (size_t)env * m.ngeom * 9;
  e.sensordata = args.b.sensordata + (size_t)env * 6;
  e.time = args.b.time + env;
  e.stats = args.b.stats + (size_t)env * 4;
  e.sh = nullptr;
}

#define PROF_BEGIN()                                        \
  unsigned long long* prof = args.prof ? args.prof + (size_t)env * RMBX_PROF_SLOTS : nullptr; \
  unsigned long long t0 = 0, t1 = 0;                        \
  if (prof) t0 = stamp();
#define PROF(k)                                   \
  if (prof) {                                     \
    __syncthreads();                              \
    t1 = stamp();                                 \
    if (threadIdx.x == 0) prof[k] += t1 - t0;     \
    t0 = t1;                                      \
  }

// front half of mj_step: kinematics -> constraint rows (one wavefront per env)
// RUNS: the two-level broadphase (a separate instantiation, so models without pair runs keep the
// one-level kernel's register allocation).  flatten: every stage is inlined -- a stage left out of
// line takes the Env (and through it the 1.5 KB kernel-argument block) by address, which hipcc then
// copies to private memory per lane (the pair-run instance did: 2.4 KB of scratch per lane)
template <bool RUNS>
__global__ void __launch_bounds__(64) __attribute__((flatten)) front_kernel(KArgs args) {
  extern __shared__ __attribute__((aligned(16))) double front_smem[];
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  if (env >= args.n_env) return;
  if (args.active && !args.active[env]) return;
  Env e;
  make_env(args, env, e);
  if (args.redo && e.stats[3] == 0) return;
  // a new env-step clears the divergence-reset marker (read by the host between env-steps)
  if (args.integrate_flag && args.sub == 1 && lane == 0) e.stats[3] = 0;
  e.sh = front_smem;
  e.subtree_end = args.subtree_end;
  __shared__ int s_anc[MAX_BODY];
  PROF_BEGIN()
  kinematics(e, lane, s_anc);
  sync();
  PROF(0)
  com_pos_crb(e, lane, args.subtree_end);
  PROF(1)
  velocity_stage(e, lane, s_anc, args.subtree_end);
  PROF(2)
  const int ncon = collision<RUNS>(e, lane, collision_lds(e, args.runs), args.runs, prof);
  sync();
  PROF(3)
  int ne = 0, nlim = 0;
  const int nefc = make_constraints(e, lane, ncon, &ne, &nlim, prof);
  PROF(4)
  if (lane == 0) {
    WI(scal)[0] = ncon;
    WI(scal)[1] = nefc;
    WI(scal)[2] = ne;
    WI(scal)[3] = nlim;
    e.stats[0] = ncon;
    e.stats[1] = nefc;
  }
}

// back half: Newton solve, constraint forces, sensors, implicitfast integration (4 waves/env)
template <int MINB>
__global__ void __launch_bounds__(SOLVER_THREADS, MINB) solver_kernel(KArgs args) {
  __shared__ SolverShared S;
  const int env = blockIdx.x;
  const int tid = threadIdx.x;
  if (env >= args.n_env) return;
  if (args.active && !args.active[env]) return;
  Env e;
  make_env(args, env, e);
  if (args.redo && e.stats[3] == 0) return;
  const int NB = (args.m.nv + 3) / 4;
  int bi = 0, bj = 0;
  const bool own = tid < NB * (NB + 1) / 2;
  if (own) blk_coords(tid, &bi, &bj);
  double a[16];
  PROF_BEGIN()
  const rmbx_model& m = args.m;
  // stage the dof axes, composite inertias and tree ranges the J-free row passes read
  for (int k = tid; k < 6 * m.nv; k += SOLVER_THREADS) S.cdof[k] = W(cdof)[k];
  for (int k = tid; k < 10 * m.nbody; k += SOLVER_THREADS) S.cinert[k] = W(cinert)[k];
  for (int k = tid; k < m.nbody; k += SOLVER_THREADS) S.send[k] = (int16_t)args.subtree_end[k];
  for (int k = tid; k < m.nv; k += SOLVER_THREADS) S.kb[k] = (int16_t)m.dof_body[k];
  for (int k = tid; k < m.nbody; k += SOLVER_THREADS) S.par[k] = (int16_t)m.body_parent[k];
  if (tid < 6) S.bv[tid] = 0.0;  // the world body's velocity (row passes read it)
  const int ncon = WI(scal)[0], nefc = WI(scal)[1], ne = WI(scal)[2], nlim = WI(scal)[3];
  // per-launch row structure: contact bodies, equality rows, limit rows
  // (a body welded to the world moves with it: no dof sees its wrench and its velocity is
  // zero, so it is staged as the world body and the row passes skip it)
  for (int q = tid; q < ncon; q += SOLVER_THREADS) {
    const int b1 = WI(con_b1)[q], b2 = WI(con_b2)[q];
    S.ccb[q][0] = (int16_t)(m.body_weldid[b1] == 0 ? 0 : b1);
    S.ccb[q][1] = (int16_t)(m.body_weldid[b2] == 0 ? 0 : b2);
  }
  for (int q = tid; q < ne; q += SOLVER_THREADS) {
    for (int i = 0; i < 12; i++) S.eqrho[q][i] = W(eqr_rho)[12 * q + i];
    for (int i = 0; i < 2; i++) {
      S.eqcoef[q][i] = W(eqr_coef)[2 * q + i];
      const int eb = WI(eqr_body)[2 * q + i];
      S.eqb[q][i] = (int16_t)(m.body_weldid[eb] == 0 ? 0 : eb);
      S.eqd[q][i] = (int16_t)WI(eqr_dof)[2 * q + i];
    }
  }
  for (int i = tid; i < nlim; i += SOLVER_THREADS)
    S.lim[i] = (int16_t)(2 * WI(efc_obj)[ne + i] + (WI(efc_kind)[ne + i] >> 3));
  __syncthreads();
  // per-body wrench lists for J^T w (counted, scanned over bodies in wave 0, then filled)
  {
    int cnt = 0;
    const int b = tid;
    const bool body = b > 0 && b < m.nbody;
    if (body) {
      for (int q = 0; q < ncon; q++) cnt += (S.ccb[q][1] == b) + (S.ccb[q][0] == b);
      for (int q = 0; q < ne; q++) cnt += (S.eqb[q][0] == b) + (S.eqb[q][1] == b);
    }
    if (tid < 64) {
      int total;
      const int off = wave_excl_scan(cnt, tid, &total);
      if (b < m.nbody) S.boff[b] = (int16_t)off;
      if (tid == 0) S.boff[m.nbody] = (int16_t)total;
    }
    __syncthreads();
    if (body) {
      int l = S.boff[b];
      for (int q = 0; q < ncon; q++) {
        if (S.ccb[q][1] == b) S.blist[l++] = (int16_t)(2 * q);
        if (S.ccb[q][0] == b) S.blist[l++] = (int16_t)(2 * q + 1);
      }
      for (int q = 0; q < ne; q++) {
        if (S.eqb[q][0] == b) S.blist[l++] = (int16_t)(EQ_TAG + 2 * q);
        if (S.eqb[q][1] == b) S.blist[l++] = (int16_t)(EQ_TAG + 2 * q + 1);
      }
    }
    __syncthreads();
  }
  const int iters = solver_newton(e, S, a, bi, bj, own, ncon, nefc, ne, nlim, args.tree_rounds, tid, prof);
  PROF(5)
  solver_sensors(e, S, ncon, args.tree_rounds, tid);
  PROF(6)
  if (tid == 0) e.stats[2] = iters;
  if (args.integrate_flag) solver_integrate(e, S, a, bi, bj, own, tid, args.sub, args.hBblk);
  PROF(7)
}

// solver blocks resident per CU (launch bound): 4 (<= 128 VGPRs) when the batch needs more than two
// envs per CU -- 1,024 envs run in one round of blocks only at that occupancy -- and 2 (up to 256
// VGPRs: 28 % fewer cycles per env, profiles/r3_solver_occupancy_minb.log) when every env already
// fits in one round at two per CU (C3's 512 envs per GPU).  Same source, same arithmetic: states
// are bitwise equal either way (tests/test_shard_gpu.py runs 512-env shards against 1,024 envs).
// RMBX_SOLVER_MINB = 2 / 3 / 4 forces one (scripts/prof_physics.py).
static int solver_minb_for(int n_env) {
  const char* v = getenv("RMBX_SOLVER_MINB");
  if (v) return atoi(v);
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 4;
  return n_env <= 2 * cus ? 2 : 4;
}

static void launch_solver(int minb, int n_env, hipStream_t st, const KArgs& a) {
  if (minb == 2)
    hipLaunchKernelGGL(solver_kernel<2>, dim3(n_env), dim3(SOLVER_THREADS), 0, st, a);
  else if (minb == 3)
    hipLaunchKernelGGL(solver_kernel<3>, dim3(n_env), dim3(SOLVER_THREADS), 0, st, a);
  else
    hipLaunchKernelGGL(solver_kernel<4>, dim3(n_env), dim3(SOLVER_THREADS), 0, st, a);
}

static Layout make_layout(const rmbx_model& m) {
  Layout L{};
  size_t o = 0;
  auto take = [&](size_t n) {
    const size_t r = o;
    o += (n + 1) & ~size_t(1);  // keep 16-byte alignment
    return r;
  };
  const int nv = m.nv, nb = m.nbody, nj = m.njnt, mc = m.max_contacts;
  L.nefc_max = 4 * mc + 6 * m.neq + 2 * nj + 8;
  L.xmat = take(9 * nb);
  L.xipos = take(3 * nb);
  L.xanchor = take(3 * nj);
  L.xaxis = take(3 * nj);
  L.sxpos = take(3 * m.nsite);
  L.sxmat = take(9 * m.nsite);
  L.cdof = take(6 * nv);
  L.cdofdot = take(6 * nv);
  L.cinert = take(10 * nb);
  L.crb = take(10 * nb);
  L.cvel = take(6 * nb);
  L.cacc = take(6 * nb);
  L.cfrc = take(6 * nb);
  const int nb4 = (nv + 3) / 4;
  L.Mblk = take(16 * (size_t)(nb4 * (nb4 + 1) / 2));
  L.qfrc_bias = take(nv);
  L.qfrc_passive = take(nv);
  L.qfrc_actuator = take(nv);
  L.qfrc_smooth = take(nv);
  L.qacc_smooth = take(nv);
  L.qfrc_constraint = take(nv);
  L.qacc = take(nv);
  L.res = take(nv);
  L.Mres = take(nv);
  L.grad = take(nv);
  L.search = take(nv);
  L.Ms = take(nv);
  L.tmp = take(nv);
  L.ten_len = take(m.ntendon);
  L.ten_vel = take(m.ntendon);
  L.con_pos = take(3 * mc);
  L.con_frame = take(9 * mc);
  L.con_dist = take(mc);
  L.con_mu = take(mc);
  const int ne = L.nefc_max;
  L.neqr_max = 6 * m.neq > 0 ? 6 * m.neq : 1;
  L.hsave = take(16 * (size_t)(nb4 * (nb4 + 1) / 2));
  L.efc_pos = take(ne);
  L.efc_aref = take(ne);
  L.efc_D = take(ne);
  L.efc_sqD = take(ne);
  L.efc_rho = take(6 * (size_t)ne);
  L.efc_R = take(ne);
  L.efc_force = take(ne);
  L.efc_jar = take(ne);
  L.efc_Js = take(ne);
  L.efc_vel = take(ne);
  L.efc_tmp = take(ne);
  L.eqr_rho = take(12 * (size_t)L.neqr_max);
  L.eqr_coef = take(2 * (size_t)L.neqr_max);
  L.con_tmp = take(28 * (size_t)collision_cap(m.npair));
  L.ints = o;
  size_t io = 0;
  auto itake = [&](size_t n) {
    const size_t r = io;
    io += (n + 3) & ~size_t(3);
    return r;
  };
  L.con_b1 = itake(mc);
  L.con_b2 = itake(mc);
  L.con_condim = itake(mc);
  L.con_pair = itake(mc);
  L.con_efcadr = itake(mc);
  L.efc_type = itake(ne);
  L.efc_act = itake(ne);
  L.efc_hact = itake(ne);
  L.efc_kind = itake(ne);
  L.efc_obj = itake(ne);
  L.eqr_body = itake(2 * (size_t)L.neqr_max);
  L.eqr_dof = itake(2 * (size_t)L.neqr_max);
  L.scal = itake(8);
  L.istride = io;
  L.stride = o + (io + 1) / 2;
  L.stride = (L.stride + 31) & ~size_t(31);  // 256-byte aligned env slices
  return L;
}

}  // namespace rmbx

using namespace rmbx;

static size_t front_launch_lds(const rmbx_engine* eng);

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
template <typename T>
static int upload(rmbx_engine* eng, const T* src, size_t n, const T** dst) {
  if (n == 0 || src == nullptr) {
    *dst = nullptr;
    return RMBX_OK;
  }
  void* p = nullptr;
  RMBX_CHECK_HIP(hipMalloc(&p, n * sizeof(T)));
  eng->allocations.push_back(p);
  RMBX_CHECK_HIP(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
  *dst = reinterpret_cast<const T*>(p);
  return RMBX_OK;
}

extern "C" {

int rmbx_engine_create(const struct rmbx_model* model, int n_env, rmbx_engine** out) {
  RMBX_CHECK_ARG(model && out && n_env > 0, "bad arguments to rmbx_engine_create");
  const rmbx_model& h = *model;
  RMBX_CHECK_ARG(h.nv > 0 && h.nv <= MAX_NVP, "nv=%d outside the supported range [1, %d]", h.nv, MAX_NVP);
  RMBX_CHECK_ARG(h.nbody > 0 && h.nbody <= MAX_BODY, "nbody=%d outside [1, %d]", h.nbody, MAX_BODY);
  RMBX_CHECK_ARG(h.max_contacts > 0 && h.max_contacts <= MAX_CON, "max_contacts=%d outside [1, %d]",
                 h.max_contacts, MAX_CON);
  RMBX_CHECK_ARG(2 * h.njnt <= MAX_LIM, "njnt=%d: more limit rows than the solver stages (%d)", h.njnt, MAX_LIM);
  {
    int neqr = 0;
    for (int q = 0; q < h.neq; q++) neqr += h.eq_type[q] == RMBX_EQ_CONNECT ? 3 : (h.eq_type[q] == RMBX_EQ_WELD ? 6 : 1);
    RMBX_CHECK_ARG(neqr <= NEQR, "%d equality rows, more than the solver stages (%d)", neqr, NEQR);
  }
  RMBX_CHECK_ARG(h.npair >= 0 && h.npair < (1 << 24), "npair=%d outside [0, 2^24)", h.npair);
  // runs of consecutive candidate pairs with the same two bodies: the two-level broadphase pays
  // where runs are long (at least 4 pairs on average) and its LDS fits
  std::vector<int32_t> prun_start, prun_body;
  std::vector<double> prun_margin;
  for (int p = 0; p < h.npair; p++) {
    const int b1 = h.geom_body[h.pair_geom1[p]], b2 = h.geom_body[h.pair_geom2[p]];
    if (p == 0 || b1 != prun_body[prun_body.size() - 2] || b2 != prun_body.back()) {
      prun_start.push_back(p);
      prun_body.push_back(b1);
      prun_body.push_back(b2);
      prun_margin.push_back(h.pair_margin[p]);
    } else if (h.pair_margin[p] > prun_margin.back()) {
      prun_margin.back() = h.pair_margin[p];
    }
  }
  int nprun = (int)prun_margin.size();
  prun_start.push_back(h.npair);
  if (nprun == 0 || h.npair < 4 * nprun || front_kernel_lds_bytes(h, nprun) > 65536) nprun = 0;
  RMBX_CHECK_ARG(h.npair <= 65535, "the collision stage indexes pairs in 16 bits (npair=%d)", h.npair);
  RMBX_CHECK_ARG(front_kernel_lds_bytes(h, nprun) <= 65536,
                 "model too large for the front kernel's LDS (nbody=%d nv=%d ngeom=%d npair=%d)", h.nbody,
                 h.nv, h.ngeom, h.npair);
  std::vector<int32_t> body_cgeom(2 * (size_t)h.nbody, 0);
  for (int g = h.ngeom - 1; g >= 0; g--) {
    const int b = h.geom_body[g];
    body_cgeom[2 * b] = g;  // geoms of a body are consecutive (MJCF order)
    body_cgeom[2 * b + 1]++;
  }
  // tree passes need DFS preorder bodies (every subtree a contiguous id range); MJCF order is
  std::vector<int32_t> subtree_end(h.nbody);
  for (int b = h.nbody - 1; b >= 0; b--) {
    subtree_end[b] = b + 1;
    for (int c = b + 1; c < h.nbody; c++)
      if (h.body_parent[c] == b) subtree_end[b] = subtree_end[b] > subtree_end[c] ? subtree_end[b] : subtree_end[c];
  }
  for (int b = 1; b < h.nbody; b++) {
    RMBX_CHECK_ARG(h.body_parent[b] >= 0 && h.body_parent[b] < b, "body %d: parent must precede it", b);
    const int p = h.body_parent[b];
    RMBX_CHECK_ARG(b < subtree_end[p], "bodies are not in DFS preorder (body %d outside its parent's range)", b);
  }
  RMBX_CHECK_ARG(make_layout(h).nefc_max <= HSEL_CAP,
                 "nefc_max=%d exceeds the solver's Hessian row-selection capacity (%d)", make_layout(h).nefc_max,
                 HSEL_CAP);
  rmbx_engine* eng = new rmbx_engine();
  {
    int maxd = 0;
    std::vector<int> depth(h.nbody, 0);
    for (int b = 1; b < h.nbody; b++) {
      depth[b] = depth[h.body_parent[b]] + 1;
      maxd = depth[b] > maxd ? depth[b] : maxd;
    }
    int r = 0;
    while ((1 << r) < maxd + 1) r++;
    eng->tree_rounds = r;
  }
  eng->host = h;
  eng->dev = h;
  eng->n_env = n_env;
  eng->bound = false;
  rmbx_model& d = eng->dev;
  int st = RMBX_OK;
#define UP(field, count)                                  \
  if (st == RMBX_OK) st = upload(eng, h.field, (size_t)(count), &d.field);
  UP(body_parent, h.nbody) UP(body_jntadr, h.nbody) UP(body_jntnum, h.nbody)
  UP(body_dofadr, h.nbody) UP(body_dofnum, h.nbody) UP(body_weldid, h.nbody)
  UP(body_rootid, h.nbody) UP(body_pos, 3 * h.nbody) UP(body_quat, 4 * h.nbody)
  UP(body_mass, h.nbody) UP(body_ipos, 3 * h.nbody) UP(body_inertia, 9 * h.nbody)
  UP(body_invweight0, 2 * h.nbody)
  UP(jnt_type, h.njnt) UP(jnt_body, h.njnt) UP(jnt_qposadr, h.njnt) UP(jnt_dofadr, h.njnt)
  UP(jnt_limited, h.njnt) UP(jnt_pos, 3 * h.njnt) UP(jnt_axis, 3 * h.njnt)
  UP(jnt_range, 2 * h.njnt) UP(jnt_stiffness, h.njnt) UP(jnt_springref, h.njnt)
  UP(jnt_solref, 2 * h.njnt) UP(jnt_solimp, 5 * h.njnt)
  UP(dof_body, h.nv) UP(dof_jnt, h.nv) UP(dof_parent, h.nv) UP(dof_armature, h.nv)
  UP(dof_damping, h.nv) UP(dof_invweight0, h.nv) UP(qpos0, h.nq)
  UP(geom_type, h.ngeom) UP(geom_body, h.ngeom) UP(geom_ctype, h.ngeom)
  UP(geom_size, 3 * h.ngeom) UP(geom_pos, 3 * h.ngeom) UP(geom_quat, 4 * h.ngeom)
  UP(geom_rgba, 4 * h.ngeom) UP(geom_csize, 3 * h.ngeom) UP(geom_cpos, 3 * h.ngeom)
  UP(geom_cquat, 4 * h.ngeom) UP(geom_rbound, h.ngeom)
  UP(pair_geom1, h.npair) UP(pair_geom2, h.npair) UP(pair_condim, h.npair)
  UP(pair_friction, 3 * h.npair) UP(pair_solref, 2 * h.npair) UP(pair_solimp, 5 * h.npair)
  UP(pair_margin, h.npair)
  UP(site_body, h.nsite) UP(site_pos, 3 * h.nsite) UP(site_quat, 4 * h.nsite)
  UP(act_trntype, h.nu) UP(act_trnid, h.nu) UP(act_ctrllimited, h.nu) UP(act_forcelimited, h.nu)
  UP(act_gain, h.nu) UP(act_bias, 3 * h.nu) UP(act_ctrlrange, 2 * h.nu)
  UP(act_forcerange, 2 * h.nu)
  UP(ten_adr, h.ntendon) UP(ten_num, h.ntendon) UP(wrap_jnt, h.nwrap) UP(wrap_coef, h.nwrap)
  UP(eq_type, h.neq) UP(eq_obj1, h.neq) UP(eq_obj2, h.neq) UP(eq_data, RMBX_EQ_DATA * h.neq)
  UP(eq_solref, 2 * h.neq) UP(eq_solimp, 5 * h.neq)
  UP(sensor_type, h.nsensor) UP(sensor_site, h.nsensor)
  UP(cam_body, h.ncam) UP(cam_pos, 3 * h.ncam) UP(cam_quat, 4 * h.ncam) UP(cam_fovy, h.ncam)
  UP(geom_hulladr, h.ngeom) UP(geom_hullnum, h.ngeom) UP(hull_vert, 3 * h.nhullvert)
#undef UP
  if (st != RMBX_OK) {
    rmbx_engine_destroy(eng);
    return st;
  }
  if (st == RMBX_OK) st = upload(eng, subtree_end.data(), (size_t)h.nbody, &eng->subtree_end);
  eng->nprun = nprun;
  eng->prun_start = eng->prun_body = eng->body_cgeom = nullptr;
  eng->prun_margin = nullptr;
  if (nprun > 0) {
    if (st == RMBX_OK) st = upload(eng, prun_start.data(), prun_start.size(), &eng->prun_start);
    if (st == RMBX_OK) st = upload(eng, prun_body.data(), prun_body.size(), &eng->prun_body);
    if (st == RMBX_OK) st = upload(eng, prun_margin.data(), prun_margin.size(), &eng->prun_margin);
    if (st == RMBX_OK) st = upload(eng, body_cgeom.data(), body_cgeom.size(), &eng->body_cgeom);
  }
  {
    // h * (dof damping + actuator velocity gains -kv: joint actuators on the diagonal, tendon
    // actuators as kv * coef_r * coef_c), the implicitfast addition to M, in packed 4x4 blocks
    const int nv = h.nv, NB = (nv + 3) / 4;
    std::vector<double> hb(16 * (size_t)(NB * (NB + 1) / 2), 0.0);
    for (int bi = 0, t = 0; bi < NB; bi++)
      for (int bj = 0; bj <= bi; bj++, t++)
        for (int p = 0; p < 4; p++)
          for (int q = 0; q < 4; q++) {
            const int r = 4 * bi + p, cc = 4 * bj + q;
            if (r >= nv || cc >= nv) continue;
            double add = 0;
            if (r == cc) add += h.dof_damping[r];
            for (int u = 0; u < h.nu; u++) {
              const double kv = -h.act_bias[3 * u + 2];
              if (kv == 0) continue;
              const int id = h.act_trnid[u];
              if (h.act_trntype[u] == RMBX_TRN_JOINT) {
                if (r == cc && h.jnt_dofadr[id] == r) add += kv;
              } else {
                double cr = 0, cq = 0;
                for (int w = h.ten_adr[id]; w < h.ten_adr[id] + h.ten_num[id]; w++) {
                  const int d = h.jnt_dofadr[h.wrap_jnt[w]];
                  if (d == r) cr += h.wrap_coef[w];
                  if (d == cc) cq += h.wrap_coef[w];
                }
                add += kv * cr * cq;
              }
            }
            hb[16 * t + 4 * p + q] = h.timestep * add;
          }
    if (st == RMBX_OK) st = upload(eng, hb.data(), hb.size(), &eng->hBblk);
  }
  if (st != RMBX_OK) {
    rmbx_engine_destroy(eng);
    return st;
  }
  eng->L = make_layout(h);
  eng->front_lds = front_launch_lds(eng);
  eng->solver_minb = solver_minb_for(n_env);
  *out = eng;
  return RMBX_OK;
}

int rmbx_engine_destroy(rmbx_engine* eng) {
  if (!eng) return RMBX_OK;
  for (void* p : eng->allocations) (void)hipFree(p);
  delete eng;
  return RMBX_OK;
}

int rmbx_engine_workspace_bytes(const rmbx_engine* eng, size_t* bytes) {
  RMBX_CHECK_ARG(eng && bytes, "NULL argument");
  *bytes = eng->L.stride * sizeof(double) * (size_t)eng->n_env;
  return RMBX_OK;
}

int rmbx_engine_ws_offset(const rmbx_engine* eng, const char* name, size_t* offset,
                          size_t* count) {
  RMBX_CHECK_ARG(eng && name && offset && count, "NULL argument");
  const Layout& L = eng->L;
  const rmbx_model& m = eng->host;
  const size_t nv = m.nv;
  struct Item {
    const char* n;
    size_t off, cnt;
  } items[] = {
      {"stride", L.stride, L.stride},
      {"Mblk", L.Mblk, 16 * (size_t)(((nv + 3) / 4) * ((nv + 3) / 4 + 1) / 2)},
      {"qfrc_bias", L.qfrc_bias, nv},
      {"qfrc_passive", L.qfrc_passive, nv},
      {"qfrc_actuator", L.qfrc_actuator, nv},
      {"qfrc_smooth", L.qfrc_smooth, nv},
      {"qacc_smooth", L.qacc_smooth, nv},
      {"qfrc_constraint", L.qfrc_constraint, nv},
      {"qacc", L.qacc, nv},
      {"cdof", L.cdof, 6 * nv},
      {"xmat", L.xmat, 9 * (size_t)m.nbody},
      {"sxpos", L.sxpos, 3 * (size_t)m.nsite},
      {"con_pos", L.con_pos, 3 * (size_t)m.max_contacts},
      {"con_dist", L.con_dist, (size_t)m.max_contacts},
      {"con_frame", L.con_frame, 9 * (size_t)m.max_contacts},
      {"efc_force", L.efc_force, (size_t)L.nefc_max},
      {"efc_D", L.efc_D, (size_t)L.nefc_max},
      {"hsave", L.hsave, 16 * (size_t)(((nv + 3) / 4) * ((nv + 3) / 4 + 1) / 2)},
      {"efc_aref", L.efc_aref, (size_t)L.nefc_max},
      // int32 arrays: offsets in int32 units from the workspace start (2 per double)
      {"con_b1", 2 * L.ints + L.con_b1, (size_t)m.max_contacts},
      {"con_b2", 2 * L.ints + L.con_b2, (size_t)m.max_contacts},
      {"con_pair", 2 * L.ints + L.con_pair, (size_t)m.max_contacts},
      {"efc_hact", 2 * L.ints + L.efc_hact, (size_t)L.nefc_max},
      {"efc_act", 2 * L.ints + L.efc_act, (size_t)L.nefc_max},
  };
  for (const Item& it : items) {
    if (strcmp(it.n, name) == 0) {
      *offset = it.off;
      *count = it.cnt;
      return RMBX_OK;
    }
  }
  rmbx::set_error("unknown workspace array '%s'", name);
  return RMBX_ERR_ARG;
}

int rmbx_engine_bind(rmbx_engine* eng, const rmbx_env_buffers* bufs) {
  RMBX_CHECK_ARG(eng && bufs, "NULL argument");
  const rmbx_env_buffers& b = *bufs;
  RMBX_CHECK_ARG(b.time && b.qpos && b.qvel && b.qacc_ws && b.ctrl && b.body_pos && b.xpos &&
                     b.xquat && b.gxpos && b.gxmat && b.sensordata && b.stats && b.workspace,
                 "every buffer of rmbx_env_buffers must be set");
  RMBX_CHECK_ARG((reinterpret_cast<uintptr_t>(b.workspace) & 255) == 0,
                 "workspace must be 256-byte aligned");
  eng->bufs = b;
  eng->bound = true;
  return RMBX_OK;
}

// Dynamic LDS of a front-kernel launch: the model's need, padded so the n_env blocks spread
// evenly over their rounds of blocks.  With k envs fitting a CU (LDS- or register-bound) the launch
// takes R = ceil(n_env / (k CUs)) rounds; asking for LDS that admits only ceil(n_env / (R CUs)) per
// CU gives every CU the same count in every round (otherwise the dispatcher may stack k on some
// CUs and leave others short, or run a last round of a few envs alone).  RMBX_FRONT_BALANCE=0: the
// plain need.
static size_t front_launch_lds(const rmbx_engine* eng) {
  const size_t need = front_kernel_lds_bytes(eng->host, eng->nprun);
  const char* be = std::getenv("RMBX_FRONT_BALANCE");
  if (be && std::atoi(be) == 0) return need;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return need;
  hipFuncAttributes fa{};
  const void* fn = eng->nprun > 0 ? reinterpret_cast<const void*>(&front_kernel<true>)
                                  : reinterpret_cast<const void*>(&front_kernel<false>);
  if (hipFuncGetAttributes(&fa, fn) != hipSuccess) return need;
  const size_t cu_lds = 160 * 1024, stat = fa.sharedSizeBytes;
  const int regs = fa.numRegs > 0 ? fa.numRegs : 256;
  const int k_reg = 4 * (512 / (((regs + 7) / 8) * 8));  // one wave per env, four SIMDs
  int k = (int)(cu_lds / (need + stat));
  if (k > k_reg) k = k_reg;
  if (k < 2) return need;
  const long long n = eng->n_env;
  const long long R = (n + (long long)k * cus - 1) / ((long long)k * cus);
  const int occ = (int)((n + R * cus - 1) / (R * cus));
  if (occ >= k || occ < 1) return need;
  size_t dyn = cu_lds / occ - stat;
  if (dyn > 65536) dyn = 65536;
  dyn &= ~(size_t)15;
  if (dyn < need || (int)(cu_lds / (dyn + stat)) != occ) return need;
  return dyn;
}

static int launch(rmbx_engine* eng, int nsub, int integ, const uint8_t* active, void* stream,
                  unsigned long long* prof = nullptr) {
  if (!eng->bound) {
    rmbx::set_error("engine buffers are not bound (rmbx_engine_bind)");
    return RMBX_ERR_STATE;
  }
  KArgs a;
  a.m = eng->dev;
  a.L = eng->L;
  a.b = eng->bufs;
  a.active = active;
  a.n_env = eng->n_env;
  a.nsub = nsub;
  a.integrate_flag = integ;
  a.redo = 0;
  a.prof = prof;
  a.subtree_end = eng->subtree_end;
  a.tree_rounds = eng->tree_rounds;
  a.hBblk = eng->hBblk;
  a.runs.n = eng->nprun;
  a.runs.start = eng->prun_start;
  a.runs.body = eng->prun_body;
  a.runs.margin = eng->prun_margin;
  a.runs.body_cgeom = eng->body_cgeom;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int reps = integ ? nsub : 1;
  for (int s = 0; s < reps; s++) {
    a.sub = s + 1;
    const size_t front_lds = eng->front_lds;
    if (eng->nprun > 0)
      hipLaunchKernelGGL(front_kernel<true>, dim3(eng->n_env), dim3(64), front_lds, st, a);
    else
      hipLaunchKernelGGL(front_kernel<false>, dim3(eng->n_env), dim3(64), front_lds, st, a);
    RMBX_CHECK_LAUNCH();
    launch_solver(eng->solver_minb, eng->n_env, st, a);
    RMBX_CHECK_LAUNCH();
  }
  if (integ) {
    // redo pass: one more substep (forward + integration) for the envs that reset during this
    // env-step, the substep MuJoCo integrates from the reset state; every other env exits at once
    a.sub = nsub + 1;
    a.redo = 1;
    a.prof = nullptr;
    const size_t front_lds = eng->front_lds;
    if (eng->nprun > 0)
      hipLaunchKernelGGL(front_kernel<true>, dim3(eng->n_env), dim3(64), front_lds, st, a);
    else
      hipLaunchKernelGGL(front_kernel<false>, dim3(eng->n_env), dim3(64), front_lds, st, a);
    RMBX_CHECK_LAUNCH();
    launch_solver(eng->solver_minb, eng->n_env, st, a);
    RMBX_CHECK_LAUNCH();
  }
  return RMBX_OK;
}

int rmbx_engine_step(rmbx_engine* eng, int nsub, const uint8_t* active, void* stream) {
  RMBX_CHECK_ARG(eng && nsub >= 1, "bad arguments");
  return launch(eng, nsub, 1, active, stream);
}

int rmbx_engine_forward(rmbx_engine* eng, const uint8_t* active, void* stream) {
  RMBX_CHECK_ARG(eng, "NULL engine");
  return launch(eng, 1, 0, active, stream);
}

int rmbx_engine_step_profiled(rmbx_engine* eng, int nsub, uint64_t* stage_cycles, void* stream) {
  RMBX_CHECK_ARG(eng && nsub >= 1 && stage_cycles, "bad arguments");
  return launch(eng, nsub, 1, nullptr, stream, reinterpret_cast<unsigned long long*>(stage_cycles));
}

}  // extern "C"
