// Batched rollout glue kernels: ACT temporal ensemble, cable success predicate, UR5e
// observation mapping, depth linearisation, rollout phase schedule.
//
// These are HBM/latency-bound integer and f64 elementwise kernels: bit-exactness against the
// reference is the contract, so every function here is compiled without FP contraction and
// follows the reference's operation order (cited per kernel).

#include <cmath>
#include <cstdarg>
#include <cstring>
#include <string>

#include "rmbx_common.h"

#pragma clang fp contract(off)

namespace rmbx {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

const char* last_error() { return g_last_error.c_str(); }

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// -----------------------------------------------------------------------------------------
// ACT temporal ensemble (policy/act/RolloutAct.py:68-101) + denormalize (DataUtils.py:26-40)
// One 64-lane workgroup per env: lanes copy the new chunk into the ring (coalesced f32),
// then lanes [0, adim) accumulate newest->oldest exactly as the reference loop does.
// -----------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) act_ensemble_kernel(
    const float* __restrict__ new_chunk, const uint8_t* __restrict__ push,
    const uint8_t* __restrict__ active, float* __restrict__ hist, int32_t* __restrict__ hist_len,
    int32_t* __restrict__ hist_head, const double* __restrict__ w_table,
    const double* __restrict__ dn_scale, const double* __restrict__ dn_sub,
    const double* __restrict__ dn_add, double* __restrict__ out, int chunk, int adim, int te) {
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  if (active && !active[env]) return;
  const bool do_push = push ? (push[env] != 0) : true;
  const size_t chunk_elems = (size_t)chunk * adim;
  // TE: [chunk slots][chunk][adim] per env; no TE: one buffer [chunk][adim] per env
  float* ring = hist + (size_t)env * (te ? (size_t)chunk : (size_t)1) * chunk_elems;
  int len = hist_len[env];
  int head = hist_head[env];

  if (te) {
    if (do_push) {
      // history.append(buf); if len > chunk_size: history.pop(0)   (RolloutAct.py:77-83)
      int slot;
      if (len < chunk) {
        slot = head + len;
        if (slot >= chunk) slot -= chunk;
      } else {
        slot = head;  // overwrite the oldest
      }
      const float* src = new_chunk + (size_t)env * chunk_elems;
      float* dst = ring + (size_t)slot * chunk_elems;
      for (size_t i = lane; i < chunk_elems; i += 64) dst[i] = src[i];
      if (len < chunk) {
        len += 1;
      } else {
        head = head + 1 == chunk ? 0 : head + 1;
      }
    }
    __syncthreads();
    if (lane < adim && len > 0) {
      // exp_weights[::-1][j] * H_newest_minus_j[j], accumulated from zeros (RolloutAct.py:93-97)
      const double* w = w_table + (size_t)(len - 1) * chunk;
      double acc = 0.0;
      int slot = head + len - 1;
      if (slot >= chunk) slot -= chunk;
      for (int j = 0; j < len; ++j) {
        const double x = (double)ring[(size_t)slot * chunk_elems + (size_t)j * adim + lane];
        const double term = w[len - 1 - j] * x;
        acc = acc + term;
        slot = slot == 0 ? chunk - 1 : slot - 1;
      }
      const double t = dn_scale[lane] * (acc - dn_sub[lane]);
      out[(size_t)env * adim + lane] = t + dn_add[lane];
    }
    if (lane == 0) {
      hist_len[env] = len;
      hist_head[env] = head;
    }
  } else {
    // --no_temp_ensem: policy_action_buf = list(chunk) when empty, then pop(0) (RolloutAct.py:70-87)
    if (do_push) {
      const float* src = new_chunk + (size_t)env * chunk_elems;
      for (size_t i = lane; i < chunk_elems; i += 64) ring[i] = src[i];
      len = chunk;
      head = 0;
    }
    __syncthreads();
    if (lane < adim && len > 0) {
      const double a = (double)ring[(size_t)head * adim + lane];
      const double t = dn_scale[lane] * (a - dn_sub[lane]);
      out[(size_t)env * adim + lane] = t + dn_add[lane];
    }
    if (lane == 0 && len > 0) {
      hist_len[env] = len - 1;
      hist_head[env] = head + 1;
    }
  }
}

// -----------------------------------------------------------------------------------------
// Cable success predicate (envs/mujoco/ur5e/MujocoUR5eCableEnv.py:48-105), one lane per env.
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ bool check_ccw(double ax, double ay, double bx, double by, double cx,
                                          double cy) {
  // (c[1] - a[1]) * (b[0] - a[0]) > (b[1] - a[1]) * (c[0] - a[0])   (:64-65)
  const double l = (cy - ay) * (bx - ax);
  const double r = (by - ay) * (cx - ax);
  return l > r;
}

__device__ double cable_reward_one(const double* __restrict__ cab, const double* __restrict__ end,
                                   const double* __restrict__ p1, const double* __restrict__ p2,
                                   int n_cable) {
  // cable height: max over z with numpy NaN propagation (:42-44)
  const double z_thre = p1[2] + 0.01;
  double zmax = cab[2];
  bool nan = isnan(zmax);
  for (int i = 1; i < n_cable; ++i) {
    const double z = cab[3 * i + 2];
    nan |= isnan(z);
    zmax = z > zmax ? z : zmax;
  }
  if (!nan && zmax > z_thre) return 0.0;
  // cable end (:47-54)
  const double x_thre = p2[0];
  const double y_thre = p1[1] - 0.05;
  if (end[0] < x_thre || end[1] > y_thre) return 0.0;
  // crossing test (:57-79)
  const double pdx = p2[0] - p1[0];
  const double pdy = p2[1] - p1[1];
  for (int i = 0; i + 1 < n_cable; ++i) {
    const double ax = cab[3 * i], ay = cab[3 * i + 1];
    const double bx = cab[3 * i + 3], by = cab[3 * i + 4];
    if ((check_ccw(ax, ay, p1[0], p1[1], p2[0], p2[1]) !=
         check_ccw(bx, by, p1[0], p1[1], p2[0], p2[1])) &&
        (check_ccw(ax, ay, bx, by, p1[0], p1[1]) != check_ccw(ax, ay, bx, by, p2[0], p2[1]))) {
      const double cdx = bx - ax;
      const double cdy = by - ay;
      const double l = pdx * cdy;
      const double r = pdy * cdx;
      const double cross = l - r;
      if (cross > 0) return 1.0;
    }
  }
  return 0.0;
}

__global__ void cable_reward_kernel(const double* __restrict__ cable_xpos,
                                    const double* __restrict__ end_xpos,
                                    const double* __restrict__ pole1,
                                    const double* __restrict__ pole2, double* __restrict__ reward,
                                    int n_env, int n_cable) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  reward[e] = cable_reward_one(cable_xpos + (size_t)e * n_cable * 3, end_xpos + 3 * (size_t)e,
                               pole1 + 3 * (size_t)e, pole2 + 3 * (size_t)e, n_cable);
}

// -----------------------------------------------------------------------------------------
// Peg-in-hole success predicate (envs/mujoco/ur5e/MujocoUR5eInsertEnv.py:43-63)
// -----------------------------------------------------------------------------------------
__device__ double insert_reward_one(const double* __restrict__ peg, const double* __restrict__ hole,
                                    const double* __restrict__ q, double xy_thre, double z_off, double cos_tilt) {
  // np.max(np.abs(peg_pos[:2] - hole_pos[:2])) < xy_thre, NaN-propagating like numpy's max
  const double dx = fabs(peg[0] - hole[0]), dy = fabs(peg[1] - hole[1]);
  if (isnan(dx) || isnan(dy)) return 0.0;
  const double m = dy > dx ? dy : dx;
  if (!(m < xy_thre)) return 0.0;
  const double z_thre = hole[2] + z_off;
  if (!(peg[2] < z_thre)) return 0.0;
  // peg z axis = xmat[:, 2] (mju_quat2Mat of xquat); np.dot with (0, 0, -1) in numpy's order
  const double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2];
  const double q11 = q[1] * q[1], q13 = q[1] * q[3], q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  const bool ident = q[0] == 1.0 && q[1] == 0.0 && q[2] == 0.0 && q[3] == 0.0;
  const double zx = ident ? 0.0 : 2.0 * (q13 + q02);
  const double zy = ident ? 0.0 : 2.0 * (q23 - q01);
  const double zz = ident ? 1.0 : ((q00 - q11) - q22) + q33;
  double dot = zx * 0.0;
  dot = dot + zy * 0.0;
  dot = dot + zz * -1.0;
  return dot > cos_tilt ? 1.0 : 0.0;
}

// -----------------------------------------------------------------------------------------
// Toolbox placement reward (envs/mujoco/ur5e/MujocoUR5eToolboxEnv.py:46-57): toolbox within
// xy_thre of the mat in x and y (numpy max, NaN -> fail) and below the mat height + z_off
// -----------------------------------------------------------------------------------------
__global__ void toolbox_reward_kernel(const double* __restrict__ box, const double* __restrict__ mat,
                                      double* __restrict__ reward, int n_env, double xy_thre, double z_off) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  const double* b = box + 3 * (size_t)e;
  const double* t = mat + 3 * (size_t)e;
  const double dx = fabs(b[0] - t[0]), dy = fabs(b[1] - t[1]);
  double r = 0.0;
  if (!isnan(dx) && !isnan(dy)) {
    const double m = dy > dx ? dy : dx;
    const double z_thre = t[2] + z_off;
    if (m < xy_thre && b[2] < z_thre) r = 1.0;
  }
  reward[e] = r;
}

// -----------------------------------------------------------------------------------------
// Ring-on-pole reward (envs/mujoco/ur5e/MujocoUR5eRingEnv.py:46-75): z gate, then matplotlib's
// Path(ring xy + first).contains_point(pole xy) -- code-less path, radius 0, identity transform
// ([ext] matplotlib src/_path.h point_in_path_impl, path_converters.h PathNanRemover): the
// identity affine poisons both coordinates of a vertex with a non-finite one, non-finite
// vertices are dropped and the next finite vertex opens a new subpath, a subpath is closed to
// its start only at the end of the path, crossing-number test per subpath, OR over subpaths.
// -----------------------------------------------------------------------------------------
struct MplVertexStream {
  const double* ring;
  int n;    // ring bodies; the path has n + 1 vertices (the first repeated)
  int pos;  // next path vertex
  bool first;
  // returns 1 MOVETO, 2 LINETO, 0 STOP
  __device__ int next(double* x, double* y) {
    bool gap = false;
    while (pos <= n) {
      const double* v = ring + 3 * (pos < n ? pos : 0);
      pos++;
      const double X = (v[0] * 1.0 + v[1] * 0.0) + 0.0;
      const double Y = (v[0] * 0.0 + v[1] * 1.0) + 0.0;
      if (!(isfinite(X) && isfinite(Y))) {
        gap = true;
        continue;
      }
      *x = X;
      *y = Y;
      const int code = (first || gap) ? 1 : 2;
      first = false;
      return code;
    }
    return 0;
  }
};

__device__ __forceinline__ bool mpl_cross(double vtx0, double vty0, double vtx1, double vty1, double tx, double ty,
                                          bool yflag1) {
  return (((vty1 - ty) * (vtx0 - vtx1)) >= ((vtx1 - tx) * (vty0 - vty1))) == yflag1;
}

__device__ double ring_reward_one(const double* __restrict__ ring, const double* __restrict__ pole, int n) {
  const double z_thre = pole[2] + 0.08;
  double zmax = ring[2];
  bool nan = isnan(zmax);
  for (int i = 1; i < n; ++i) {
    const double z = ring[3 * i + 2];
    nan |= isnan(z);
    zmax = z > zmax ? z : zmax;
  }
  if (!nan && zmax > z_thre) return 0.0;
  const double tx = pole[0], ty = pole[1];
  if (!(isfinite(tx) && isfinite(ty))) return 0.0;
  MplVertexStream st{ring, n, 0, true};
  bool inside = false;
  int code = -1;
  double x = 0.0, y = 0.0;
  while (true) {
    if (code != 1) {
      code = st.next(&x, &y);
      if (code == 0) break;
    }
    const double sx = x, sy = y;
    double vtx0 = x, vty0 = y, vtx1 = x, vty1 = y;
    bool yflag0 = vty0 >= ty;
    bool flag = false;
    while (true) {
      code = st.next(&x, &y);
      if (code == 0) {
        x = sx;
        y = sy;
      } else if (code == 1) {
        break;
      }
      const bool yflag1 = vty1 >= ty;
      if (yflag0 != yflag1 && mpl_cross(vtx0, vty0, vtx1, vty1, tx, ty, yflag1)) flag = !flag;
      yflag0 = yflag1;
      vtx0 = vtx1;
      vty0 = vty1;
      vtx1 = x;
      vty1 = y;
      if (code == 0) break;
    }
    const bool yflag1 = vty1 >= ty;
    if (yflag0 != yflag1 && mpl_cross(vtx0, vty0, vtx1, vty1, tx, ty, yflag1)) flag = !flag;
    inside = inside || flag;
    if (inside || code == 0) break;
  }
  return inside ? 1.0 : 0.0;
}

__global__ void ring_reward_kernel(const double* __restrict__ ring_xpos, const double* __restrict__ pole_xpos,
                                   double* __restrict__ reward, int n_env, int n_ring) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  reward[e] = ring_reward_one(ring_xpos + (size_t)e * n_ring * 3, pole_xpos + 3 * (size_t)e, n_ring);
}


// -----------------------------------------------------------------------------------------
// Door-opening reward (envs/mujoco/ur5e/MujocoUR5eDoorEnv.py:52-67): continuous, success iff 1.0
// -----------------------------------------------------------------------------------------
__device__ double door_reward_one(const double* __restrict__ pinch, const double* __restrict__ handle, double angle,
                                  double margin, double target) {
  // np.linalg.norm(gripper_pos - handle_pos) = sqrt(x . x)
  const double d0 = pinch[0] - handle[0], d1 = pinch[1] - handle[1], d2 = pinch[2] - handle[2];
  double ss = d0 * d0;
  ss = ss + d1 * d1;
  ss = ss + d2 * d2;
  const double dist = sqrt(ss);
  // np.exp(-10.0 * np.max([dist - margin, 0.0])) (numpy max propagates NaN)
  const double ex = dist - margin;
  const double mx = isnan(ex) ? ex : (ex > 0.0 ? ex : 0.0);
  double reaching = exp(-10.0 * mx);
  // np.clip(door_angle / target, 0.0, 1.0)
  double opening = angle / target;
  opening = opening < 0.0 ? 0.0 : (opening > 1.0 ? 1.0 : opening);
  if (opening >= 1.0) reaching = 1.0;
  return 0.5 * (reaching + opening);
}

__global__ void door_reward_kernel(const double* __restrict__ pinch, const double* __restrict__ handle,
                                   const double* __restrict__ angle, double* __restrict__ reward, int n_env,
                                   double margin, double target) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  reward[e] = door_reward_one(pinch + 3 * (size_t)e, handle + 3 * (size_t)e, angle[e], margin, target);
}

// -----------------------------------------------------------------------------------------
// Cabinet reward (envs/mujoco/ur5e/MujocoUR5eCabinetEnv.py:57-73): hinge opened past the angle
// threshold and/or drawer slid past the distance threshold, per target task (0 any, 1 hinge,
// 2 slide); NaN joint values compare false, as numpy's
// -----------------------------------------------------------------------------------------
__global__ void cabinet_reward_kernel(const double* __restrict__ qpos, int qpos_stride, int hinge_adr, int slide_adr,
                                      double hinge_thre, double slide_thre, int target_task,
                                      double* __restrict__ reward, int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  const double* q = qpos + (size_t)e * qpos_stride;
  const bool hinge = q[hinge_adr] > hinge_thre;
  const bool slide = q[slide_adr] > slide_thre;
  const bool ok = target_task == 1 ? hinge : (target_task == 2 ? slide : (hinge || slide));
  reward[e] = ok ? 1.0 : 0.0;
}

__global__ void insert_reward_kernel(const double* __restrict__ peg_xpos, const double* __restrict__ hole_xpos,
                                     const double* __restrict__ peg_xquat, double* __restrict__ reward, int n_env,
                                     double xy_thre, double z_off, double cos_tilt) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  reward[e] = insert_reward_one(peg_xpos + 3 * (size_t)e, hole_xpos + 3 * (size_t)e, peg_xquat + 4 * (size_t)e,
                                xy_thre, z_off, cos_tilt);
}

// -----------------------------------------------------------------------------------------
// UR5e observation mapping (envs/mujoco/ur5e/MujocoUR5eEnvBase.py:78-119)
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ double gripper_joint_pos(const double* g) {
  // np.rad2deg(gripper_qpos.mean(keepdims=True)) / 45.0 * 255.0   (:106)
  double s = 0.0;
  s = s + g[0];
  s = s + g[1];
  s = s + g[2];
  s = s + g[3];
  const double mean = s / 4.0;
  const double deg = mean * (180.0 / 3.14159265358979323846);
  return deg / 45.0 * 255.0;
}

__global__ void ur5e_obs_kernel(const double* __restrict__ arm_qpos,
                                const double* __restrict__ arm_qvel,
                                const double* __restrict__ grip_qpos,
                                const double* __restrict__ force, const double* __restrict__ torque,
                                double* __restrict__ joint_pos, double* __restrict__ joint_vel,
                                double* __restrict__ wrench, int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  for (int i = 0; i < 6; ++i) {
    joint_pos[7 * (size_t)e + i] = arm_qpos[6 * (size_t)e + i];
    joint_vel[7 * (size_t)e + i] = arm_qvel[6 * (size_t)e + i];
  }
  joint_pos[7 * (size_t)e + 6] = gripper_joint_pos(grip_qpos + 4 * (size_t)e);
  joint_vel[7 * (size_t)e + 6] = 0.0;
  for (int i = 0; i < 3; ++i) {
    wrench[6 * (size_t)e + i] = force[3 * (size_t)e + i];
    wrench[6 * (size_t)e + 3 + i] = torque[3 * (size_t)e + i];
  }
}

// -----------------------------------------------------------------------------------------
// Depth linearisation (envs/mujoco/MujocoEnvBase.py:122-125), f32 with numpy NEP-50 scalars.
// -----------------------------------------------------------------------------------------
__global__ void depth_linearize_kernel(const float* __restrict__ z, float* __restrict__ d,
                                       size_t n, float near32, float c32) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float t = z[i] * c32;
  const float u = 1.0f - t;
  d[i] = near32 / u;
}

// -----------------------------------------------------------------------------------------
// Phase schedule (RolloutBase.py:28-132, PhaseBase.py:19-34, PhaseManager.py:20-37)
// -----------------------------------------------------------------------------------------
__global__ void sched_reset_kernel(rmbx_sched_t* __restrict__ s, const double* __restrict__ time,
                                   const uint8_t* __restrict__ mask, int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  if (mask && !mask[e]) return;
  rmbx_sched_t v;
  memset(&v, 0, sizeof(v));
  v.phase = 0;
  v.phase_start = time[e];  // PhaseManager.reset -> _set_phase(0) -> start()
  s[e] = v;
}

__global__ void sched_update_kernel(rmbx_sched_t* __restrict__ s, const double* __restrict__ time,
                                    const double* __restrict__ reward,
                                    const double* __restrict__ pre_dur, int n_pre,
                                    double max_duration, double post_success, int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  rmbx_sched_t v = s[e];
  if (v.done) return;
  const double t = time[e];
  const double r = reward[e];
  const double elapsed = t - v.phase_start;  // get_elapsed_duration (PhaseBase.py:33-34)
  bool transition = false;
  if (v.phase < n_pre) {
    transition = elapsed > pre_dur[v.phase];
  } else if (v.phase == n_pre) {
    // post_update: rollout_time_idx += 1 (RolloutBase.py:70) happens before check_transition
    v.rollout_time_idx += 1;
    if (r >= 1.0 && !v.has_success_time) {
      v.success_time = elapsed;
      v.has_success_time = 1;
    }
    if (v.has_success_time) {
      transition = elapsed > v.success_time + post_success;
    } else {
      transition = elapsed > max_duration;
    }
    if (transition) {
      v.success = r >= 1.0;
      v.result_reward = r;
      v.duration = elapsed;
    }
  } else {
    // EndRolloutPhase.check_transition with auto_exit: one world per env -> quit (:124-132)
    v.done = 1;
  }
  if (transition) {
    v.phase += 1;
    v.phase_start = t;  // next phase start()
    if (v.phase == n_pre) {
      v.rollout_time_idx = 0;  // RolloutPhase.start (RolloutBase.py:47-48)
      v.has_success_time = 0;
      v.success_time = 0.0;
    }
  }
  s[e] = v;
}

__global__ void sched_active_kernel(const rmbx_sched_t* __restrict__ s, int n_pre, uint8_t* __restrict__ active,
                                    int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  active[e] = (!s[e].done && s[e].phase <= n_pre) ? 1 : 0;
}

}  // namespace rmbx

// =========================================================================================
// C ABI
// =========================================================================================
using namespace rmbx;

extern "C" {

int rmbx_abi_version(void) { return RMBX_ABI_VERSION; }

const char* rmbx_last_error(void) { return rmbx::last_error(); }

int rmbx_device_count(int* count) {
  RMBX_CHECK_ARG(count != nullptr, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = (e == hipSuccess) ? n : 0;
  return RMBX_OK;
}

int rmbx_act_ensemble(const float* new_chunk, const uint8_t* push, const uint8_t* active,
                      float* hist, int32_t* hist_len, int32_t* hist_head, const double* w_table,
                      const double* dn_scale, const double* dn_sub, const double* dn_add,
                      double* out, int n_env, int chunk, int adim, int temporal_ensemble,
                      void* stream) {
  RMBX_CHECK_ARG(n_env >= 0 && chunk > 0 && adim > 0 && adim <= 64,
                 "bad sizes n_env=%d chunk=%d adim=%d (adim must be in [1, 64])", n_env, chunk,
                 adim);
  RMBX_CHECK_ARG(hist && hist_len && hist_head && w_table && dn_scale && dn_sub && dn_add && out,
                 "NULL buffer");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(act_ensemble_kernel, dim3(n_env), dim3(64), 0, as_stream(stream), new_chunk,
                     push, active, hist, hist_len, hist_head, w_table, dn_scale, dn_sub, dn_add,
                     out, chunk, adim, temporal_ensemble ? 1 : 0);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_cable_reward(const double* cable_xpos, const double* end_xpos, const double* pole1_xpos,
                      const double* pole2_xpos, double* reward, int n_env, int n_cable,
                      void* stream) {
  RMBX_CHECK_ARG(n_env >= 0 && n_cable >= 1, "bad sizes n_env=%d n_cable=%d", n_env, n_cable);
  RMBX_CHECK_ARG(cable_xpos && end_xpos && pole1_xpos && pole2_xpos && reward, "NULL buffer");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(cable_reward_kernel, dim3((n_env + 255) / 256), dim3(256), 0,
                     as_stream(stream), cable_xpos, end_xpos, pole1_xpos, pole2_xpos, reward,
                     n_env, n_cable);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_cabinet_reward(const double* qpos, int qpos_stride, int hinge_adr, int slide_adr, double hinge_thre,
                        double slide_thre, int target_task, double* reward, int n_env, void* stream) {
  RMBX_CHECK_ARG(n_env >= 0, "bad n_env=%d", n_env);
  RMBX_CHECK_ARG(qpos && reward, "NULL buffer");
  RMBX_CHECK_ARG(hinge_adr >= 0 && hinge_adr < qpos_stride && slide_adr >= 0 && slide_adr < qpos_stride,
                 "joint addresses (%d, %d) outside qpos rows of %d", hinge_adr, slide_adr, qpos_stride);
  RMBX_CHECK_ARG(target_task >= 0 && target_task <= 2, "Invalid target task: %d", target_task);
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(cabinet_reward_kernel, dim3((n_env + 255) / 256), dim3(256), 0, as_stream(stream), qpos,
                     qpos_stride, hinge_adr, slide_adr, hinge_thre, slide_thre, target_task, reward, n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_toolbox_reward(const double* toolbox_xpos, const double* mat_xpos, double* reward, int n_env,
                        double xy_thre, double z_offset, void* stream) {
  RMBX_CHECK_ARG(n_env >= 0, "bad n_env=%d", n_env);
  RMBX_CHECK_ARG(toolbox_xpos && mat_xpos && reward, "NULL buffer");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(toolbox_reward_kernel, dim3((n_env + 255) / 256), dim3(256), 0, as_stream(stream),
                     toolbox_xpos, mat_xpos, reward, n_env, xy_thre, z_offset);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_ring_reward(const double* ring_xpos, const double* pole_xpos, double* reward, int n_env, int n_ring,
                     void* stream) {
  RMBX_CHECK_ARG(n_env >= 0 && n_ring >= 1, "bad sizes n_env=%d n_ring=%d", n_env, n_ring);
  RMBX_CHECK_ARG(ring_xpos && pole_xpos && reward, "NULL buffer");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(ring_reward_kernel, dim3((n_env + 255) / 256), dim3(256), 0, as_stream(stream), ring_xpos,
                     pole_xpos, reward, n_env, n_ring);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_door_reward(const double* pinch_xpos, const double* handle_xpos, const double* door_angle, double* reward,
                     int n_env, double margin, double target_angle, void* stream) {
  RMBX_CHECK_ARG(n_env >= 0, "bad n_env=%d", n_env);
  RMBX_CHECK_ARG(pinch_xpos && handle_xpos && door_angle && reward, "NULL buffer");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(door_reward_kernel, dim3((n_env + 255) / 256), dim3(256), 0, as_stream(stream), pinch_xpos,
                     handle_xpos, door_angle, reward, n_env, margin, target_angle);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_insert_reward(const double* peg_xpos, const double* hole_xpos, const double* peg_xquat, double* reward,
                       int n_env, double xy_thre, double z_offset, double cos_tilt, void* stream) {
  RMBX_CHECK_ARG(n_env >= 0, "bad n_env=%d", n_env);
  RMBX_CHECK_ARG(peg_xpos && hole_xpos && peg_xquat && reward, "NULL buffer");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(insert_reward_kernel, dim3((n_env + 255) / 256), dim3(256), 0, as_stream(stream), peg_xpos,
                     hole_xpos, peg_xquat, reward, n_env, xy_thre, z_offset, cos_tilt);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_ur5e_obs(const double* arm_qpos, const double* arm_qvel, const double* grip_qpos,
                  const double* force, const double* torque, double* joint_pos, double* joint_vel,
                  double* wrench, int n_env, void* stream) {
  RMBX_CHECK_ARG(n_env >= 0, "bad n_env=%d", n_env);
  RMBX_CHECK_ARG(arm_qpos && arm_qvel && grip_qpos && force && torque && joint_pos && joint_vel &&
                     wrench,
                 "NULL buffer");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(ur5e_obs_kernel, dim3((n_env + 255) / 256), dim3(256), 0, as_stream(stream),
                     arm_qpos, arm_qvel, grip_qpos, force, torque, joint_pos, joint_vel, wrench,
                     n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_depth_linearize(const float* zbuf, float* depth, size_t n_pix, double near_, double far_,
                         void* stream) {
  RMBX_CHECK_ARG(zbuf && depth, "NULL buffer");
  RMBX_CHECK_ARG(near_ > 0 && far_ > near_, "bad clip planes near=%g far=%g", near_, far_);
  if (n_pix == 0) return RMBX_OK;
  const float c32 = (float)(1.0 - near_ / far_);
  hipLaunchKernelGGL(depth_linearize_kernel, dim3((unsigned)((n_pix + 255) / 256)), dim3(256), 0,
                     as_stream(stream), zbuf, depth, n_pix, (float)near_, c32);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_sched_reset(rmbx_sched_t* sched, const double* time, const uint8_t* mask, int n_env,
                     void* stream) {
  RMBX_CHECK_ARG(sched && time && n_env >= 0, "bad arguments");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(sched_reset_kernel, dim3((n_env + 255) / 256), dim3(256), 0,
                     as_stream(stream), sched, time, mask, n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_sched_update(rmbx_sched_t* sched, const double* time, const double* reward,
                      const double* pre_durations, int n_pre, double max_duration,
                      double post_success_duration, int n_env, void* stream) {
  RMBX_CHECK_ARG(sched && time && reward && n_env >= 0 && n_pre >= 0, "bad arguments");
  RMBX_CHECK_ARG(n_pre == 0 || pre_durations, "pre_durations is NULL");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(sched_update_kernel, dim3((n_env + 255) / 256), dim3(256), 0,
                     as_stream(stream), sched, time, reward, pre_durations, n_pre, max_duration,
                     post_success_duration, n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_sched_active(const rmbx_sched_t* sched, int n_pre, uint8_t* active, int n_env, void* stream) {
  RMBX_CHECK_ARG(sched && active && n_env >= 0 && n_pre >= 0, "rmbx_sched_active: bad arguments");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(sched_active_kernel, dim3((n_env + 255) / 256), dim3(256), 0, as_stream(stream), sched, n_pre,
                     active, n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

}  // extern "C"
