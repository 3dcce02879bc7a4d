// Arm command kernels: batched forward kinematics and one damped-least-squares IK step per env.
// Replaces common/body/ArmManager.py:148-153 (set_command_eef_pose) -> :220-243
// (inverse_kinematics: pin.log6, pin.computeJointJacobian (local frame), pin.Jlog6, 6x6 solve,
// pin.integrate) and :213-218 (forward_kinematics), for the UR5e chain of the URDF with the
// arm root pose folded into the first placement.  One lane per env (f64, 6x6 algebra in VGPRs).

#include "rmbx_common.h"
#include "rmbx_math.h"

namespace rmbx {

__device__ __forceinline__ void rotz_mul(const double* R, double q, double* out) {
  // out = R * Rz(q)
  double s, c;
  sincos(q, &s, &c);
  for (int i = 0; i < 3; i++) {
    const double a = R[3 * i], b = R[3 * i + 1];
    out[3 * i] = a * c + b * s;
    out[3 * i + 1] = -a * s + b * c;
    out[3 * i + 2] = R[3 * i + 2];
  }
}

__device__ void arm_fk(const double* P, const double* q, double* Rk, double* pk) {
  double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, p[3] = {0, 0, 0};
  for (int k = 0; k < 6; k++) {
    const double* Pr = P + 12 * k;
    const double* Pp = P + 12 * k + 9;
    double t[3], RP[9];
    matvec3(R, Pp, t);
    for (int i = 0; i < 3; i++) p[i] += t[i];
    matmul3(R, Pr, RP);
    rotz_mul(RP, q[k], R);
    for (int i = 0; i < 9; i++) Rk[9 * k + i] = R[i];
    for (int i = 0; i < 3; i++) pk[3 * k + i] = p[i];
  }
}

__device__ void skew3(const double* v, double* S) {
  S[0] = 0;
  S[1] = -v[2];
  S[2] = v[1];
  S[3] = v[2];
  S[4] = 0;
  S[5] = -v[0];
  S[6] = -v[1];
  S[7] = v[0];
  S[8] = 0;
}

// Pinocchio's log3 (spatial/log.hxx [ext], restated): theta from the clamped trace; within 1e-2
// of pi the axis comes from the diagonal (sqrt((R_ii + cos(theta - pi)) * theta^2 / (1 +
// cos(theta - pi))), sign from the antisymmetric part), where theta / (2 sin theta) * (R - R^T)
// loses its digits; below the Taylor threshold eps^(1/4) the factor is 1/2.
constexpr double kPi = 3.14159265358979323846;
constexpr double kTaylor3 = 1.2207031250000000e-04;  // DBL_EPSILON^(1/4) = 2^-13

__device__ double log3(const double* R, double* w) {
  const double tr = R[0] + R[4] + R[8];
  double t;
  if (tr >= 3.0)
    t = 0.0;
  else if (tr <= -1.0)
    t = kPi;
  else
    t = acos((tr - 1.0) * 0.5);
  if (t >= kPi - 1e-2) {
    const double cphi = cos(t - kPi);
    const double beta = t * t / (1.0 + cphi);
    const double tmp0 = (R[0] + cphi) * beta, tmp1 = (R[4] + cphi) * beta, tmp2 = (R[8] + cphi) * beta;
    w[0] = (R[7] > R[5] ? 1.0 : -1.0) * (tmp0 > 0 ? sqrt(tmp0) : 0.0);
    w[1] = (R[2] > R[6] ? 1.0 : -1.0) * (tmp1 > 0 ? sqrt(tmp1) : 0.0);
    w[2] = (R[3] > R[1] ? 1.0 : -1.0) * (tmp2 > 0 ? sqrt(tmp2) : 0.0);
    return t;
  }
  const double f = (t > kTaylor3 ? t / sin(t) : 1.0) * 0.5;
  w[0] = f * (R[7] - R[5]);
  w[1] = f * (R[2] - R[6]);
  w[2] = f * (R[3] - R[1]);
  return t;
}

__device__ void jlog3(double t, const double* w, double* A) {
  double S[9];
  skew3(w, S);
  if (t < kTaylor3) {
    for (int i = 0; i < 9; i++) A[i] = 0.5 * S[i];
    A[0] += 1;
    A[4] += 1;
    A[8] += 1;
    return;
  }
  const double st = sin(t), ct = cos(t);
  const double st1mct = st / (1 - ct);
  const double d = 0.5 * t * st1mct;
  const double c = 1 / (t * t) - 0.5 * st1mct / t;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) A[3 * i + j] = c * w[i] * w[j] + 0.5 * S[3 * i + j] + (i == j ? d : 0);
}

// J (6x6, row-major) of log6 at (R, p)
__device__ void jlog6(const double* R, const double* p, double* J) {
  double w[3], A[9];
  const double t = log3(R, w);
  jlog3(t, w, A);
  double beta, bdot;
  if (t < kTaylor3) {
    beta = 1.0 / 12 + t * t / 720;
    bdot = 1.0 / 360;
  } else {
    const double st = sin(t), ct = cos(t);
    const double tinv = 1 / t, t2inv = tinv * tinv, inv_2_2ct = 1 / (2 * (1 - ct));
    beta = t2inv - st * tinv * inv_2_2ct;
    bdot = -2 * t2inv * t2inv + (1 + st * tinv) * t2inv * inv_2_2ct;
  }
  const double wTp = dot3(w, p);
  double v3[3];
  for (int i = 0; i < 3; i++) v3[i] = (bdot * wTp) * w[i] - (t * t * bdot + 2 * beta) * p[i];
  double C[9], Sp[9];
  skew3(p, Sp);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      C[3 * i + j] = v3[i] * w[j] + beta * w[i] * p[j] + (i == j ? wTp * beta : 0) + 0.5 * Sp[3 * i + j];
  double B[9];
  matmul3(C, A, B);
  for (int i = 0; i < 36; i++) J[i] = 0;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      J[6 * i + j] = A[3 * i + j];
      J[6 * i + 3 + j] = B[3 * i + j];
      J[6 * (3 + i) + 3 + j] = A[3 * i + j];
    }
}

__device__ void log6(const double* R, const double* p, double* e) {
  double w[3];
  const double t = log3(R, w);
  double alpha, beta;
  if (t < kTaylor3) {
    alpha = 1 - t * t / 12 - t * t * t * t / 720;
    beta = 1.0 / 12 + t * t / 720;
  } else {
    const double st = sin(t), ct = cos(t);
    alpha = t * st / (2 * (1 - ct));
    beta = 1 / (t * t) - st / (2 * t * (1 - ct));
  }
  double wxp[3];
  cross3(w, p, wxp);
  const double wp = dot3(w, p);
  for (int i = 0; i < 3; i++) {
    e[i] = alpha * p[i] - 0.5 * wxp[i] + beta * wp * w[i];
    e[3 + i] = w[i];
  }
}

// Cholesky solve of a 6x6 SPD system in registers
__device__ void spd6_solve(double* A, double* b) {
  for (int j = 0; j < 6; j++) {
    double s = A[6 * j + j];
    for (int k = 0; k < j; k++) s -= A[6 * j + k] * A[6 * j + k];
    const double d = sqrt(s > 1e-300 ? s : 1e-300);
    A[6 * j + j] = d;
    for (int i = j + 1; i < 6; i++) {
      double t = A[6 * i + j];
      for (int k = 0; k < j; k++) t -= A[6 * i + k] * A[6 * j + k];
      A[6 * i + j] = t / d;
    }
  }
  for (int i = 0; i < 6; i++) {
    double t = b[i];
    for (int k = 0; k < i; k++) t -= A[6 * i + k] * b[k];
    b[i] = t / A[6 * i + i];
  }
  for (int i = 5; i >= 0; i--) {
    double t = b[i];
    for (int k = i + 1; k < 6; k++) t -= A[6 * k + i] * b[k];
    b[i] = t / A[6 * i + i];
  }
}

// One ArmManager.inverse_kinematics iteration (ArmManager.py:220-243) on q in place.
__device__ void ik_step(const double* P, double* q, const double* Rt, const double* pt) {
  double Rk[54], pk[18];
  arm_fk(P, q, Rk, pk);
  const double* R6 = Rk + 45;
  const double* p6 = pk + 15;
  // error = current^-1 * target
  double Re[9], pe[3], dp[3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      Re[3 * i + j] = R6[i] * Rt[j] + R6[3 + i] * Rt[3 + j] + R6[6 + i] * Rt[6 + j];
  for (int i = 0; i < 3; i++) dp[i] = pt[i] - p6[i];
  mattvec3(R6, dp, pe);
  double err[6];
  log6(Re, pe, err);
  // joint Jacobian in the local frame of joint 6
  double Jj[36];
  for (int k = 0; k < 6; k++) {
    const double wz[3] = {Rk[9 * k + 2], Rk[9 * k + 5], Rk[9 * k + 8]};
    const double d[3] = {pk[3 * k] - p6[0], pk[3 * k + 1] - p6[1], pk[3 * k + 2] - p6[2]};
    double c[3], v[3], w[3];
    cross3(d, wz, c);
    mattvec3(R6, c, v);
    mattvec3(R6, wz, w);
    for (int i = 0; i < 3; i++) {
      Jj[6 * i + k] = v[i];
      Jj[6 * (3 + i) + k] = w[i];
    }
  }
  // Jlog6(error.inverse()): inverse = (Re^T, -Re^T pe)
  double Ri[9], pi_[3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Ri[3 * i + j] = Re[3 * j + i];
  mattvec3(Re, pe, pi_);
  for (int i = 0; i < 3; i++) pi_[i] = -pi_[i];
  double Jl[36], J[36];
  jlog6(Ri, pi_, Jl);
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) {
      double s = 0;
      for (int k = 0; k < 6; k++) s += Jl[6 * i + k] * Jj[6 * k + j];
      J[6 * i + j] = -s;
    }
  const double damp = err[0] * err[0] + err[1] * err[1] + err[2] * err[2] + err[3] * err[3] +
                      err[4] * err[4] + err[5] * err[5] + 1e-6;
  double A[36], x[6];
  for (int i = 0; i < 6; i++) {
    for (int j = 0; j < 6; j++) {
      double s = 0;
      for (int k = 0; k < 6; k++) s += J[6 * i + k] * J[6 * j + k];
      A[6 * i + j] = s + (i == j ? damp : 0);
    }
    x[i] = err[i];
  }
  spd6_solve(A, x);
  for (int k = 0; k < 6; k++) {
    double s = 0;
    for (int i = 0; i < 6; i++) s += J[6 * i + k] * x[i];
    q[k] -= s;
  }
}

__global__ void arm_ik_kernel(const double* __restrict__ P, double* __restrict__ q_cmd,
                              const double* __restrict__ tgt_R, const double* __restrict__ tgt_p,
                              const uint8_t* __restrict__ mask, int n_env, int n_iter) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  if (mask && !mask[e]) return;
  double q[6];
  for (int k = 0; k < 6; k++) q[k] = q_cmd[6 * (size_t)e + k];
  const double* Rt = tgt_R + 9 * (size_t)e;
  const double* pt = tgt_p + 3 * (size_t)e;
  for (int it = 0; it < n_iter; it++) ik_step(P, q, Rt, pt);
  for (int k = 0; k < 6; k++) q_cmd[6 * (size_t)e + k] = q[k];
}

__global__ void arm_fk_kernel(const double* __restrict__ P, const double* __restrict__ q,
                              double* __restrict__ R_out, double* __restrict__ p_out, int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  double Rk[54], pk[18];
  arm_fk(P, q + 6 * (size_t)e, Rk, pk);
  for (int i = 0; i < 9; i++) R_out[9 * (size_t)e + i] = Rk[45 + i];
  for (int i = 0; i < 3; i++) p_out[3 * (size_t)e + i] = pk[15 + i];
}

// ---------------------------------------------------------------------------------------------
// DataKey routing (MotionManager / ArmManager for the single UR5e arm + gripper).
// The SE3 <-> pose conversions restate the Eigen routines pinocchio calls (MathUtils.py:27-46):
// pin.Quaternion(R) = Eigen's matrix -> quaternion (trace branch, else the largest diagonal),
// SE3(Quaternion(w, x, y, z), t) = Eigen's toRotationMatrix of the UNnormalised quaternion,
// pin.rpy.rpyToMatrix(r, p, y) = (AngleAxis(y, z) * AngleAxis(p, y) * AngleAxis(r, x)) as
// quaternion products, then toRotationMatrix.
// ---------------------------------------------------------------------------------------------
__device__ void quat_from_mat(const double* m, double* wxyz) {
#pragma clang fp contract(off)
  double t = m[0] + m[4] + m[8];
  if (t > 0.0) {
    t = sqrt(t + 1.0);
    wxyz[0] = 0.5 * t;
    t = 0.5 / t;
    wxyz[1] = (m[7] - m[5]) * t;
    wxyz[2] = (m[2] - m[6]) * t;
    wxyz[3] = (m[3] - m[1]) * t;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[4 * i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
    double v[3];
    v[i] = 0.5 * t;
    t = 0.5 / t;
    wxyz[0] = (m[3 * k + j] - m[3 * j + k]) * t;
    v[j] = (m[3 * j + i] + m[3 * i + j]) * t;
    v[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    wxyz[1] = v[0];
    wxyz[2] = v[1];
    wxyz[3] = v[2];
  }
}

__device__ void mat_from_quat(double w, double x, double y, double z, double* R) {
#pragma clang fp contract(off)
  const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1.0 - (tyy + tzz);
  R[1] = txy - twz;
  R[2] = txz + twy;
  R[3] = txy + twz;
  R[4] = 1.0 - (txx + tzz);
  R[5] = tyz - twx;
  R[6] = txz - twy;
  R[7] = tyz + twx;
  R[8] = 1.0 - (txx + tyy);
}

// Eigen's quaternion product a * b (w, x, y, z)
__device__ void quat_mul(const double* a, const double* b, double* o) {
#pragma clang fp contract(off)
  o[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  o[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  o[2] = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
  o[3] = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
}

__device__ void rpy_to_mat(double r, double p, double y, double* R) {
  double sr, cr, sp, cp, sy, cy;
  sincos(0.5 * r, &sr, &cr);
  sincos(0.5 * p, &sp, &cp);
  sincos(0.5 * y, &sy, &cy);
  const double qz[4] = {cy, 0.0, 0.0, sy}, qy[4] = {cp, 0.0, sp, 0.0}, qx[4] = {cr, sr, 0.0, 0.0};
  double a[4], q[4];
  quat_mul(qz, qy, a);
  quat_mul(a, qx, q);
  mat_from_quat(q[0], q[1], q[2], q[3], R);
}

__device__ __forceinline__ double clip(double x, double lo, double hi) {
  // np.clip: NaN propagates
  return x < lo ? lo : (x > hi ? hi : x);
}

struct MotionKeys {
  int32_t code[RMBX_MAX_DATA_KEYS];
  int32_t n;
};

__device__ void write_pose(const double* R, const double* p, double* out) {
  out[0] = p[0];
  out[1] = p[1];
  out[2] = p[2];
  quat_from_mat(R, out + 3);
}

// RolloutBase.get_state (:463-477) -> MotionManager.get_data (:41-90) before normalize_data:
// the raw f64 state of every env, keys concatenated in order.
__global__ void motion_state_kernel(const double* __restrict__ P, const double* __restrict__ jpos,
                                    const double* __restrict__ jvel, const double* __restrict__ wrench,
                                    const double* __restrict__ q_cmd, const double* __restrict__ grip_cmd,
                                    const double* __restrict__ tgt_R, const double* __restrict__ tgt_p,
                                    MotionKeys keys, double* __restrict__ out, int dim, int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  const double* jp = jpos + 7 * (size_t)e;
  double* o = out + (size_t)dim * e;
  for (int ki = 0; ki < keys.n; ki++) {
    switch (keys.code[ki]) {
      case RMBX_KEY_MEASURED_JOINT_POS:
        for (int i = 0; i < 7; i++) o[i] = jp[i];
        o += 7;
        break;
      case RMBX_KEY_MEASURED_JOINT_VEL:
        for (int i = 0; i < 7; i++) o[i] = jvel[7 * (size_t)e + i];
        o += 7;
        break;
      case RMBX_KEY_MEASURED_GRIPPER_JOINT_POS:
        o[0] = jp[6];
        o += 1;
        break;
      case RMBX_KEY_MEASURED_EEF_POSE: {
        // ArmManager.get_eef_pose_from_joint_pos (:161-165) of the measured arm joints
        double Rk[54], pk[18];
        arm_fk(P, jp, Rk, pk);
        write_pose(Rk + 45, pk + 15, o);
        o += 7;
        break;
      }
      case RMBX_KEY_MEASURED_EEF_WRENCH:
        for (int i = 0; i < 6; i++) o[i] = wrench[6 * (size_t)e + i];
        o += 6;
        break;
      case RMBX_KEY_COMMAND_JOINT_POS:
        for (int i = 0; i < 6; i++) o[i] = q_cmd[6 * (size_t)e + i];
        o[6] = grip_cmd[e];
        o += 7;
        break;
      case RMBX_KEY_COMMAND_GRIPPER_JOINT_POS:
        o[0] = grip_cmd[e];
        o += 1;
        break;
      case RMBX_KEY_COMMAND_EEF_POSE:
        // ArmManager.get_command_eef_pose (:185-186): the IK target
        write_pose(tgt_R + 9 * (size_t)e, tgt_p + 3 * (size_t)e, o);
        o += 7;
        break;
      default:
        break;  // validated on the host
    }
  }
}

// RolloutBase.set_command_data (:496-509) -> MotionManager.set_command_data (:25-39) ->
// ArmManager.set_command_data (:88-123), keys in order, on the per-env command state (arm joint
// command, gripper command, IK target SE3).
__global__ void motion_command_kernel(const double* __restrict__ P, const double* __restrict__ action,
                                      int action_dim, MotionKeys keys, int is_skip, double glo, double ghi,
                                      double* __restrict__ q_cmd, double* __restrict__ grip_cmd,
                                      double* __restrict__ tgt_R, double* __restrict__ tgt_p,
                                      const uint8_t* __restrict__ mask, int n_env) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_env) return;
  if (mask && !mask[e]) return;
  double q[6], g = grip_cmd[e], Rt[9], pt[3];
  for (int i = 0; i < 6; i++) q[i] = q_cmd[6 * (size_t)e + i];
  for (int i = 0; i < 9; i++) Rt[i] = tgt_R[9 * (size_t)e + i];
  for (int i = 0; i < 3; i++) pt[i] = tgt_p[3 * (size_t)e + i];
  const double* a = action + (size_t)action_dim * e;
  for (int ki = 0; ki < keys.n; ki++) {
    const int code = keys.code[ki];
    if (code == RMBX_KEY_COMMAND_JOINT_POS || code == RMBX_KEY_COMMAND_JOINT_POS_REL) {
      if (code == RMBX_KEY_COMMAND_JOINT_POS) {
        for (int i = 0; i < 6; i++) q[i] = a[i];
        g = a[6];
      } else if (!is_skip) {  // set_command_joint_pos_rel (:131-139)
        for (int i = 0; i < 6; i++) q[i] = q[i] + a[i];
        g = g + a[6];
      }
      // set_command_joint_pos (:125-129): FK, target = current, then the gripper clip (:141-146)
      double Rk[54], pk[18];
      arm_fk(P, q, Rk, pk);
      for (int i = 0; i < 9; i++) Rt[i] = Rk[45 + i];
      for (int i = 0; i < 3; i++) pt[i] = pk[15 + i];
      g = clip(g, glo, ghi);
      a += 7;
    } else if (code == RMBX_KEY_COMMAND_GRIPPER_JOINT_POS) {
      g = clip(a[0], glo, ghi);
      a += 1;
    } else if (code == RMBX_KEY_COMMAND_EEF_POSE) {
      // set_command_eef_pose (:148-153): target = SE3(Quaternion(w, x, y, z), t), one IK step
      for (int i = 0; i < 3; i++) pt[i] = a[i];
      mat_from_quat(a[3], a[4], a[5], a[6], Rt);
      ik_step(P, q, Rt, pt);
      a += 7;
    } else if (code == RMBX_KEY_COMMAND_EEF_POSE_REL) {
      // ArmManager.set_command_data (:115-119) calls set_command_eef_pose_rel WITHOUT is_skip, so
      // the relative pose composes on every env-step: target = target * SE3(rpy, t), one IK step
      double Rr[9], Rn[9], t[3];
      rpy_to_mat(a[3], a[4], a[5], Rr);
      matvec3(Rt, a, t);
      matmul3(Rt, Rr, Rn);
      for (int i = 0; i < 3; i++) pt[i] = pt[i] + t[i];
      for (int i = 0; i < 9; i++) Rt[i] = Rn[i];
      ik_step(P, q, Rt, pt);
      a += 6;
    }
  }
  for (int i = 0; i < 6; i++) q_cmd[6 * (size_t)e + i] = q[i];
  grip_cmd[e] = g;
  for (int i = 0; i < 9; i++) tgt_R[9 * (size_t)e + i] = Rt[i];
  for (int i = 0; i < 3; i++) tgt_p[3 * (size_t)e + i] = pt[i];
}

}  // namespace rmbx

namespace {

int key_dim(int code) {
  switch (code) {
    case RMBX_KEY_MEASURED_JOINT_POS:
    case RMBX_KEY_MEASURED_JOINT_VEL:
    case RMBX_KEY_MEASURED_EEF_POSE:
    case RMBX_KEY_COMMAND_JOINT_POS:
    case RMBX_KEY_COMMAND_JOINT_POS_REL:
    case RMBX_KEY_COMMAND_EEF_POSE:
      return 7;
    case RMBX_KEY_MEASURED_GRIPPER_JOINT_POS:
    case RMBX_KEY_COMMAND_GRIPPER_JOINT_POS:
      return 1;
    case RMBX_KEY_MEASURED_EEF_WRENCH:
    case RMBX_KEY_COMMAND_EEF_POSE_REL:
      return 6;
    default:
      return -1;
  }
}

bool is_state_key(int code) {
  return code == RMBX_KEY_MEASURED_JOINT_POS || code == RMBX_KEY_MEASURED_JOINT_VEL ||
         code == RMBX_KEY_MEASURED_GRIPPER_JOINT_POS || code == RMBX_KEY_MEASURED_EEF_POSE ||
         code == RMBX_KEY_MEASURED_EEF_WRENCH || code == RMBX_KEY_COMMAND_JOINT_POS ||
         code == RMBX_KEY_COMMAND_GRIPPER_JOINT_POS || code == RMBX_KEY_COMMAND_EEF_POSE;
}

bool is_action_key(int code) {
  return code == RMBX_KEY_COMMAND_JOINT_POS || code == RMBX_KEY_COMMAND_JOINT_POS_REL ||
         code == RMBX_KEY_COMMAND_GRIPPER_JOINT_POS || code == RMBX_KEY_COMMAND_EEF_POSE ||
         code == RMBX_KEY_COMMAND_EEF_POSE_REL;
}

}  // namespace

extern "C" {

int rmbx_arm_ik(const double* placement, double* q_cmd, const double* target_R,
                const double* target_p, const uint8_t* mask, int n_env, int n_iter,
                void* stream) {
  RMBX_CHECK_ARG(placement && q_cmd && target_R && target_p && n_env >= 0 && n_iter >= 0,
                 "bad arguments to rmbx_arm_ik");
  if (n_env == 0 || n_iter == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::arm_ik_kernel, dim3((n_env + 63) / 64), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), placement, q_cmd, target_R, target_p,
                     mask, n_env, n_iter);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_arm_fk(const double* placement, const double* q, double* R_out, double* p_out,
                int n_env, void* stream) {
  RMBX_CHECK_ARG(placement && q && R_out && p_out && n_env >= 0, "bad arguments to rmbx_arm_fk");
  if (n_env == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::arm_fk_kernel, dim3((n_env + 63) / 64), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), placement, q, R_out, p_out, n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_motion_state(const double* placement, const double* joint_pos, const double* joint_vel,
                      const double* wrench, const double* q_cmd, const double* grip_cmd,
                      const double* target_R, const double* target_p, const int32_t* keys,
                      int n_keys, double* state_out, int state_dim, int n_env, void* stream) {
  RMBX_CHECK_ARG(placement && joint_pos && joint_vel && wrench && q_cmd && grip_cmd && target_R &&
                     target_p && n_env >= 0 && n_keys >= 0 && n_keys <= RMBX_MAX_DATA_KEYS &&
                     (n_keys == 0 || keys) && (state_dim == 0 || state_out),
                 "bad arguments to rmbx_motion_state");
  rmbx::MotionKeys k{};
  int dim = 0;
  for (int i = 0; i < n_keys; i++) {
    RMBX_CHECK_ARG(is_state_key(keys[i]), "rmbx_motion_state: data key not supported as state");
    k.code[i] = keys[i];
    dim += key_dim(keys[i]);
  }
  k.n = n_keys;
  RMBX_CHECK_ARG(dim == state_dim, "rmbx_motion_state: state_dim does not match the keys");
  if (n_env == 0 || n_keys == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::motion_state_kernel, dim3((n_env + 63) / 64), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), placement, joint_pos, joint_vel, wrench,
                     q_cmd, grip_cmd, target_R, target_p, k, state_out, state_dim, n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

int rmbx_motion_command(const double* placement, const double* action, int action_dim,
                        const int32_t* keys, int n_keys, int is_skip, double grip_low,
                        double grip_high, double* q_cmd, double* grip_cmd, double* target_R,
                        double* target_p, const uint8_t* mask, int n_env, void* stream) {
  RMBX_CHECK_ARG(placement && action && q_cmd && grip_cmd && target_R && target_p && n_env >= 0 &&
                     n_keys >= 0 && n_keys <= RMBX_MAX_DATA_KEYS && (n_keys == 0 || keys),
                 "bad arguments to rmbx_motion_command");
  rmbx::MotionKeys k{};
  int dim = 0;
  for (int i = 0; i < n_keys; i++) {
    RMBX_CHECK_ARG(is_action_key(keys[i]), "rmbx_motion_command: command data key not supported");
    k.code[i] = keys[i];
    dim += key_dim(keys[i]);
  }
  k.n = n_keys;
  RMBX_CHECK_ARG(dim == action_dim, "rmbx_motion_command: action_dim does not match the keys");
  if (n_env == 0 || n_keys == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::motion_command_kernel, dim3((n_env + 63) / 64), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), placement, action, action_dim, k,
                     is_skip, grip_low, grip_high, q_cmd, grip_cmd, target_R, target_p, mask, n_env);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

}  // extern "C"
