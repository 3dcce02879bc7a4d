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
  for (int it = 0; it < n_iter; it++) {
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

}  // namespace rmbx

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

}  // extern "C"
