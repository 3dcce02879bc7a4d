// Small f64 vector/quaternion/spatial-algebra helpers for the dynamics kernels (device).
// Spatial vectors are [angular; linear] about the world origin; spatial inertia is stored as
// 10 numbers: m, h = m*c (3), rotational inertia about the origin (xx yy zz xy xz yz).
#pragma once

#include <hip/hip_runtime.h>

#define RMBX_MINVAL 1e-15

namespace rmbx {

__device__ __forceinline__ void quat2mat(const double* q, double* R) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
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
__device__ __forceinline__ void quatmul(const double* a, const double* b, double* r) {
  const double t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  const double t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  const double t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  const double t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
  r[3] = t3;
}
__device__ __forceinline__ void quatnorm(double* q) {
  const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < RMBX_MINVAL) {
    q[0] = 1;
    q[1] = q[2] = q[3] = 0;
    return;
  }
  const double inv = 1.0 / n;
  q[0] *= inv;
  q[1] *= inv;
  q[2] *= inv;
  q[3] *= inv;
}
__device__ __forceinline__ void axisangle_quat(const double* ax, double ang, double* q) {
  double s, c;
  sincos(0.5 * ang, &s, &c);
  q[0] = c;
  q[1] = ax[0] * s;
  q[2] = ax[1] * s;
  q[3] = ax[2] * s;
}
__device__ __forceinline__ void matvec3(const double* R, const double* v, double* r) {
  const double t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  const double t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  const double t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
__device__ __forceinline__ void mattvec3(const double* R, const double* v, double* r) {
  const double t0 = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
  const double t1 = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
  const double t2 = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
__device__ __forceinline__ void matmul3(const double* A, const double* B, double* C) {
  double t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) C[i] = t[i];
}
__device__ __forceinline__ void cross3(const double* a, const double* b, double* r) {
  const double t0 = a[1] * b[2] - a[2] * b[1];
  const double t1 = a[2] * b[0] - a[0] * b[2];
  const double t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
__device__ __forceinline__ double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ double norm3(const double* a) { return sqrt(dot3(a, a)); }
__device__ __forceinline__ double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

__device__ __forceinline__ void inert_mul(const double* I, const double* v, double* r) {
  const double m = I[0];
  const double* h = I + 1;
  const double* w = v;
  const double* u = v + 3;
  double n[3], hxu[3], hxw[3];
  n[0] = I[4] * w[0] + I[7] * w[1] + I[8] * w[2];
  n[1] = I[7] * w[0] + I[5] * w[1] + I[9] * w[2];
  n[2] = I[8] * w[0] + I[9] * w[1] + I[6] * w[2];
  cross3(h, u, hxu);
  cross3(h, w, hxw);
  r[0] = n[0] + hxu[0];
  r[1] = n[1] + hxu[1];
  r[2] = n[2] + hxu[2];
  r[3] = m * u[0] - hxw[0];
  r[4] = m * u[1] - hxw[1];
  r[5] = m * u[2] - hxw[2];
}
__device__ __forceinline__ void cross_motion(const double* V, const double* U, double* r) {
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
__device__ __forceinline__ void cross_force(const double* V, const double* F, double* r) {
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

// 64-lane wave reductions (one wavefront per environment)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
// exclusive prefix sum across the wave (lane order)
__device__ __forceinline__ int wave_excl_scan(int v, int lane, int* total) {
  int x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

}  // namespace rmbx
