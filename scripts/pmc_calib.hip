// Calibration kernels for the FETCH_SIZE / WRITE_SIZE counters (MI355X_MICROARCH.md: widths other
// than 16 B/lane are uncalibrated).  Each reads and writes a known byte count with the access width
// the physics kernels use (8 B per lane, f64) and, for comparison, 16 B per lane.
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(256) calib_f64(const double* __restrict__ a, double* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i] + 1.0;
}

__global__ void __launch_bounds__(256) calib_f32x4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    float4 v = a[i];
    v.x += 1.f;
    b[i] = v;
  }
}

extern "C" int pmc_calib(const void* a, void* b, size_t bytes, int wide, void* stream) {
  if (wide)
    hipLaunchKernelGGL(calib_f32x4, dim3(4096), dim3(256), 0, (hipStream_t)stream, (const float4*)a, (float4*)b,
                       bytes / 16);
  else
    hipLaunchKernelGGL(calib_f64, dim3(4096), dim3(256), 0, (hipStream_t)stream, (const double*)a, (double*)b,
                       bytes / 8);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
