// Latency microbenchmark (diagnostic): cycles per dependent op for the primitives the physics
// solver chains: block barrier (4 waves), LDS load->use, f64 FMA, L2-resident global load, and
// a dependent LDS broadcast + f64 multiply-add (the Cholesky update pattern).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) k_lat(const int* __restrict__ chase, double* out, unsigned long long* cyc, int n) {
  __shared__ int lds_chase[1024];
  __shared__ double lds_d[1024];
  const int tid = threadIdx.x;
  for (int i = tid; i < 1024; i += 256) { lds_chase[i] = (i * 37 + 11) & 1023; lds_d[i] = 1.0 + i * 1e-9; }
  __syncthreads();
  unsigned long long t0, t1;
  // barrier
  t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i++) __syncthreads();
  t1 = __builtin_readcyclecounter();
  if (tid == 0) cyc[blockIdx.x * 8 + 0] = t1 - t0;
  // LDS chase (wave 0 only, others wait at the end barrier)
  int p = tid & 1023;
  __syncthreads();
  t0 = __builtin_readcyclecounter();
  if (tid < 64) for (int i = 0; i < n; i++) p = lds_chase[p];
  t1 = __builtin_readcyclecounter();
  if (tid == 0) cyc[blockIdx.x * 8 + 1] = t1 - t0;
  // f64 FMA chain
  double x = 1.0 + tid * 1e-7;
  __syncthreads();
  t0 = __builtin_readcyclecounter();
  if (tid < 64) for (int i = 0; i < n; i++) x = fma(x, 0.999999, 1e-9);
  t1 = __builtin_readcyclecounter();
  if (tid == 0) cyc[blockIdx.x * 8 + 2] = t1 - t0;
  // global chase (L2 resident: 4 KB table)
  int g = (tid + blockIdx.x) & 1023;
  __syncthreads();
  t0 = __builtin_readcyclecounter();
  if (tid < 64) for (int i = 0; i < n / 8; i++) g = chase[g];
  t1 = __builtin_readcyclecounter();
  if (tid == 0) cyc[blockIdx.x * 8 + 3] = (t1 - t0) * 8;
  // LDS f64 load -> fma chain (dependent address)
  double y = 0.0;
  int q = tid & 1023;
  __syncthreads();
  t0 = __builtin_readcyclecounter();
  if (tid < 64) for (int i = 0; i < n; i++) { y = fma(lds_d[q], y, 1.0); q = (q + (int)y) & 1023; }
  t1 = __builtin_readcyclecounter();
  if (tid == 0) cyc[blockIdx.x * 8 + 4] = t1 - t0;
  // barrier + LDS write/read round (the solver's step pattern), all 4 waves
  double z = tid;
  __syncthreads();
  t0 = __builtin_readcyclecounter();
  for (int i = 0; i < n; i++) {
    lds_d[(tid + i) & 1023] = z;
    __syncthreads();
    z += lds_d[(tid * 7 + i) & 1023];
  }
  t1 = __builtin_readcyclecounter();
  if (tid == 0) cyc[blockIdx.x * 8 + 5] = t1 - t0;
  out[blockIdx.x * 256 + tid] = x + p + g + y + q + z;
}

int main() {
  const int n = 2000;
  int* chase;
  double* out;
  unsigned long long* cyc;
  std::vector<int> h(1024);
  for (int i = 0; i < 1024; i++) h[i] = (i * 101 + 7) & 1023;
  hipMalloc(&chase, 4096);
  hipMemcpy(chase, h.data(), 4096, hipMemcpyHostToDevice);
  hipMalloc(&out, 1024 * 256 * 8);
  hipMalloc(&cyc, 1024 * 8 * 8);
  const char* names[6] = {"barrier(4 waves)", "lds load->addr", "f64 fma chain", "global load->addr (L2)", "lds f64 load->fma->addr", "lds st+barrier+ld round"};
  for (int nb : {64, 256, 1024}) {
    for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k_lat, dim3(nb), dim3(256), 0, 0, chase, out, cyc, n);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(nb * 8);
    hipMemcpy(c.data(), cyc, nb * 8 * 8, hipMemcpyDeviceToHost);
    printf("blocks %d:\n", nb);
    for (int k = 0; k < 6; k++) {
      double s = 0;
      for (int b = 0; b < nb; b++) s += c[b * 8 + k];
      printf("  %-28s %8.1f cycles/op\n", names[k], s / nb / n);
    }
  }
  return 0;
}
