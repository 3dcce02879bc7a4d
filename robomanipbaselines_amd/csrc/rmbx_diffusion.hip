// Diffusion-policy sampler steps (DDPM for DiffusionPolicy, DDIM for 3D-DiffusionPolicy),
// batched over environments.
//
// Replace the per-step scheduler arithmetic of the reference's conditional_sample loop
// (diffusion_policy / 3D-Diffusion-Policy `conditional_sample`, third_party submodules absent;
// schedulers from diffusers==0.11.1, pyproject.toml:69) driven by
// policy/diffusion_policy/RolloutDiffusionPolicy.py:66-87 (DDPMScheduler args
// TrainDiffusionPolicy.py:130-138) and policy/diffusion_policy_3d/RolloutDiffusionPolicy3d.py:83-101
// (DDIMScheduler args TrainDiffusionPolicy3d.py:203-211).
//
// The per-timestep scalars (sqrt(1 - acp_t), 1 / sqrt(acp_t), x0 / x_t coefficients, sigma) are
// computed once on the host in f32 exactly as the scheduler computes them (0-dim f32 tensors);
// here every element does the f32 tensor arithmetic of one `scheduler.step` in the same
// operation order, with each op rounded (no contraction), including PyTorch's device-side
// "divide by a CPU scalar = multiply by its f32 reciprocal".  One launch covers all envs.

#include "rmbx_common.h"

#include <cstdint>

namespace rmbx {
namespace {

__device__ __forceinline__ float clampf(float v, float lo, float hi) {
  // torch.clamp: NaN propagates
  return v != v ? v : fminf(fmaxf(v, lo), hi);
}

// DDPM epsilon-prediction step with clip_sample, fixed_small variance:
//   x0   = clamp((x - c_eps * eps) * inv_sqrt_acp, -1, 1)
//   prev = c_x0 * x0 + c_xt * x  (+ sigma * noise when t > 0)
__global__ void __launch_bounds__(256) ddpm_step_kernel(const float* __restrict__ eps, const float* __restrict__ x,
                                                        const float* __restrict__ noise, float* __restrict__ out,
                                                        size_t n, float c_eps, float inv_sqrt_acp, float c_x0,
                                                        float c_xt, float sigma, int add_noise) {
#pragma clang fp contract(off)
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float xi = x[i];
    const float t1 = c_eps * eps[i];
    const float t2 = xi - t1;
    float x0 = t2 * inv_sqrt_acp;
    x0 = clampf(x0, -1.f, 1.f);
    const float a = c_x0 * x0;
    const float b = c_xt * xi;
    float prev = a + b;
    if (add_noise) {
      const float v = sigma * noise[i];
      prev = prev + v;
    } else {
      prev = prev + 0.f;  // `pred_prev_sample + 0` of the t = 0 step (turns -0 into +0)
    }
    out[i] = prev;
  }
}

// DDIM step, eta = 0, prediction_type "sample", clip_sample (diffusers 0.11.1 form):
//   x0   = clamp(m, -1, 1)
//   prev = c_x0 * x0 + c_dir * d,  d = m (0.11.1) or the epsilon re-derived from the unclipped
//   x0: (x - sqrt(acp_t) * m) * inv_sqrt_beta (later diffusers releases), selected by eps_mode
__global__ void __launch_bounds__(256) ddim_step_kernel(const float* __restrict__ m, const float* __restrict__ x,
                                                        float* __restrict__ out, size_t n, float c_x0, float c_dir,
                                                        float sqrt_acp, float inv_sqrt_beta, int eps_mode) {
#pragma clang fp contract(off)
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float mi = m[i];
    float d = mi;
    if (eps_mode) {
      const float t1 = sqrt_acp * mi;
      const float t2 = x[i] - t1;
      d = t2 * inv_sqrt_beta;
    }
    const float x0 = clampf(mi, -1.f, 1.f);
    const float a = c_x0 * x0;
    const float b = c_dir * d;
    out[i] = a + b;
  }
}

int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

}  // namespace
}  // namespace rmbx

extern "C" int rmbx_ddpm_step(const float* model_output, const float* sample, const float* noise, float* prev_sample,
                              size_t n, const float* coeffs, void* stream) {
  RMBX_CHECK_ARG(model_output && sample && prev_sample && coeffs, "rmbx_ddpm_step: null pointer");
  const int add_noise = coeffs[5] != 0.f;
  RMBX_CHECK_ARG(!add_noise || noise, "rmbx_ddpm_step: noise required when t > 0");
  if (n == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::ddpm_step_kernel, dim3(rmbx::grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     model_output, sample, noise, prev_sample, n, coeffs[0], coeffs[1], coeffs[2], coeffs[3],
                     coeffs[4], add_noise);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}

extern "C" int rmbx_ddim_step(const float* model_output, const float* sample, float* prev_sample, size_t n,
                              const float* coeffs, int eps_mode, void* stream) {
  RMBX_CHECK_ARG(model_output && prev_sample && coeffs, "rmbx_ddim_step: null pointer");
  RMBX_CHECK_ARG(!eps_mode || sample, "rmbx_ddim_step: sample required for eps_mode");
  if (n == 0) return RMBX_OK;
  hipLaunchKernelGGL(rmbx::ddim_step_kernel, dim3(rmbx::grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     model_output, sample, prev_sample, n, coeffs[0], coeffs[1], coeffs[2], coeffs[3], eps_mode);
  RMBX_CHECK_LAUNCH();
  return RMBX_OK;
}
