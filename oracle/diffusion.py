"""TEST INFRASTRUCTURE ONLY (the oracle; never imported by the product path).

CPU restatement of the diffusers==0.11.1 scheduler steps the reference's diffusion policies use
(pyproject.toml:69; DDPMScheduler args policy/diffusion_policy/TrainDiffusionPolicy.py:130-138,
DDIMScheduler args policy/diffusion_policy_3d/TrainDiffusionPolicy3d.py:203-211), written the way
the library writes them: betas_for_alpha_bar -> f32 tensor, alphas_cumprod = torch.cumprod,
per-step 0-dim CPU f32 tensors, then the element tensor ops.  The reference runs the policy on the
GPU, where PyTorch divides a device tensor by a CPU scalar as a multiply by the f32 reciprocal
(BinaryDivTrueKernel "is_cpu_scalar" path); `_div_cpu_scalar` restates that.  diffusers is not
installed here, so parity against the library is UNPINNED; the restatement follows its published
0.11.1 source.
"""

import math

import torch


def betas_for_alpha_bar(num_diffusion_timesteps, max_beta=0.999):
    def alpha_bar(time_step):
        return math.cos((time_step + 0.008) / 1.008 * math.pi / 2) ** 2

    betas = []
    for i in range(num_diffusion_timesteps):
        t1 = i / num_diffusion_timesteps
        t2 = (i + 1) / num_diffusion_timesteps
        betas.append(min(1 - alpha_bar(t2) / alpha_bar(t1), max_beta))
    return torch.tensor(betas, dtype=torch.float32)


def _div_cpu_scalar(x, s):
    inv = torch.tensor(1.0, dtype=torch.float32) / s
    return x * inv.item()


def _mul_cpu_scalar(s, x):
    return x * s.item()


class DDPMSchedulerRef:
    def __init__(self, num_train_timesteps=100):
        self.T = num_train_timesteps
        self.betas = betas_for_alpha_bar(num_train_timesteps)
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.one = torch.tensor(1.0)
        self.num_inference_steps = None

    def set_timesteps(self, num_inference_steps):
        self.num_inference_steps = min(self.T, num_inference_steps)
        import numpy as np

        self.timesteps = torch.from_numpy(np.arange(0, self.T, self.T // self.num_inference_steps)[::-1].copy())

    def _get_variance(self, t):
        prev_t = t - self.T // self.num_inference_steps
        alpha_prod_t = self.alphas_cumprod[t]
        alpha_prod_t_prev = self.alphas_cumprod[prev_t] if prev_t >= 0 else self.one
        current_beta_t = 1 - alpha_prod_t / alpha_prod_t_prev
        variance = (1 - alpha_prod_t_prev) / (1 - alpha_prod_t) * current_beta_t
        return torch.clamp(variance, min=1e-20)

    def step(self, model_output, timestep, sample, variance_noise):
        """prev_sample of DDPMScheduler.step (epsilon, clip_sample, fixed_small); f32 tensors."""
        t = int(timestep)
        prev_t = t - self.T // self.num_inference_steps
        alpha_prod_t = self.alphas_cumprod[t]
        alpha_prod_t_prev = self.alphas_cumprod[prev_t] if prev_t >= 0 else self.one
        beta_prod_t = 1 - alpha_prod_t
        beta_prod_t_prev = 1 - alpha_prod_t_prev
        current_alpha_t = alpha_prod_t / alpha_prod_t_prev
        current_beta_t = 1 - current_alpha_t
        pred_original_sample = _div_cpu_scalar(sample - _mul_cpu_scalar(beta_prod_t ** 0.5, model_output),
                                               alpha_prod_t ** 0.5)
        pred_original_sample = torch.clamp(pred_original_sample, -1, 1)
        pred_original_sample_coeff = (alpha_prod_t_prev ** 0.5 * current_beta_t) / beta_prod_t
        current_sample_coeff = current_alpha_t ** 0.5 * beta_prod_t_prev / beta_prod_t
        pred_prev_sample = (_mul_cpu_scalar(pred_original_sample_coeff, pred_original_sample)
                            + _mul_cpu_scalar(current_sample_coeff, sample))
        variance = 0
        if t > 0:
            variance = _mul_cpu_scalar(self._get_variance(t) ** 0.5, variance_noise)
        return pred_prev_sample + variance


class DDIMSchedulerRef:
    def __init__(self, num_train_timesteps=100, set_alpha_to_one=True, steps_offset=0):
        self.T = num_train_timesteps
        self.betas = betas_for_alpha_bar(num_train_timesteps)
        self.alphas = 1.0 - self.betas
        self.alphas_cumprod = torch.cumprod(self.alphas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.steps_offset = steps_offset

    def set_timesteps(self, num_inference_steps):
        import numpy as np

        self.num_inference_steps = num_inference_steps
        step_ratio = self.T // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * step_ratio).round()[::-1].copy().astype(np.int64)
        self.timesteps = torch.from_numpy(ts) + self.steps_offset

    def step(self, model_output, timestep, sample, eta=0.0, eps_mode=0):
        """prev_sample of DDIMScheduler.step, prediction_type "sample", clip_sample.
        eps_mode 0: the 0.11.1 direction term uses model_output; 1: re-derived epsilon."""
        t = int(timestep)
        prev_timestep = t - self.T // self.num_inference_steps
        alpha_prod_t = self.alphas_cumprod[t]
        alpha_prod_t_prev = self.alphas_cumprod[prev_timestep] if prev_timestep >= 0 else self.final_alpha_cumprod
        beta_prod_t = 1 - alpha_prod_t
        pred_original_sample = model_output
        direction_src = model_output
        if eps_mode:
            direction_src = _div_cpu_scalar(sample - _mul_cpu_scalar(alpha_prod_t ** 0.5, pred_original_sample),
                                            beta_prod_t ** 0.5)
        pred_original_sample = torch.clamp(pred_original_sample, -1, 1)
        std_dev_t = torch.tensor(eta, dtype=torch.float32) * 0.0  # eta = 0 in the reference
        pred_sample_direction = _mul_cpu_scalar((1 - alpha_prod_t_prev - std_dev_t ** 2) ** 0.5, direction_src)
        return _mul_cpu_scalar(alpha_prod_t_prev ** 0.5, pred_original_sample) + pred_sample_direction
