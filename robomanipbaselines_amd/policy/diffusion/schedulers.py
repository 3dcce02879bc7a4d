"""Noise schedulers of the diffusion policies, batched sampler steps on the device.

Restates the two diffusers==0.11.1 schedulers the reference configures (pyproject.toml:69):
  * DDPMScheduler for DiffusionPolicy (TrainDiffusionPolicy.py:130-138): 100 train steps,
    squaredcos_cap_v2 betas, epsilon prediction, clip_sample, fixed_small variance, 100
    inference steps;
  * DDIMScheduler for 3D-DiffusionPolicy (TrainDiffusionPolicy3d.py:203-211): 100 train steps,
    squaredcos_cap_v2, prediction_type "sample", clip_sample, set_alpha_to_one, steps_offset 0,
    eta 0, 10 inference steps.
diffusers is absent from this image, so the published algorithm is restated; parity vs the
library itself is unpinned (tests pin the device kernels against oracle/diffusion.py).

The per-timestep scalars are computed here with the scheduler's own 0-dim CPU f32 tensor
expressions (same operations, order and rounding), and handed to the rmbx_ddpm_step / rmbx_ddim_step kernels, which
apply the per-element f32 arithmetic (including the device-side reciprocal multiply PyTorch
uses for division by a CPU scalar).
"""

import math

import numpy as np
import torch

from ... import _native as N

def cosine_betas(num_train_timesteps, max_beta=0.999):
    """betas_for_alpha_bar (squaredcos_cap_v2): python floats, then a f32 tensor."""
    def alpha_bar(t):
        return math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2

    T = num_train_timesteps
    return torch.tensor([min(1 - alpha_bar((i + 1) / T) / alpha_bar(i / T), max_beta) for i in range(T)],
                        dtype=torch.float32)


def alphas_cumprod(betas):
    return torch.cumprod(1.0 - betas, dim=0)  # CPU f32 (f64 accumulator), as the scheduler holds it


# The per-step scalars are evaluated with 0-dim CPU f32 tensors, the scheduler's own arithmetic:
# `x ** 0.5` of a CPU float tensor is PyTorch's vectorised pow (not always the correctly rounded
# sqrt), so the host evaluates exactly those tensor expressions rather than numpy equivalents.
def _recip(x):
    return torch.tensor(1.0, dtype=torch.float32) / x  # device: tensor / cpu_scalar = tensor * (1 / scalar)


class DDPMSampler:
    """DDPMScheduler (epsilon, clip_sample, fixed_small) as a table of per-step coefficients."""

    def __init__(self, num_train_timesteps=100, num_inference_steps=100, beta_schedule="squaredcos_cap_v2",
                 clip_sample=True, prediction_type="epsilon", variance_type="fixed_small", **_):
        if beta_schedule != "squaredcos_cap_v2" or prediction_type != "epsilon" or not clip_sample \
                or variance_type != "fixed_small":
            raise ValueError("DDPMSampler supports the reference configuration only "
                             "(squaredcos_cap_v2, epsilon, clip_sample, fixed_small)")
        self.T = num_train_timesteps
        self.num_inference_steps = min(num_train_timesteps, num_inference_steps)
        self.acp = alphas_cumprod(cosine_betas(num_train_timesteps))
        self.one = torch.tensor(1.0)
        ratio = self.T // self.num_inference_steps
        self.timesteps = np.arange(0, self.T, ratio)[::-1].copy()
        self.coeffs = np.array([self._coeffs(int(t), ratio) for t in self.timesteps], dtype=np.float32)

    def _coeffs(self, t, ratio):
        prev_t = t - ratio
        alpha_prod_t = self.acp[t]
        alpha_prod_t_prev = self.acp[prev_t] if prev_t >= 0 else self.one
        beta_prod_t = 1 - alpha_prod_t
        beta_prod_t_prev = 1 - alpha_prod_t_prev
        current_alpha_t = alpha_prod_t / alpha_prod_t_prev
        current_beta_t = 1 - current_alpha_t
        c_eps = beta_prod_t ** 0.5
        inv_sqrt_acp = _recip(alpha_prod_t ** 0.5)
        c_x0 = (alpha_prod_t_prev ** 0.5 * current_beta_t) / beta_prod_t
        c_xt = current_alpha_t ** 0.5 * beta_prod_t_prev / beta_prod_t
        sigma = torch.tensor(0.0)
        if t > 0:  # _get_variance (fixed_small)
            var = (1 - alpha_prod_t_prev) / (1 - alpha_prod_t) * (1 - alpha_prod_t / alpha_prod_t_prev)
            sigma = torch.clamp(var, min=1e-20) ** 0.5
        return [float(v) for v in (c_eps, inv_sqrt_acp, c_x0, c_xt, sigma)] + [1.0 if t > 0 else 0.0]

    def step(self, i, model_output, sample, noise=None, out=None):
        """Step i of the loop (timestep self.timesteps[i]); f32 device tensors of equal shape."""
        return _launch_ddpm(self.coeffs[i], model_output, sample, noise, out)


class DDIMSampler:
    """DDIMScheduler (eta 0, prediction "sample", clip_sample, set_alpha_to_one)."""

    def __init__(self, num_train_timesteps=100, num_inference_steps=10, beta_schedule="squaredcos_cap_v2",
                 clip_sample=True, prediction_type="sample", set_alpha_to_one=True, steps_offset=0,
                 eps_mode=0, **_):
        if beta_schedule != "squaredcos_cap_v2" or prediction_type != "sample" or not clip_sample:
            raise ValueError("DDIMSampler supports the reference configuration only")
        self.T = num_train_timesteps
        self.num_inference_steps = num_inference_steps
        self.acp = alphas_cumprod(cosine_betas(num_train_timesteps))
        self.final_acp = torch.tensor(1.0) if set_alpha_to_one else self.acp[0]
        ratio = self.T // num_inference_steps
        self.timesteps = ((np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
                          + steps_offset)
        self.eps_mode = int(eps_mode)
        self.coeffs = np.array([self._coeffs(int(t), ratio) for t in self.timesteps], dtype=np.float32)

    def _coeffs(self, t, ratio):
        prev_t = t - ratio
        alpha_prod_t = self.acp[t]
        alpha_prod_t_prev = self.acp[prev_t] if prev_t >= 0 else self.final_acp
        beta_prod_t = 1 - alpha_prod_t
        std_dev_t = torch.tensor(0.0) * torch.tensor(0.0)  # eta (0) * variance ** 0.5
        c_x0 = alpha_prod_t_prev ** 0.5
        c_dir = (1 - alpha_prod_t_prev - std_dev_t ** 2) ** 0.5
        return [float(v) for v in (c_x0, c_dir, alpha_prod_t ** 0.5, _recip(beta_prod_t ** 0.5))]

    def step(self, i, model_output, sample, out=None):
        return _launch_ddim(self.coeffs[i], model_output, sample, self.eps_mode, out)


def _chk(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous f32 device tensor")


def _launch_ddpm(coeffs, model_output, sample, noise, out):
    _chk(model_output, "model_output")
    _chk(sample, "sample")
    if coeffs[5] != 0:
        if noise is None:
            raise ValueError("noise is required for t > 0")
        _chk(noise, "noise")
    if out is None:
        out = torch.empty_like(sample)
    c = np.ascontiguousarray(coeffs, dtype=np.float32)
    N.call("rmbx_ddpm_step", N.ptr(model_output), N.ptr(sample), N.ptr(noise), N.ptr(out), sample.numel(),
           c.ctypes.data, N.stream_ptr())
    return out


def _launch_ddim(coeffs, model_output, sample, eps_mode, out):
    _chk(model_output, "model_output")
    _chk(sample, "sample")
    if out is None:
        out = torch.empty_like(sample)
    c = np.ascontiguousarray(coeffs, dtype=np.float32)
    N.call("rmbx_ddim_step", N.ptr(model_output), N.ptr(sample), N.ptr(out), sample.numel(), c.ctypes.data,
           int(eps_mode), N.stream_ptr())
    return out
