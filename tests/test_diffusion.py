"""Diffusion sampler steps: host coefficient tables vs the oracle restatement of the diffusers
0.11.1 schedulers (CPU), and the rmbx_ddpm_step / rmbx_ddim_step kernels vs the oracle over
whole sampling loops, bit-exact (GPU).  Parity vs the diffusers library itself is unpinned
(diffusers is not installed here); the oracle follows its published 0.11.1 source."""

import numpy as np
import pytest
import torch

from oracle.diffusion import DDIMSchedulerRef, DDPMSchedulerRef


def _emulate_ddpm(c, eps, x, nz):
    f = np.float32
    x0 = np.clip((x - f(c[0]) * eps) * f(c[1]), -1, 1)
    prev = f(c[2]) * x0 + f(c[3]) * x
    return prev + (f(c[4]) * nz if c[5] else f(0))


def test_ddpm_tables_match_oracle():
    from robomanipbaselines_amd.policy.diffusion.schedulers import DDPMSampler

    ref = DDPMSchedulerRef(100)
    ref.set_timesteps(100)
    s = DDPMSampler()
    assert torch.equal(ref.alphas_cumprod, s.acp)
    assert np.array_equal(ref.timesteps.numpy(), s.timesteps)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(8, 16, 7, generator=g)
    for i, t in enumerate(s.timesteps):  # table + element order reproduce the oracle step
        eps, nz = torch.randn(8, 16, 7, generator=g) * 2, torch.randn(8, 16, 7, generator=g)
        want = ref.step(eps, t, x, nz)
        assert np.array_equal(_emulate_ddpm(s.coeffs[i], eps.numpy(), x.numpy(), nz.numpy()), want.numpy()), t
        x = want


def test_ddim_tables_match_oracle():
    from robomanipbaselines_amd.policy.diffusion.schedulers import DDIMSampler

    ref = DDIMSchedulerRef(100)
    ref.set_timesteps(10)
    s = DDIMSampler()
    assert np.array_equal(ref.timesteps.numpy(), s.timesteps)
    assert s.timesteps.tolist() == [90, 80, 70, 60, 50, 40, 30, 20, 10, 0]


@pytest.mark.gpu
def test_ddpm_kernel_full_loop_bit_exact():
    from robomanipbaselines_amd.policy.diffusion.schedulers import DDPMSampler

    dev = "cuda:0"
    ref = DDPMSchedulerRef(100)
    ref.set_timesteps(100)
    s = DDPMSampler()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(257, 16, 7, generator=g)  # ragged size
    xd = x.to(dev)
    for i, t in enumerate(s.timesteps):
        eps = torch.randn(257, 16, 7, generator=g) * 3  # pushes x0 past the clip
        nz = torch.randn(257, 16, 7, generator=g)
        x = ref.step(eps, t, x, nz)
        xd = s.step(i, eps.to(dev), xd, nz.to(dev))
        assert torch.equal(xd.cpu(), x), int(t)


@pytest.mark.gpu
@pytest.mark.parametrize("eps_mode", [0, 1])
def test_ddim_kernel_full_loop_bit_exact(eps_mode):
    from robomanipbaselines_amd.policy.diffusion.schedulers import DDIMSampler

    dev = "cuda:0"
    ref = DDIMSchedulerRef(100)
    ref.set_timesteps(10)
    s = DDIMSampler(eps_mode=eps_mode)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(100, 16, 7, generator=g)
    xd = x.to(dev)
    for i, t in enumerate(s.timesteps):
        m = torch.randn(100, 16, 7, generator=g) * 1.5
        x = ref.step(m, t, x, eps_mode=eps_mode)
        xd = s.step(i, m.to(dev), xd)
        assert torch.equal(xd.cpu(), x), int(t)


@pytest.mark.gpu
def test_ddpm_step_requires_noise():
    from robomanipbaselines_amd.policy.diffusion.schedulers import DDPMSampler

    s = DDPMSampler()
    x = torch.zeros(4, device="cuda:0")
    with pytest.raises(ValueError):
        s.step(0, x, x, None)


def test_ddpm_step_known_answers():
    """Pins the scheduler restatement (and through the bit-exact kernel tests above, the HIP step)
    to the published DDPM equations, independent of any library code: the squaredcos_cap_v2
    schedule's cumulative alphas equal alpha_bar(t+1)/alpha_bar(0) (Nichol & Dhariwal eq. 17);
    fed the true noise of x_t = sqrt(abar_t) x0 + sqrt(1-abar_t) eps, one step returns the
    posterior mean mu~_t(x_t, x0) (Ho et al. eq. 7), and the fixed_small noise scale is
    sqrt(beta~_t) = sqrt((1-abar_{t-1}) / (1-abar_t) beta_t)."""
    T = 100
    ref = DDPMSchedulerRef(T)
    ref.set_timesteps(T)
    f = lambda t: np.cos((t / T + 0.008) / 1.008 * np.pi / 2) ** 2  # noqa: E731
    abar = ref.alphas_cumprod.double().numpy()
    want = np.array([f(t + 1) / f(0) for t in range(T)])
    np.testing.assert_allclose(abar[:-1], want[:-1], rtol=2e-5)  # (the last beta is clipped at 0.999)
    rng = np.random.default_rng(0)
    for t in (99, 60, 20, 1, 0):
        x0 = rng.uniform(-0.9, 0.9, (64, 16, 7))
        eps = rng.standard_normal((64, 16, 7))
        a_t = abar[t]
        a_p = abar[t - 1] if t > 0 else 1.0
        b_t = 1 - a_t / a_p
        xt = np.sqrt(a_t) * x0 + np.sqrt(1 - a_t) * eps
        zero = torch.zeros(64, 16, 7)
        got = ref.step(torch.tensor(eps, dtype=torch.float32), t, torch.tensor(xt, dtype=torch.float32), zero).double().numpy()
        mu = np.sqrt(a_p) * b_t / (1 - a_t) * x0 + np.sqrt(1 - b_t) * (1 - a_p) / (1 - a_t) * xt
        np.testing.assert_allclose(got, mu, rtol=0, atol=2e-5 * (1 + np.abs(mu).max()))
        if t > 0:
            z = torch.ones(64, 16, 7)
            noisy = ref.step(torch.tensor(eps, dtype=torch.float32), t, torch.tensor(xt, dtype=torch.float32), z)
            sigma = float((noisy.double().numpy() - got).mean())
            np.testing.assert_allclose(sigma, np.sqrt((1 - a_p) / (1 - a_t) * b_t), rtol=1e-4)


@pytest.mark.parametrize("eps_mode", [0, 1])
def test_ddim_step_known_answers(eps_mode):
    """DDIM with x0 ("sample") prediction and eta = 0 (Song et al. eq. 12): fed the true x0 of
    x_t = sqrt(abar_t) x0 + sqrt(1-abar_t) eps, a step lands on sqrt(abar_prev) x0 +
    sqrt(1-abar_prev) eps, the forward-process sample of the same noise (eps_mode 1, epsilon
    re-derived from x_t); diffusers 0.11.1's direction term uses the model output itself
    (eps_mode 0), giving sqrt(abar_prev) x0 + sqrt(1-abar_prev) x0."""
    ref = DDIMSchedulerRef(100)
    ref.set_timesteps(10)
    abar = ref.alphas_cumprod.double().numpy()
    rng = np.random.default_rng(1)
    for t in (90, 50, 10, 0):
        x0 = rng.uniform(-0.9, 0.9, (64, 16, 7))
        eps = rng.standard_normal((64, 16, 7))
        a_t = abar[t]
        a_p = abar[t - 10] if t >= 10 else 1.0
        xt = np.sqrt(a_t) * x0 + np.sqrt(1 - a_t) * eps
        got = ref.step(torch.tensor(x0, dtype=torch.float32), t, torch.tensor(xt, dtype=torch.float32),
                       eps_mode=eps_mode).double().numpy()
        direction = eps if eps_mode else x0
        want = np.sqrt(a_p) * x0 + np.sqrt(1 - a_p) * direction
        np.testing.assert_allclose(got, want, rtol=0, atol=2e-5 * (1 + np.abs(want).max()))
