"""DiffusionPolicy and DP3 at production size, fp32 device vs fp32 CPU (SURVEY §8a a9/a10, §8c bar:
1e-4 on actions in fp32 mode against the CPU restatement on identical inputs).

* DP (TrainDiffusionPolicy.py:114-138): the GroupNorm ResNet-18 + SpatialSoftmax encoder on the
  216x288 eval crop with 2 obs steps, and the whole predict_action (encoder + 100-step DDPM loop,
  HIP-graph replayed on the device) with the initial trajectory and every step's variance noise
  injected, on 8 envs.
* DP3 (TrainDiffusionPolicy3d.py:194-218): the PointNet encoder (512 points, LayerNorm) + state MLP,
  and the whole predict_action (10-step DDIM) on 8 envs.

The upstream networks are absent (parity vs upstream unpinned); the CPU module is the same
restatement evaluated by PyTorch-CPU in f32.  The bf16 device error is measured and printed."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
B = 8


def _randomize_norms(m, seed):
    """Non-trivial GroupNorm / LayerNorm affine parameters (default init is 1 / 0)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, (torch.nn.GroupNorm, torch.nn.LayerNorm)):
                mod.weight.copy_(torch.rand(mod.weight.shape, generator=g) + 0.5)
                mod.bias.copy_(torch.rand(mod.bias.shape, generator=g) * 0.4 - 0.2)
    return m


def _cpu_predict(m, state, obs, x0, noise=None):
    """predict_action on the CPU: the module's encoder and UNet in f32, the scheduler steps of
    oracle/diffusion.py (the diffusers 0.11.1 restatement; the device samplers are HIP kernels)."""
    from oracle.diffusion import DDIMSchedulerRef, DDPMSchedulerRef
    from robomanipbaselines_amd.policy.diffusion.schedulers import DDPMSampler

    gc = m.encode_obs(state, obs)
    ddpm = isinstance(m.sampler, DDPMSampler)
    s = DDPMSchedulerRef(100) if ddpm else DDIMSchedulerRef(100)
    s.set_timesteps(len(m.sampler.timesteps))
    traj, k = x0, 0
    for t in s.timesteps:
        out = m.model(traj, t, gc)
        if ddpm:
            nz = None
            if int(t) > 0:
                nz = noise[k]
                k += 1
            traj = s.step(out, t, traj, nz)
        else:
            traj = s.step(out, t, traj, eps_mode=m.sampler.eps_mode)
    start = m.n_obs_steps - 1
    return traj[:, start:start + m.n_action_steps]


def _rel(got, want):
    return ((got - want).abs().max() / max(1.0, want.abs().max().item())).item()


def _dp_inputs():
    g = torch.Generator().manual_seed(5)
    state = torch.rand(B, 2, 7, generator=g) * 2 - 1
    images = torch.rand(B, 1, 2, 3, 216, 288, generator=g) * 2 - 1
    x0 = torch.randn(B, 16, 7, generator=g)
    return state, images, x0, g


@torch.no_grad()
def test_dp_encoder_production_size_fp32():
    from robomanipbaselines_amd.policy.diffusion_policy.dp_model import DiffusionPolicyModel

    torch.manual_seed(0)
    m = _randomize_norms(DiffusionPolicyModel(7, 7, 1), 1).eval()
    state, images, _, _ = _dp_inputs()
    want = m.encode_obs(state, images)
    assert want.shape == (B, 2 * (7 + 64))
    md = m.to(DEV)
    md.obs_nets = md.obs_nets.to(memory_format=torch.channels_last)
    got = md.encode_obs(state.to(DEV), images.to(DEV)).cpu()
    err = _rel(got, want)
    print(f"DP encoder fp32 rel err {err:.3e}")
    assert err <= 1e-4, err
    m16 = md.to(torch.bfloat16)
    got16 = m16.encode_obs(state.to(DEV), images.to(DEV)).float().cpu()
    print(f"DP encoder bf16 rel err {_rel(got16, want):.3e}")


@torch.no_grad()
def test_dp_predict_action_production_size_fp32():
    """Encoder + 100 DDPM steps with the reference's scheduler, noise injected: actions within 1e-4."""
    from robomanipbaselines_amd.policy.diffusion_policy.dp_model import DiffusionPolicyModel

    torch.manual_seed(2)
    m = _randomize_norms(DiffusionPolicyModel(7, 7, 1, num_inference_steps=100), 3).eval()
    state, images, x0, g = _dp_inputs()
    noise = torch.randn(m._n_noise(), B, 16, 7, generator=g)
    want = _cpu_predict(m, state, images, x0, noise)
    assert want.shape == (B, 8, 7)
    md = m.to(DEV)
    md.obs_nets = md.obs_nets.to(memory_format=torch.channels_last)
    args = (state.to(DEV), images.to(DEV))
    kw = dict(x0=x0.to(DEV), noise=noise.to(DEV))
    got = md.predict_action(*args, use_graph=True, **kw).cpu()
    err = _rel(got, want)
    print(f"DP predict_action fp32 rel err {err:.3e} (max |a| {want.abs().max().item():.3f})")
    assert err <= 1e-4, err
    m16 = md.to(torch.bfloat16)
    got16 = m16.predict_action(*args, use_graph=True, **kw).float().cpu()
    print(f"DP predict_action bf16 rel err {_rel(got16, want):.3e}")


def _dp3_inputs():
    g = torch.Generator().manual_seed(7)
    state = torch.rand(B, 2, 7, generator=g) * 2 - 1
    pc = torch.rand(B, 2, 512, 6, generator=g) * 2 - 1
    x0 = torch.randn(B, 16, 7, generator=g)
    return state, pc, x0


@torch.no_grad()
@pytest.mark.parametrize("use_pc_color", [False, True])
def test_dp3_encoder_and_predict_action_fp32(use_pc_color):
    from robomanipbaselines_amd.policy.diffusion_policy_3d.dp3_model import DP3Model

    torch.manual_seed(4)
    m = _randomize_norms(DP3Model(7, 7, use_pc_color=use_pc_color), 5).eval()
    state, pc, x0 = _dp3_inputs()
    enc_want = m.encode_obs(state, pc)
    assert enc_want.shape == (B, 2 * 128)
    want = _cpu_predict(m, state, pc, x0)
    md = m.to(DEV)
    enc_got = md.encode_obs(state.to(DEV), pc.to(DEV)).cpu()
    enc_err = _rel(enc_got, enc_want)
    assert enc_err <= 1e-4, enc_err
    got = md.predict_action(state.to(DEV), pc.to(DEV), use_graph=True, x0=x0.to(DEV)).cpu()
    err = _rel(got, want)
    print(f"DP3 (colour {use_pc_color}) encoder rel err {enc_err:.3e}, predict_action fp32 rel err {err:.3e}")
    assert err <= 1e-4, err
    m16 = md.to(torch.bfloat16)
    got16 = m16.predict_action(state.to(DEV), pc.to(DEV), use_graph=True, x0=x0.to(DEV)).float().cpu()
    print(f"DP3 predict_action bf16 rel err {_rel(got16, want):.3e}")
