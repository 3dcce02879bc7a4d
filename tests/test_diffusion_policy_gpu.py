"""DiffusionPolicy on the device: HIP-graph replay of the denoising loop equals the eager loop
on the same noise bit for bit (deterministic MIOpen solvers), the fp32 device network matches its CPU evaluation, and the
batched rollout's env actions follow the reference's pop + limits-denormalisation arithmetic
(RolloutDiffusionPolicy.py:66-87, DataUtils.py:26-40) on the recorded predictions."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _small_model(**kw):
    from robomanipbaselines_amd.policy.diffusion_policy.dp_model import DiffusionPolicyModel

    torch.manual_seed(0)
    return DiffusionPolicyModel(7, 7, 1, crop_hw=(64, 96), down_dims=(64, 128, 256), **kw).eval().requires_grad_(False)


@torch.no_grad()
@pytest.mark.parametrize("widths,B,dtype", [((64, 128, 256), 5, torch.float32),
                                            ((512, 1024, 2048), 1024, torch.float32),
                                            ((512, 1024, 2048), 2048, torch.bfloat16)])
def test_graph_replay_equals_eager(widths, B, dtype):
    """The captured 100-step DDPM loop replays bit-identically to the eager loop, up to the
    production widths and batches of BASELINE configs 3 (DP x2048).  (With MIOpen's f32 conv1d in
    the loop, capture at 1024 envs crashed the process after an 85 s MIOpen Find: profiles/
    r2_dp_capture_1024_fp32_100steps_segv.log; the GEMM device form has no MIOpen call to capture:
    profiles/r2_dp_capture_gemm_*.log.)"""
    from robomanipbaselines_amd.policy.diffusion_policy.dp_model import DiffusionPolicyModel

    torch.backends.cudnn.deterministic = True  # as RolloutDiffusionPolicy sets them
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(0)
    m = DiffusionPolicyModel(7, 7, 1, crop_hw=(64, 96), down_dims=widths, num_inference_steps=100)
    m = m.eval().requires_grad_(False).to(DEV, dtype)
    assert m.graph_max_batch is None or B <= m.graph_max_batch
    g = torch.Generator(device=DEV).manual_seed(3)
    gc = torch.randn(B, m.obs_feature_dim * 2, device=DEV, generator=g)
    x0 = torch.randn(B, 16, 7, device=DEV, generator=g)
    noise = torch.randn(m._n_noise(), B, 16, 7, device=DEV, generator=g)
    gc = gc.to(dtype)
    eager = m.conditional_sample(gc, use_graph=False, x0=x0, noise=noise).clone()
    eager2 = m.conditional_sample(gc, use_graph=False, x0=x0, noise=noise).clone()
    graph = m.conditional_sample(gc, use_graph=True, x0=x0, noise=noise).clone()
    again = m.conditional_sample(gc, use_graph=True, x0=x0, noise=noise).clone()
    assert torch.equal(eager, eager2) and torch.equal(graph, again)
    assert torch.equal(graph, eager)
    assert torch.isfinite(graph).all()


@torch.no_grad()
def test_device_network_matches_cpu_fp32():
    m = _small_model()
    st = torch.randn(3, 2, 7)
    im = torch.rand(3, 1, 2, 3, 64, 96) * 2 - 1
    gc_cpu = m.encode_obs(st, im)
    t = torch.tensor(37)
    x = torch.randn(3, 16, 7)
    out_cpu = m.model(x, t, gc_cpu)
    md = m.to(DEV)
    gc_dev = md.encode_obs(st.to(DEV), im.to(DEV)).cpu()
    out_dev = md.model(x.to(DEV), t.to(DEV), gc_cpu.to(DEV)).cpu()
    assert (gc_dev - gc_cpu).abs().max() <= 1e-3 * max(1.0, gc_cpu.abs().max().item())
    assert (out_dev - out_cpu).abs().max() <= 1e-3 * max(1.0, out_cpu.abs().max().item())


def test_rollout_dp_actions_follow_reference_arithmetic():
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.diffusion_policy.rollout_diffusion_policy import RolloutDiffusionPolicy

    class Rollout(OperationMujocoUR5eCable, RolloutDiffusionPolicy):
        pass

    ro = Rollout(argv=["--num_envs", "3", "--device", DEV, "--precision", "fp32"])
    rec = []
    pa = ro.policy.predict_action

    def spy(*a, **k):
        out = pa(*a, **k)
        rec.append(out.float().cpu().numpy().astype(np.float64))
        return out

    ro.policy.predict_action = spy
    ro.reset()
    ro._active = None
    while ro.phase_idx < len(ro.pre_durations):
        ro.step_once()
    st = ro.model_meta_info["action"]
    scale = st["range"] / (st["norm_config"]["out_max"] - st["norm_config"]["out_min"])
    calls = 0
    for _ in range(3 * 10):
        call = ro.rollout_time_idx % ro.args.skip == 0
        ro.step_once()
        if call:
            a = rec[calls // 8][:, calls % 8]
            want = scale * (a - st["norm_config"]["out_min"]) + st["min"]
            assert np.array_equal(ro.policy_action.cpu().numpy(), want), calls
            calls += 1
    assert len(rec) == 2
    assert np.isfinite(ro.env.engine.qpos.cpu().numpy()).all()


def test_rollout_dp3_pointcloud_and_actions():
    """Batched RolloutDiffusionPolicy3d: the point-cloud observation equals the oracle pipeline on
    the rendered frames, and the env actions follow the pop + denormalisation arithmetic."""
    from oracle import image as OI
    from oracle import pointcloud as OP
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.diffusion_policy_3d.rollout_diffusion_policy_3d import RolloutDiffusionPolicy3d

    class Rollout(OperationMujocoUR5eCable, RolloutDiffusionPolicy3d):
        pass

    ro = Rollout(argv=["--num_envs", "2", "--device", DEV, "--precision", "fp32"])
    rec = []
    pa = ro.policy.predict_action

    def spy(state, pc, **k):
        out = pa(state, pc, **k)
        rec.append((out.float().cpu().numpy().astype(np.float64), pc[:, -1].cpu().numpy(),
                    ro.info["rgb_images"][ro.camera_names[0]].cpu().numpy(),
                    ro.info["depth_images"][ro.camera_names[0]].cpu().numpy()))
        return out

    ro.policy.predict_action = spy
    ro.reset()
    ro._active = None
    while ro.phase_idx < len(ro.pre_durations):
        ro.step_once()
    st = ro.model_meta_info["action"]
    scale = st["range"] / (st["norm_config"]["out_max"] - st["norm_config"]["out_min"])
    calls = 0
    for _ in range(3 * 9):
        call = ro.rollout_time_idx % ro.args.skip == 0
        ro.step_once()
        if call:
            a = rec[calls // 8][0][:, calls % 8]
            want = scale * (a - st["norm_config"]["out_min"]) + st["min"]
            assert np.array_equal(ro.policy_action.cpu().numpy(), want)
            calls += 1
    d = ro.model_meta_info["data"]
    _, pc_last, rgb, depth = rec[0]
    fovy = ro.env.get_camera_fovy(ro.camera_names[0])
    for e in range(2):
        rgb_s = OI.resize_u8(rgb[e], tuple(d["image_size"]))
        dep_s = OI.resize_f32(depth[e], tuple(d["image_size"]))
        n_ref, _, c_ref = OP.observation(dep_s, rgb_s, fovy, d["min_bound"], d["max_bound"], d["num_points"],
                                         ro.model_meta_info["pointcloud"])
        assert c_ref > 0
        assert np.array_equal(pc_last[e], n_ref)


@pytest.mark.parametrize("B,C,Co,T,k", [(4, 64, 128, 16, 5), (3, 256, 256, 8, 5), (2, 32, 64, 4, 3)])
def test_conv1d_gemm_matches_conv1d(B, C, Co, T, k):
    """The bf16 device form of the UNet's stride-1 Conv1d (unfold + one hipBLASLt GEMM) agrees with
    F.conv1d in f32 on the same bf16 operands to bf16 output rounding."""
    import torch.nn as nn

    from robomanipbaselines_amd.policy.diffusion.unet1d import conv1d_gemm

    g = torch.Generator(device=DEV).manual_seed(11)
    conv = nn.Conv1d(C, Co, k, padding=k // 2).to(DEV)
    x = torch.randn(B, C, T, device=DEV, generator=g).to(torch.bfloat16)
    convb = conv.to(torch.bfloat16)
    got = conv1d_gemm(x, convb).float()
    want = F.conv1d(x.float(), convb.weight.float(), convb.bias.float(), padding=k // 2)
    assert got.shape == want.shape == (B, Co, T)
    assert (got - want).abs().max().item() <= 2 ** -7 * want.abs().max().item() + 1e-3


def test_conv_transpose1d_gemm_matches():
    import torch.nn as nn

    from robomanipbaselines_amd.policy.diffusion.unet1d import conv_transpose1d_gemm

    g = torch.Generator(device=DEV).manual_seed(12)
    ct = nn.ConvTranspose1d(128, 64, 4, 2, 1).to(DEV).to(torch.bfloat16)
    x = torch.randn(5, 128, 8, device=DEV, generator=g).to(torch.bfloat16)
    got = conv_transpose1d_gemm(x, ct).float()
    want = F.conv_transpose1d(x.float(), ct.weight.float(), ct.bias.float(), 2, 1)
    assert got.shape == want.shape == (5, 64, 16)
    assert (got - want).abs().max().item() <= 2 ** -6 * want.abs().max().item() + 1e-3


@torch.no_grad()
def test_unet1d_device_form_matches_fp32():
    """The whole ConditionalUnet1D in its bf16 device form (every conv as a GEMM) against the f32
    module on the CPU."""
    from robomanipbaselines_amd.policy.diffusion.unet1d import ConditionalUnet1D

    torch.manual_seed(0)
    ref = ConditionalUnet1D(7, global_cond_dim=64, down_dims=(64, 128, 256), kernel_size=5,
                            cond_predict_scale=True).eval()
    dev = ConditionalUnet1D(7, global_cond_dim=64, down_dims=(64, 128, 256), kernel_size=5,
                            cond_predict_scale=True).eval()
    dev.load_state_dict(ref.state_dict())
    dev = dev.to(DEV, torch.bfloat16)
    x = torch.randn(6, 16, 7)
    gc = torch.randn(6, 64)
    t = torch.tensor(37)
    want = ref(x, t, gc)
    got = dev(x.to(DEV, torch.bfloat16), t.to(DEV), gc.to(DEV, torch.bfloat16)).float().cpu()
    assert got.shape == want.shape
    assert (got - want).abs().max().item() <= 5e-2 * max(1.0, want.abs().max().item())


@torch.no_grad()
@pytest.mark.parametrize("kind", ["dp", "dp3"])
def test_unet1d_production_widths_fp32_and_bf16_error(kind):
    """ConditionalUnet1D at the production widths (512, 1024, 2048) with DP's / DP3's global
    condition sizes: the f32 device form (every conv as an f32 hipBLASLt GEMM) against the f32
    module on the CPU within 1e-4 relative; the bf16 device form's error is measured and bounded."""
    from robomanipbaselines_amd.policy.diffusion.unet1d import ConditionalUnet1D

    cond = 2 * (512 + 7) if kind == "dp" else 2 * (64 + 64)
    torch.manual_seed(1)
    ref = ConditionalUnet1D(7, global_cond_dim=cond, down_dims=(512, 1024, 2048), kernel_size=5,
                            cond_predict_scale=True).eval()
    x = torch.randn(8, 16, 7)
    gc = torch.randn(8, cond)
    t = torch.tensor(61)
    want = ref(x, t, gc)
    scale = max(1.0, want.abs().max().item())
    dev32 = ConditionalUnet1D(7, global_cond_dim=cond, down_dims=(512, 1024, 2048), kernel_size=5,
                              cond_predict_scale=True).eval()
    dev32.load_state_dict(ref.state_dict())
    dev32 = dev32.to(DEV)
    got32 = dev32(x.to(DEV), t.to(DEV), gc.to(DEV)).cpu()
    err32 = (got32 - want).abs().max().item()
    assert err32 <= 1e-4 * scale, err32
    dev16 = dev32.to(torch.bfloat16)
    got16 = dev16(x.to(DEV, torch.bfloat16), t.to(DEV), gc.to(DEV, torch.bfloat16)).float().cpu()
    err16 = (got16 - want).abs().max().item()
    print(f"{kind}: fp32 max|d| {err32:.3e}, bf16 max|d| {err16:.3e} (scale {scale:.3f})")
    assert err16 <= 5e-2 * scale, err16


@torch.no_grad()
def test_rollout_dp_fp32_encoder_is_deterministic():
    """fp32 (the parity mode) restricts MIOpen to deterministic solvers: the image
    encoder at the production crop gives bit-identical features on repeated calls."""
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.diffusion_policy.rollout_diffusion_policy import RolloutDiffusionPolicy

    class Rollout(OperationMujocoUR5eCable, RolloutDiffusionPolicy):
        pass

    ro = Rollout(argv=["--num_envs", "2", "--device", DEV, "--precision", "fp32"])
    assert torch.backends.cudnn.deterministic
    B, ncam = 64, len(ro.camera_names)
    g = torch.Generator(device=DEV).manual_seed(5)
    st = torch.randn(B, ro.n_obs_steps, len(ro.model_meta_info["state"]["example"]), device=DEV, generator=g)
    im = torch.rand(B, ncam, ro.n_obs_steps, 3, ro.crop_size[1], ro.crop_size[0], device=DEV, generator=g) * 2 - 1
    a = ro.policy.encode_obs(st, im).clone()
    b = ro.policy.encode_obs(st, im).clone()
    assert torch.isfinite(a).all() and torch.equal(a, b)
