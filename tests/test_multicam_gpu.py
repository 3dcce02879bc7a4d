"""A two-camera policy through the batched rollout (`camera_names` from the
model meta info, RolloutBase.get_images :480-490 stacking one image per camera, ACT's backbone run
per camera with the features concatenated, third_party/act detr_vae.py [absent]).

At the policy call: every camera slice of the policy tensor equals a single-camera render of the
same env state, and the fp32 device ACT (fused trunk, bf16x6 GEMMs) on that two-camera input
matches the unfused fp32 CPU module within the 1e-4 action bar of tests/test_act_full_gpu.py."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _s2d_to_nchw(s):
    """Inverse of kernels.image_to_s2d: [B, H/2, W/2, 16] (channel (dy*2+dx)*3+c) -> [B, 3, H, W]."""
    B, h, w, _ = s.shape
    x = s[..., :12].reshape(B, h, w, 2, 2, 3)  # dy, dx, c
    return x.permute(0, 5, 1, 3, 2, 4).reshape(B, 3, 2 * h, 2 * w)


@torch.no_grad()
def test_act_two_camera_policy_input_and_network():
    from robomanipbaselines_amd.envs.operation.OperationMujocoUR5eCable import OperationMujocoUR5eCable
    from robomanipbaselines_amd.policy.act.act_model import ActModel
    from robomanipbaselines_amd.policy.act.rollout_act import RolloutAct

    class Rollout(OperationMujocoUR5eCable, RolloutAct):
        pass

    ro = Rollout(argv=["--num_envs", "2", "--device", DEV, "--precision", "fp32", "--act_prune_dead_decoder"])
    cams = list(ro.env.camera_names[:2])
    assert len(cams) == 2
    ro.model_meta_info["image"]["camera_names"] = cams
    ro.camera_names = cams
    ro.setup_policy()
    assert ro.policy.num_cams == 2
    seen = []
    fwd = ro.policy.forward

    def spy(state, images):
        out = fwd(state, images)
        # the same env state rendered one camera at a time
        per_cam = []
        for i, cam in enumerate(cams):
            buf = torch.empty_like(images[:, i])
            ro.env.render_images(cam, policy=buf, mean=ro.image_norm[0], std=ro.image_norm[1])
            per_cam.append(buf)
        seen.append((state.clone(), images.clone(), out.float().clone(), per_cam))
        return out

    ro.policy.forward = spy
    ro.reset()
    ro._active = None
    while ro.phase_idx < len(ro.pre_durations):
        ro.step_once()
    for _ in range(3):
        ro.step_once()
    assert len(seen) == 1
    state, images, out, per_cam = seen[0]
    assert images.shape[:2] == (2, 2)
    for i in range(2):
        assert torch.equal(per_cam[i], images[:, i]), cams[i]
    assert not torch.equal(images[:, 0], images[:, 1])  # two different viewpoints
    # fp32 CPU reference module with the same weights on the NCHW form of the same input
    ref = ActModel(num_cams=2).eval()
    sd = {k: v.float().cpu() for k, v in ro.policy.state_dict().items() if not k.startswith("_fused.")}
    ref.load_state_dict(sd)
    imgs = images if images.dim() == 5 and images.shape[-1] != 16 else torch.stack(
        [_s2d_to_nchw(images[:, i].cpu()) for i in range(2)], dim=1)
    if imgs.dtype == torch.uint8:
        # the fp32 rollout's 8-bit frame: the reference's ToDtype(scale) + ImageNet normalisation,
        # computed here on the CPU in f32 (independent of the product's kernels)
        m = torch.tensor(ro.image_norm[0], dtype=torch.float32).reshape(1, 1, 3, 1, 1)
        s = torch.tensor(ro.image_norm[1], dtype=torch.float32).reshape(1, 1, 3, 1, 1)
        imgs = (imgs.cpu().float() / 255.0 - m) / s
    want = ref(state.float().cpu(), imgs.float().cpu())
    err = (out.cpu() - want).abs().max().item()
    print(f"\ntwo-camera ACT fp32 device vs CPU: max |d chunk| {err:.3e}")
    assert err <= 1e-4 * max(1.0, want.abs().max().item())
    assert np.isfinite(ro.env.engine.qpos.cpu().numpy()).all()
