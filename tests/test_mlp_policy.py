"""MlpModel vs the reference's own MlpPolicy.forward (policy/mlp/MlpPolicy.py:7-111), from the
fixture tools/gen_golden.py minted by running the reference module (with the build's ResNet-18
restatement stubbed in for torchvision.resnet18, whose weights are a download).  The weights are
the build's MlpModel at the fixture's seed, loaded into the reference module with strict=True, so
the fixture pins the head, the feature order, the reshapes and the state_dict key names."""

import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN


def _model(d, name):
    from robomanipbaselines_amd.policy.backbone import FrozenBatchNorm2d
    from robomanipbaselines_amd.policy.mlp.mlp_model import MlpModel

    seed = int(d[f"{name}_seed"])
    n_obs, n_act, sfd = (int(x) for x in d[f"{name}_cfg"])
    torch.manual_seed(seed)
    m = MlpModel(7, 7, 1, n_obs_steps=n_obs, n_action_steps=n_act, hidden_dim_list=[int(h) for h in d[f"{name}_hidden"]],
                 state_feature_dim=sfd)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():  # the generator's frozen BN statistics, same draw order
        for mod in m.modules():
            if isinstance(mod, FrozenBatchNorm2d):
                mod.weight.copy_(torch.rand(mod.weight.shape, generator=g) + 0.5)
                mod.bias.copy_(torch.rand(mod.bias.shape, generator=g) * 0.4 - 0.2)
                mod.running_mean.copy_(torch.rand(mod.running_mean.shape, generator=g) * 0.4 - 0.2)
                mod.running_var.copy_(torch.rand(mod.running_var.shape, generator=g) * 1.5 + 0.5)
    return m.eval().requires_grad_(False)


@pytest.mark.parametrize("name", ["c1", "obs2_act4"])
def test_mlp_model_matches_reference_module_cpu(name):
    d = np.load(os.path.join(GOLDEN, "mlp_policy.npz"))
    m = _model(d, name)
    with torch.no_grad():
        got = m(torch.from_numpy(d[f"{name}_state"]), torch.from_numpy(d[f"{name}_images"])).numpy()
    want = d[f"{name}_action"]
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * np.abs(want).max())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1", "obs2_act4"])
def test_mlp_model_device_fp32_matches_reference_module(name):
    """The device inference form (BN folded, MIOpen convs + rmbx epilogues, fp32) against the
    reference module's outputs."""
    d = np.load(os.path.join(GOLDEN, "mlp_policy.npz"))
    m = _model(d, name).fuse_backbone().to("cuda:0")
    m._fused = m._fused.to(memory_format=torch.channels_last)
    with torch.no_grad():
        got = m(torch.from_numpy(d[f"{name}_state"]).cuda(), torch.from_numpy(d[f"{name}_images"]).cuda()).cpu().numpy()
    want = d[f"{name}_action"]
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4 * np.abs(want).max())
