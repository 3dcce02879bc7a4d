"""3D Diffusion Policy (DP3) inference, batched over environments.

Restates the inference path of 3D-Diffusion-Policy's DP3 (public upstream
3D-Diffusion-Policy/diffusion_policy_3d/policy/dp3.py and model/vision/pointnet_extractor.py; the
reference's third_party/3D-Diffusion-Policy submodule is absent) with the reference's
configuration (policy/diffusion_policy_3d/TrainDiffusionPolicy3d.py:163-211): DP3Encoder =
PointNet (per-point Linear-LayerNorm-ReLU 3->64->128->256, or 6->64->128->256->512 with colour,
max-pool, Linear->encoder_output_dim (64) + LayerNorm) + state MLP (S->64->ReLU->64);
global conditioning on n_obs_steps (2) encoded steps; ConditionalUnet1D (down [512, 1024, 2048],
k 5, 8 groups, FiLM); DDIMScheduler (prediction "sample", 10 steps); action =
prediction[:, To-1 : To-1+8].  Normalizer = identity (inputs arrive normalised,
RolloutDiffusionPolicy3d.py:83-160).  Parity vs upstream: unpinned.
"""

import torch
import torch.nn as nn

from ..diffusion.unet1d import ConditionalUnet1D
from ..diffusion_policy.dp_model import DiffusionPolicyModel


class PointNetEncoder(nn.Module):
    def __init__(self, in_channels=3, out_channels=64):
        super().__init__()
        blocks = [64, 128, 256] if in_channels == 3 else [64, 128, 256, 512]
        layers, c = [], in_channels
        for b in blocks:
            layers += [nn.Linear(c, b), nn.LayerNorm(b), nn.ReLU()]
            c = b
        self.mlp = nn.Sequential(*layers)
        self.final_projection = nn.Sequential(nn.Linear(c, out_channels), nn.LayerNorm(out_channels))

    def forward(self, x):
        return self.final_projection(torch.max(self.mlp(x), 1)[0])


class DP3Encoder(nn.Module):
    def __init__(self, state_dim, use_pc_color=False, out_channels=64, state_mlp_size=(64, 64)):
        super().__init__()
        self.use_pc_color = use_pc_color
        self.extractor = PointNetEncoder(6 if use_pc_color else 3, out_channels)
        self.state_mlp = nn.Sequential(nn.Linear(state_dim, state_mlp_size[0]), nn.ReLU(),
                                       nn.Linear(state_mlp_size[0], state_mlp_size[1]))
        self.out_dim = out_channels + state_mlp_size[-1]

    def forward(self, points, state):
        return torch.cat([self.extractor(points), self.state_mlp(state)], dim=-1)


class DP3Model(DiffusionPolicyModel):
    """predict_action(state [B, To, S], point_cloud [B, To, P, 6]) -> [B, n_action, A]."""

    def __init__(self, state_dim, action_dim, horizon=16, n_obs_steps=2, n_action_steps=8, use_pc_color=False,
                 encoder_output_dim=64, num_inference_steps=10, down_dims=(512, 1024, 2048), kernel_size=5,
                 n_groups=8, diffusion_step_embed_dim=128, eps_mode=0):
        nn.Module.__init__(self)
        self.horizon, self.n_obs_steps, self.n_action_steps = horizon, n_obs_steps, n_action_steps
        self.action_dim, self.state_dim = action_dim, state_dim
        self.obs_encoder = DP3Encoder(state_dim, use_pc_color, encoder_output_dim)
        self.obs_feature_dim = self.obs_encoder.out_dim
        self.model = ConditionalUnet1D(action_dim, self.obs_feature_dim * n_obs_steps, diffusion_step_embed_dim,
                                       down_dims, kernel_size, n_groups, cond_predict_scale=True)
        from ..diffusion.schedulers import DDIMSampler

        self.sampler = DDIMSampler(num_train_timesteps=100, num_inference_steps=num_inference_steps, eps_mode=eps_mode)
        self._graphs = {}

    def encode_obs(self, state, points):
        B, To = state.shape[:2]
        pc = points[:, :To]
        if not self.obs_encoder.use_pc_color:
            pc = pc[..., :3]
        f = self.obs_encoder(pc.reshape(B * To, *pc.shape[2:]).to(self.dtype), state[:, :To].reshape(B * To, -1).to(self.dtype))
        return f.reshape(B, -1)
