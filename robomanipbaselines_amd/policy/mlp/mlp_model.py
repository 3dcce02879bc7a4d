"""MLP policy with a ResNet-18 image trunk, batched over environments.

Restates policy/mlp/MlpPolicy.py:7-111 of the reference: state features ReLU(Linear(S*n_obs ->
state_feature_dim)); per image ResNet-18 (FrozenBN, no fc) -> 512-d global-average feature;
concat -> [Linear -> ReLU]* over hidden_dim_list -> Linear -> action_dim * n_action_steps;
kaiming-normal Linear weights with zero bias (:66-71).  Module names match the reference's so a
reference `policy_*.ckpt` state_dict loads with strict=True (`image_feature_extractor.0` =
conv1, `.1` = bn1, `.4`-`.7` = layer1-4, as torchvision's `children()[:-1]`).

Batched call form: forward(state_seq [B, n_obs, S], images_seq [B, ncam, n_obs, 3, H, W]) ->
[B, n_action_steps, A].  (The reference stacks cameras in front of the batch axis,
RolloutMlp.py:99-104, which is the same thing at its batch size 1.)

Inference path on the device: the trunk runs through FusedResNet18Trunk (BN folded, MIOpen
convs + rmbx HIP epilogues) in bf16 or fp32; the unfused module is the fp32 reference.
"""

import types

import torch
import torch.nn as nn

from ..backbone import FusedResNet18Trunk, ResNet18Trunk


class MlpModel(nn.Module):
    def __init__(self, state_dim, action_dim, num_images, n_obs_steps=1, n_action_steps=1,
                 hidden_dim_list=(512, 512), state_feature_dim=512):
        super().__init__()
        self.n_obs_steps, self.n_action_steps = n_obs_steps, n_action_steps
        self.state_feature_extractor = nn.Sequential(nn.Linear(state_dim * n_obs_steps, state_feature_dim), nn.ReLU())
        t = ResNet18Trunk()
        self.image_feature_extractor = nn.Sequential(
            t.conv1, t.bn1, nn.ReLU(), nn.MaxPool2d(3, 2, 1), t.layer1, t.layer2, t.layer3, t.layer4,
            nn.AdaptiveAvgPool2d((1, 1)))
        dims = [state_feature_dim + num_images * n_obs_steps * 512] + list(hidden_dim_list) + [action_dim * n_action_steps]
        layers = []
        for i in range(len(dims) - 1):
            layers.append(nn.Linear(dims[i], dims[i + 1]))
            if i < len(dims) - 2:
                layers.append(nn.ReLU())
        self.linear_layer_seq = nn.Sequential(*layers)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.kaiming_normal_(m.weight, nonlinearity="relu")
                nn.init.zeros_(m.bias)
        self._fused = None

    def _trunk_view(self):
        s = self.image_feature_extractor
        return types.SimpleNamespace(conv1=s[0], bn1=s[1], layer1=s[4], layer2=s[5], layer3=s[6], layer4=s[7])

    def fuse_backbone(self):
        # kept out of the module tree so the state_dict keeps the reference's keys
        object.__setattr__(self, "_fused", FusedResNet18Trunk(self._trunk_view()))
        return self

    def _apply(self, fn, *args, **kwargs):
        super()._apply(fn, *args, **kwargs)
        if self._fused is not None:
            self._fused._apply(fn, *args, **kwargs)
        return self

    @property
    def accepts_s2d(self):
        return self._fused is not None

    def image_features(self, x):
        """[B, 3, H, W] in [0, 1] (or the space-to-depth form [B, H/2, W/2, 16]) -> [B, 512]."""
        if self._fused is not None:
            if x.shape[-1] == 16 and x.dim() == 4:
                f = self._fused.forward_s2d(x.contiguous())
            else:
                f = self._fused(x.contiguous(memory_format=torch.channels_last))
            return f.float().mean(dim=(2, 3)).to(f.dtype)
        return self.image_feature_extractor(x).flatten(1)

    def forward(self, state_seq, images_seq):
        B = state_seq.shape[0]
        feats = [self.state_feature_extractor(state_seq.reshape(B, -1))]
        imgs = images_seq.reshape(B, -1, *images_seq.shape[-3:])
        for i in range(imgs.shape[1]):
            feats.append(self.image_features(imgs[:, i]))
        out = self.linear_layer_seq(torch.cat(feats, dim=1))
        return out.reshape(B, self.n_action_steps, -1)
