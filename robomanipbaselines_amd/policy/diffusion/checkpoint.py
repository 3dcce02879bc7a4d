"""Strict loading of the reference's diffusion-policy checkpoints onto the restated modules.

RolloutBase.load_ckpt (common/base/RolloutBase.py:376-385) loads `policy_*.ckpt` into the
upstream policy with a strict `load_state_dict`; TrainBase saves `policy.state_dict()`
(common/base/TrainBase.py:470-482; the EMA copy when --use_ema, same keys).  The upstream modules
live in absent submodules, so their key layout is restated from the public sources:

* DiffusionUnetHybridImagePolicy (diffusion_policy/policy/diffusion_unet_hybrid_image_policy.py):
  `obs_encoder` = robomimic ObservationEncoder, one VisualCore per rgb key
  `obs_encoder.obs_nets.<camera>_rgb_image.` (DataKey.get_rgb_image_key, DataKey.py:201-203) with
  `backbone.nets.*` (ResNet18Conv children[:-2], BatchNorm replaced by GroupNorm), `pool.*`
  (SpatialSoftmax: `nets` 1x1 conv, `pos_x` / `pos_y` buffers) and the feature Linear; VisualCore
  also registers the same modules again inside `nets` (Sequential(backbone, pool, Flatten,
  Linear)), so `nets.0.*`, `nets.1.*`, `nets.3.*` alias `backbone.*`, `pool.*`, the Linear;
  `model.*` = ConditionalUnet1D (same names here); `normalizer.*` = LinearNormalizer.
* DP3 (3D-Diffusion-Policy/diffusion_policy_3d/policy/dp3.py): `obs_encoder.extractor.*`
  (PointNetEncoderXYZ[RGB] mlp / final_projection), `obs_encoder.state_mlp.*`, `model.*`,
  `normalizer.*` -- the same names as DP3Model.

The RoboManipBaselines rollouts feed already-normalised data, so a normalizer that is present must
be the identity (scale 1, offset 0); anything else, any unmapped key, any missing parameter and
any disagreeing alias fails loudly (ValueError), never a silent partial load."""

import re

import torch


def _check_normalizer(key, value):
    if key.endswith(".scale") and not torch.all(value == 1):
        raise ValueError(f"non-identity normalizer {key}: the rollout feeds normalised data")
    if key.endswith(".offset") and not torch.all(value == 0):
        raise ValueError(f"non-identity normalizer {key}: the rollout feeds normalised data")


def _is_dummy(key, value):
    """diffusion_policy's ModuleAttrMixin registers `_dummy_variable = nn.Parameter()` (an empty
    tensor used only to find the module's device/dtype) on the policy and on its
    LowdimMaskGenerator, so a real state_dict carries `_dummy_variable` and
    `mask_generator._dummy_variable`.  They hold no weights; drop them (an empty tensor only)."""
    return (key == "_dummy_variable" or key.endswith("._dummy_variable")) and value.numel() == 0


def _put(out, key, value, src):
    if key in out:
        if out[key].shape != value.shape or not torch.equal(out[key], value):
            raise ValueError(f"checkpoint aliases disagree for {key} ({src})")
        return
    out[key] = value


def dp_state_dict_from_reference(sd, camera_names):
    """Map a DiffusionUnetHybridImagePolicy state_dict (or DiffusionPolicyModel's own) onto
    DiffusionPolicyModel's names."""
    cams = {f"{c.lower()}_rgb_image": i for i, c in enumerate(camera_names)}
    vis = re.compile(r"^obs_encoder\.obs_nets\.([^.]+)\.(.*)$")
    out, unexpected = {}, []
    for k, v in sd.items():
        if _is_dummy(k, v):
            continue
        if k.startswith("model.") or k.startswith("obs_nets."):
            _put(out, k, v, k)
            continue
        if k.startswith("normalizer."):
            _check_normalizer(k, v)
            continue
        m = vis.match(k)
        if m and m.group(1) in cams:
            ci, rest = cams[m.group(1)], m.group(2)
            for src, dst in (("backbone.", "backbone."), ("nets.0.", "backbone."), ("pool.", "pool."),
                             ("nets.1.", "pool."), ("linear.", "linear."), ("nets.3.", "linear.")):
                if rest.startswith(src):
                    _put(out, f"obs_nets.{ci}.{dst}{rest[len(src):]}", v, k)
                    break
            else:
                unexpected.append(k)
            continue
        unexpected.append(k)
    if unexpected:
        raise ValueError(f"unexpected keys in the DiffusionPolicy checkpoint: {unexpected[:8]}"
                         f"{' ...' if len(unexpected) > 8 else ''}")
    return out


def dp3_state_dict_from_reference(sd):
    """Map a DP3 state_dict onto DP3Model's names (identical apart from the normalizer)."""
    out, unexpected = {}, []
    for k, v in sd.items():
        if _is_dummy(k, v):
            continue
        if k.startswith("normalizer."):
            _check_normalizer(k, v)
        elif k.startswith("model.") or k.startswith("obs_encoder."):
            out[k] = v
        else:
            unexpected.append(k)
    if unexpected:
        raise ValueError(f"unexpected keys in the DP3 checkpoint: {unexpected[:8]}")
    return out


def _load_sd(path_or_sd):
    if isinstance(path_or_sd, dict):
        return path_or_sd
    sd = torch.load(path_or_sd, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    return sd


def load_dp_checkpoint(model, path_or_sd, camera_names):
    """Strict load (RolloutBase.py:376-385): missing or unexpected keys raise."""
    model.load_state_dict(dp_state_dict_from_reference(_load_sd(path_or_sd), camera_names), strict=True)
    return model


def load_dp3_checkpoint(model, path_or_sd):
    model.load_state_dict(dp3_state_dict_from_reference(_load_sd(path_or_sd)), strict=True)
    return model
