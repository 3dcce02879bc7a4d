"""Trained-ACT checkpoint loading.

The reference saves `ACTPolicy.state_dict()` as `policy_*.ckpt` and loads it back strictly with
`torch.load(path, weights_only=True)` (common/base/RolloutBase.py:376-385).  ACTPolicy wraps
DETRVAE as `self.model` (third_party/act policy.py [absent]; public upstream tonyzhaozh/act), so
the keys are:

    model.backbones.0.0.body.{conv1,bn1,layer1..layer4}.*     torchvision resnet18 trunk
                                                              (Joiner(backbone, pos)[0].body =
                                                              IntermediateLayerGetter, FrozenBN)
    model.transformer.encoder.layers.{i}.*                    post-norm encoder layers
    model.transformer.decoder.layers.{i}.*, .decoder.norm.*   decoder layers + final norm
    model.{input_proj, input_proj_robot_state, latent_out_proj, query_embed,
           additional_pos_embed, action_head, is_pad_head}.*
    model.{encoder.*, cls_embed, encoder_action_proj, encoder_joint_proj, latent_proj, pos_table}
                                                              CVAE encoder: training only

`act_state_dict_from_reference` maps those names onto ActModel (which keeps the upstream leaf
names: self_attn.in_proj_weight, linear1, norm1, ...), drops the training-only CVAE keys and
fails loudly on anything else, so a reference checkpoint either loads completely or not at all.
ActModel's own state_dict (what `torch.save(model.state_dict())` writes here) loads unchanged.
"""

import re

import torch

# DETRVAE modules used only by the CVAE posterior during training (latent is zero at inference)
_TRAINING_ONLY = ("encoder.", "cls_embed.", "encoder_action_proj.", "encoder_joint_proj.", "latent_proj.")
_TRAINING_ONLY_EXACT = ("pos_table",)

_RULES = [
    (re.compile(r"^backbones\.0\.0\.body\."), "backbone."),
    (re.compile(r"^transformer\.encoder\.layers\.(\d+)\."), r"encoder_layers.\1."),
    (re.compile(r"^transformer\.decoder\.layers\.(\d+)\."), r"decoder_layers.\1."),
    (re.compile(r"^transformer\.decoder\.norm\."), "decoder_norm."),
]


def is_reference_state_dict(sd):
    return any(k.startswith("model.") or k.startswith("backbones.") or k.startswith("transformer.") for k in sd)


def act_state_dict_from_reference(sd):
    """ACTPolicy / DETRVAE state_dict -> ActModel state_dict (tensors shared, not copied)."""
    out = {}
    for key, val in sd.items():
        k = key[len("model."):] if key.startswith("model.") else key
        if k.startswith(_TRAINING_ONLY) or k in _TRAINING_ONLY_EXACT:
            continue
        if k.startswith("backbones.0.1."):  # the sine position embedding has no parameters
            continue
        for pat, rep in _RULES:
            if pat.match(k):
                k = pat.sub(rep, k, count=1)
                break
        out[k] = val
    return out


def load_act_checkpoint(model, path_or_sd):
    """Load a checkpoint (path or state_dict) into an ActModel, strictly: every inference
    parameter/buffer must be present with the right shape and nothing unknown may be left over.
    Accepts the reference's ACTPolicy state_dict and ActModel's own."""
    sd = path_or_sd
    if not isinstance(sd, dict):
        sd = torch.load(path_or_sd, map_location="cpu", weights_only=True)
    if is_reference_state_dict(sd):
        sd = act_state_dict_from_reference(sd)
    own = model.state_dict()
    missing = sorted(set(own) - set(sd))
    unexpected = sorted(set(sd) - set(own))
    if missing or unexpected:
        raise ValueError(f"ACT checkpoint does not match the model: missing {missing[:8]}{'...' if len(missing) > 8 else ''}, "
                         f"unexpected {unexpected[:8]}{'...' if len(unexpected) > 8 else ''}")
    bad = [k for k in own if tuple(own[k].shape) != tuple(sd[k].shape)]
    if bad:
        raise ValueError("ACT checkpoint shape mismatch: " +
                         ", ".join(f"{k} {tuple(sd[k].shape)} vs {tuple(own[k].shape)}" for k in bad[:8]))
    model.load_state_dict(sd, strict=True)
    return model
