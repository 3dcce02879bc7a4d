"""Batched RolloutDiffusionPolicy: policy/diffusion_policy/RolloutDiffusionPolicy.py of the
reference for n_env envs.

* get_state (:89-105): normalised state, n_obs_steps history -> [n, To, S].
* get_images (:107-138): renderer u8 frames -> rmbx_resize_crop_u8 (cv2.resize to image_size,
  ToDtype(scale), * 2 - 1, and the obs encoder's eval centre crop to image_crop_size) ->
  n_obs_steps history [n, ncam, To, 3, ch, cw].
* infer_policy (:66-87): when the action buffer is empty, predict_action (obs encoder + 100-step
  DDPM loop, HIP-graph captured) -> n_action_steps actions; each call pops one and
  denormalises it (rmbx_act_ensemble, no-ensemble mode, bit-exact f64).
Training-side defaults (TrainDiffusionPolicy.py:26-84): limits normalisation to [-1, 1],
horizon 16, n_obs_steps 2, n_action_steps 8, image_size 320x240, crop 288x216.
"""

import numpy as np
import os

import torch

from ... import kernels as K
from ...common.rollout_base import BatchedRolloutBase
from ..diffusion.checkpoint import load_dp_checkpoint
from .dp_model import DiffusionPolicyModel


def _limits_meta(meta, out_min=-1.0, out_max=1.0):
    for key in ("state", "action"):
        meta[key]["norm_config"] = {"type": "limits", "out_min": out_min, "out_max": out_max}


class RolloutDiffusionPolicy(BatchedRolloutBase):
    policy_name = "DiffusionPolicy"

    def set_additional_args(self, parser):
        parser.add_argument("--no_graph", action="store_true", help="run the denoising loop eagerly")

    def setup_model_meta_info(self):
        super().setup_model_meta_info()
        meta = self.model_meta_info
        if meta["data"].get("name") == "synthetic":
            _limits_meta(meta)
            meta["data"].update({"horizon": 16, "n_obs_steps": 2, "n_action_steps": 8,
                                 "image_size": [320, 240], "image_crop_size": [288, 216]})

    def setup_policy(self):
        meta = self.model_meta_info
        d = meta["data"]
        self.n_obs_steps, self.n_action_steps = int(d["n_obs_steps"]), int(d["n_action_steps"])
        self.image_size, self.crop_size = list(d["image_size"]), list(d["image_crop_size"])
        self.policy = DiffusionPolicyModel(
            len(meta["state"]["example"]), len(meta["action"]["example"]), len(meta["image"]["camera_names"]),
            horizon=int(d["horizon"]), n_obs_steps=self.n_obs_steps, n_action_steps=self.n_action_steps,
            crop_hw=(self.crop_size[1], self.crop_size[0]), num_inference_steps=100)
        if self.args.checkpoint:
            # the reference's DiffusionUnetHybridImagePolicy checkpoint, strictly (RolloutBase.py:376-385)
            load_dp_checkpoint(self.policy, self.args.checkpoint, self.camera_names)
        self.policy_dtype = torch.bfloat16 if self.args.precision == "bf16" else torch.float32
        # (the UNet's convs are GEMMs in both precisions, so MIOpen serves the image encoder only:
        # Find picks its solvers once per shape, outside the captured denoising loop).  fp32 is the
        # parity mode: deterministic MIOpen solvers only (no atomic split-K), so a seed reproduces
        # its episodes bit for bit, as the reference's TrainDiffusionPolicy/rollout setup intends
        torch.backends.cudnn.benchmark = True
        torch.backends.cudnn.deterministic = (self.policy_dtype == torch.float32
                                              and os.environ.get("RMBX_DP_DETERMINISTIC", "1") != "0")
        self.policy = self.policy.eval().requires_grad_(False).to(device=self.device, dtype=self.policy_dtype)
        self.policy.obs_nets = self.policy.obs_nets.to(memory_format=torch.channels_last)

    def reset_variables(self):
        self.ens = K.ActEnsembleState(self.n, self.n_action_steps, self.action_dim, self.model_meta_info["action"],
                                      self.device, temporal_ensemble=False)
        self.state_buf = None
        self.images_buf = None
        self._calls = 0

    def get_state(self):
        s = super().get_state()
        if self.state_buf is None:
            self.state_buf = s[:, None].repeat(1, self.n_obs_steps, 1)
        else:
            self.state_buf = torch.cat([self.state_buf[:, 1:], s[:, None]], dim=1)
        return self.state_buf

    def get_images(self, dtype):
        """RolloutDiffusionPolicy.get_images (:111-143): info["rgb_images"][camera] of the last
        env-step, resized / scaled / cropped on the device."""
        rw, rh = self.image_size
        cw, ch = self.crop_size
        crop = ((rh - ch) // 2, (rw - cw) // 2, ch, cw)
        imgs = []
        for cam in self.camera_names:
            rgb = self.info["rgb_images"][cam]
            imgs.append(K.resize_crop_u8(rgb, (rw, rh), crop, a=2.0, b=-1.0, dtype=dtype))
        img = torch.stack(imgs, dim=1)  # [n, ncam, 3, ch, cw]
        if self.images_buf is None:
            self.images_buf = img[:, :, None].repeat(1, 1, self.n_obs_steps, 1, 1, 1)
        else:
            self.images_buf = torch.cat([self.images_buf[:, :, 1:], img[:, :, None]], dim=2)
        return self.images_buf

    @torch.no_grad()
    def infer_policy(self):
        push = self._calls % self.n_action_steps == 0
        chunk = None
        if push:
            state = self.get_state()
            images = self.get_images(self.policy_dtype)
            chunk = self.policy.predict_action(state, images, use_graph=not self.args.no_graph).float().contiguous()
        p = torch.full((self.n,), int(push), dtype=torch.uint8, device=self.device)
        self.policy_action = self.ens(chunk, push=p)
        self._calls += 1
