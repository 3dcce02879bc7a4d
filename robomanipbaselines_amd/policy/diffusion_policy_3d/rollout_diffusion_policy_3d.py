"""Batched RolloutDiffusionPolicy3d: policy/diffusion_policy_3d/RolloutDiffusionPolicy3d.py of
the reference for n_env envs.

* get_pointcloud (:132-160): renderer rgb + depth of the first camera -> cv2.resize to
  image_size (rmbx_resize_crop_u8 / rmbx_resize_f32) -> rmbx_pointcloud_fps (depth -> points,
  bounding-box crop, farthest point sampling to num_points, normalisation) -> n_obs_steps
  history [n, To, P, 6].
* get_state (:110-130), infer_policy (:83-101): as DiffusionPolicy, with the 10-step DDIM loop
  (HIP-graph captured) and the pop + denormalisation kernel.
Defaults for synthetic runs follow misc/AddPointCloudToRmbData.py:29-55 (84x84 images, bounds
[-0.4]^3 .. [1.0]^3, 512 points) and TrainDiffusionPolicy3d.py:54-84 (limits normalisation,
horizon 16, 2 obs steps, 8 action steps, no colour, encoder output 64).
"""

import numpy as np
import torch

from ... import kernels as K
from ..diffusion_policy.rollout_diffusion_policy import RolloutDiffusionPolicy, _limits_meta
from ..diffusion.checkpoint import load_dp3_checkpoint
from .dp3_model import DP3Model


class RolloutDiffusionPolicy3d(RolloutDiffusionPolicy):
    policy_name = "DiffusionPolicy3d"

    def setup_model_meta_info(self):
        super(RolloutDiffusionPolicy, self).setup_model_meta_info()
        meta = self.model_meta_info
        if meta["data"].get("name") == "synthetic":
            _limits_meta(meta)
            lo, hi = [-0.4, -0.4, -0.4], [1.0, 1.0, 1.0]
            meta["data"].update({"horizon": 16, "n_obs_steps": 2, "n_action_steps": 8, "use_pc_color": False,
                                 "num_points": 512, "n_point_dim": 3, "image_size": [84, 84],
                                 "min_bound": lo, "max_bound": hi})
            mn = np.array(lo + [0.0, 0.0, 0.0])
            mx = np.array(hi + [1.0, 1.0, 1.0])
            meta["pointcloud"] = {"norm_config": {"type": "limits", "out_min": -1.0, "out_max": 1.0},
                                  "min": mn, "max": mx, "range": mx - mn}

    def setup_policy(self):
        meta = self.model_meta_info
        d = meta["data"]
        self.n_obs_steps, self.n_action_steps = int(d["n_obs_steps"]), int(d["n_action_steps"])
        self.image_size = list(d["image_size"])
        self.num_points = int(d["num_points"])
        self.policy = DP3Model(len(meta["state"]["example"]), len(meta["action"]["example"]), horizon=int(d["horizon"]),
                               n_obs_steps=self.n_obs_steps, n_action_steps=self.n_action_steps,
                               use_pc_color=bool(d["use_pc_color"]))
        if self.args.checkpoint:
            # the reference's DP3 checkpoint, strictly (RolloutBase.py:376-385)
            load_dp3_checkpoint(self.policy, self.args.checkpoint)
        self.policy_dtype = torch.bfloat16 if self.args.precision == "bf16" else torch.float32
        # the DP3 encoder is PointNet Linears and the UNet's convs are GEMMs (deterministic
        # hipBLASLt) in both precisions: no MIOpen call in the captured denoising loop
        torch.backends.cudnn.benchmark = False
        torch.backends.cudnn.deterministic = True
        self.policy = self.policy.eval().requires_grad_(False).to(device=self.device, dtype=self.policy_dtype)

    def reset_variables(self):
        super().reset_variables()
        self.pointcloud_buf = None

    def get_pointcloud(self):
        """RolloutDiffusionPolicy3d.get_pointcloud (:127-171): info["rgb_images"] and
        info["depth_images"] of the first camera from the last env-step."""
        cam = self.camera_names[0]
        rgb, depth = self.info["rgb_images"][cam], self.info["depth_images"][cam]
        rw, rh = self.image_size
        rgb_s = K.resize_crop_u8(rgb, (rw, rh), None, dtype=torch.uint8)
        depth_s = K.resize_f32(depth, (rw, rh))
        d = self.model_meta_info["data"]
        pc, self.pc_count, _ = K.pointcloud_fps(depth_s, rgb_s, self.env.get_camera_fovy(cam), self.num_points,
                                                self.model_meta_info["pointcloud"], d["min_bound"], d["max_bound"])
        if self.pointcloud_buf is None:
            self.pointcloud_buf = pc[:, None].repeat(1, self.n_obs_steps, 1, 1)
        else:
            self.pointcloud_buf = torch.cat([self.pointcloud_buf[:, 1:], pc[:, None]], dim=1)
        return self.pointcloud_buf

    @torch.no_grad()
    def infer_policy(self):
        push = self._calls % self.n_action_steps == 0
        chunk = None
        if push:
            state = self.get_state()
            pc = self.get_pointcloud()
            chunk = self.policy.predict_action(state, pc, use_graph=not self.args.no_graph).float().contiguous()
        p = torch.full((self.n,), int(push), dtype=torch.uint8, device=self.device)
        self.policy_action = self.ens(chunk, push=p)
        self._calls += 1
