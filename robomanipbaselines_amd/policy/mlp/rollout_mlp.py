"""Batched RolloutMlp: policy/mlp/RolloutMlp.py of the reference for n_env envs.

* get_state (:48-72): normalised joint state, kept as an n_obs_steps history (first call fills
  it with copies, later calls shift by one) -> [n, n_obs, S] f32.
* get_images (:74-105): rendered [0, 1] images (v2.ToDtype(scale=True), no ImageNet
  normalisation), same n_obs history per camera -> [n, ncam, n_obs, 3, H, W].
* infer_policy (:107-124): when the per-env action buffer is empty run the network and load
  its n_action_steps actions; every call pops the first one (f32 -> f64) and denormalises it.
  The pop + denormalisation run in the rmbx_act_ensemble kernel in its no-ensemble mode
  (bit-exact f64 `std * a + mean`, DataUtils.py:26-40); envs step in lockstep, so the buffer
  refills on the same call for every env.
"""


import torch

from ... import kernels as K
from ...common.rollout_base import BatchedRolloutBase
from .mlp_model import MlpModel


class RolloutMlp(BatchedRolloutBase):
    policy_name = "Mlp"

    def setup_policy(self):
        meta = self.model_meta_info
        args = dict(meta["policy"].get("args", {}))
        self.n_obs_steps = int(args.pop("n_obs_steps", meta["data"].get("n_obs_steps", 1)))
        self.n_action_steps = int(args.pop("n_action_steps", meta["data"].get("n_action_steps", 1)))
        self.policy = MlpModel(len(meta["state"]["example"]), len(meta["action"]["example"]),
                               len(meta["image"]["camera_names"]), n_obs_steps=self.n_obs_steps,
                               n_action_steps=self.n_action_steps,
                               hidden_dim_list=args.get("hidden_dim_list", [512, 512]),
                               state_feature_dim=args.get("state_feature_dim", 512))
        if self.args.checkpoint:
            sd = torch.load(self.args.checkpoint, map_location="cpu", weights_only=True)
            self.policy.load_state_dict(sd)
        self.policy_dtype = torch.bfloat16 if self.args.precision == "bf16" else torch.float32
        if self.policy_dtype == torch.float32:
            # the reference's precision: IEEE fp32 convolutions and GEMMs, no TF32-class mode
            torch.backends.cudnn.allow_tf32 = False
            torch.backends.cuda.matmul.allow_tf32 = False
        self.policy = self.policy.eval().requires_grad_(False)
        self.policy.fuse_backbone()
        torch.backends.cudnn.benchmark = True
        # (MIOpen's naive reference solver, which Find times for seconds per shape at 1024-env batch
        # sizes and never selects, is excluded by bench.py / bin/Rollout.py for large batches via
        # MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0: process-wide, so not set here, where a
        # diffusion policy's small convs may need it)
        self.policy = self.policy.to(device=self.device, dtype=self.policy_dtype)
        self.policy._fused = self.policy._fused.to(memory_format=torch.channels_last)

    def reset_variables(self):
        self.ens = K.ActEnsembleState(self.n, self.n_action_steps, self.action_dim, self.model_meta_info["action"],
                                      self.device, temporal_ensemble=False)
        self.state_buf = None
        self.images_buf = None
        self._calls = 0

    def get_state(self):
        s = super().get_state()  # [n, S] f32
        if self.state_buf is None:
            self.state_buf = s[:, None].repeat(1, self.n_obs_steps, 1)
        else:
            self.state_buf = torch.cat([self.state_buf[:, 1:], s[:, None]], dim=1)
        return self.state_buf

    def get_images(self, dtype):
        img = super().get_images(dtype)  # [n, ncam, 3, H, W]
        if self.n_obs_steps == 1:
            return img[:, :, None]
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
            chunk = self.policy(state.to(self.policy_dtype), images).float().contiguous()
        p = torch.full((self.n,), int(push), dtype=torch.uint8, device=self.device)
        self.policy_action = self.ens(chunk, push=p)
        self._calls += 1
