"""Batched RolloutAct: policy/act/RolloutAct.py of the reference for n_env envs.

infer_policy (RolloutAct.py:68-101): state + rendered images -> ACT chunk [n,100,7] -> per-env
chunk history + temporal ensembling + denormalisation in one HIP kernel (rmbx_act_ensemble),
bit-exact with the reference's f64 numpy arithmetic.
"""


import torch

from ... import kernels as K
from ...common.rollout_base import BatchedRolloutBase
from .act_model import IMAGENET_MEAN, IMAGENET_STD, ActModel
from .checkpoint import load_act_checkpoint


class RolloutAct(BatchedRolloutBase):
    policy_name = "Act"
    # ACTPolicy.__call__ normalises with ImageNet statistics before the backbone
    image_norm = (IMAGENET_MEAN, IMAGENET_STD)

    def set_additional_args(self, parser):
        parser.add_argument("--no_temp_ensem", action="store_true",
                            help="whether to disable temporal ensembling of the inferred policy")
        parser.add_argument("--act_prune_dead_decoder", action="store_true",
                            help="skip ACT decoder layers 1..6 whose outputs the reference discards")

    def setup_policy(self):
        meta = self.model_meta_info
        self.chunk_size = meta["data"]["chunk_size"]
        args = meta["policy"].get("args", {})
        self.policy = ActModel(
            state_dim=len(meta["state"]["example"]), action_dim=len(meta["action"]["example"]),
            num_queries=self.chunk_size, hidden_dim=args.get("hidden_dim", 512),
            dim_feedforward=args.get("dim_feedforward", 3200), nheads=args.get("nheads", 8),
            enc_layers=args.get("enc_layers", 4), dec_layers=args.get("dec_layers", 7),
            num_cams=len(meta["image"]["camera_names"]),
        )
        if self.args.checkpoint:
            # the reference's ACTPolicy checkpoint (or ActModel's own), strictly (RolloutBase.py:376-385)
            load_act_checkpoint(self.policy, self.args.checkpoint)
        self.policy.prune_dead_decoder = bool(self.args.act_prune_dead_decoder)
        # the 8-bit stem folds in the same (mean, std) the renderer applies to float policy images
        self.policy.u8_image_norm = tuple(tuple(float(v) for v in x) for x in self.image_norm)
        self.policy_dtype = torch.bfloat16 if self.args.precision == "bf16" else torch.float32
        if self.policy_dtype == torch.float32:
            # the reference's precision: IEEE fp32 convolutions and GEMMs, never a TF32-style
            # reduced-mantissa mode (torch enables it for cuDNN/MIOpen convs by default)
            torch.backends.cudnn.allow_tf32 = False
            torch.backends.cuda.matmul.allow_tf32 = False
        # MIOpen Find (measured solver choice per conv shape; once per shape, during warm-up):
        # 66 -> 53 ms for the 1024-env trunk on MI355X (scripts/prof_act.py)
        torch.backends.cudnn.benchmark = True
        # (MIOpen's naive reference solver, which Find times for seconds per shape at 1024-env batch
        # sizes and never selects, is excluded by bench.py / bin/Rollout.py for large batches via
        # MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0: process-wide, so not set here, where a
        # diffusion policy's small convs may need it)
        self.policy = self.policy.eval().requires_grad_(False)
        self.policy.fuse_backbone()
        self.policy = self.policy.to(device=self.device, dtype=self.policy_dtype).requires_grad_(False)
        self.policy._fused = self.policy._fused.to(memory_format=torch.channels_last)
        if self.device.type == "cuda":
            from ...common.tuning import enable_gemm_tuning

            self.policy.fuse_transformer()
            enable_gemm_tuning()

    def reset_variables(self):
        self.ens = K.ActEnsembleState(self.n, self.chunk_size, self.action_dim, self.model_meta_info["action"],
                                      self.device, temporal_ensemble=not self.args.no_temp_ensem)
        self._calls = 0

    @torch.no_grad()
    def infer_policy(self):
        te = not self.args.no_temp_ensem
        push = te or (self._calls % self.chunk_size == 0)
        chunk = None
        if push:
            state = self.get_state()
            images = self.get_images(self.policy_dtype)
            chunk = self.policy(state.to(self.policy_dtype), images).float().contiguous()
        p = None if te else torch.full((self.n,), int(push), dtype=torch.uint8, device=self.device)
        self.policy_action = self.ens(chunk, push=p)
        self._calls += 1
