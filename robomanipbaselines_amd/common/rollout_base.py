"""Batched rollout plugin base: n_env environments step in lockstep on one GPU.

Mirrors common/base/RolloutBase.py of the reference (hook names, argparse flags, phase
semantics, results schema) for a batch of envs:

* phases: InitialRolloutPhase (1.0 s), the Operation's pre-motion phases (timed reach/grasp),
  RolloutPhase (policy every `skip` steps, success latch, +1.0 s after success or max_duration,
  --auto_exit), EndRolloutPhase — RolloutBase.py:28-132, PhaseBase.py:41-106.  All phase
  transitions are driven by the simulation clock, so the pre-rollout schedule is identical for
  every env and is tracked on the host; per-env termination/results live in the device
  schedule (rmbx_sched_update).
* the step loop (RolloutBase.py:387-426): pre_update -> env action -> env.step ->
  post_update -> check_transition, with cv2.waitKey / plotting removed (headless).
* results: {"success": [...], "reward": [...], "duration": [...]} per env in env order, the
  `Rollout result: success|failure` stdout contract (RolloutBase.py:96-107) and the optional
  YAML file (RolloutBase.py:417-422); inference-duration statistics (RolloutBase.py:528-539).
"""

import argparse
import datetime
import os
import sys
import time

import numpy as np
import torch
import yaml

from .. import kernels as K
from ..common.data_key import DataKey, action_key_codes, state_key_codes
from ..common.data_utils import make_meta_info


class PhaseSpec:
    """Timed phase of the pre-rollout motion (PhaseBase.ReachPhaseBase / GraspPhaseBase)."""

    def __init__(self, name, duration, kind, pos_z=None, grip=None, target=None):
        # grip: gripper command of a grasp phase (None = action_space.high, set_target_close;
        # "low" = action_space.low, set_target_open; or a value)
        # target: reach phases of tasks other than the cable: callable(rollout) -> (R [n, 9],
        # p [n, 3]) f64 device tensors, the phase's set_target (evaluated when the phase starts)
        self.name, self.duration, self.kind, self.pos_z, self.grip = name, duration, kind, pos_z, grip
        self.target = target


class BatchedRolloutBase:
    require_task_desc = False
    policy_name = "Policy"

    def __init__(self, argv=None, **overrides):
        self.setup_args(argv=argv)
        for k, v in overrides.items():
            setattr(self.args, k, v)
        torch.manual_seed(self.args.seed)
        np.random.seed(self.args.seed)
        self.device = torch.device(self.args.device)
        self.setup_env()
        self.setup_model_meta_info()
        self.setup_policy()
        self.n = self.env.num_envs
        self.pre_phases = self.get_pre_motion_phases()
        self.pre_durations = [1.0] + [p.duration for p in self.pre_phases]  # Initial phase: 1.0 s
        self.result = {key: [] for key in ("success", "reward", "duration")}
        self.inference_duration_list = []
        self._infer_events = []
        self.datetime_now = datetime.datetime.now()
        self._active = None  # optional caller override of the per-env step mask
        self.phase_timer = None  # optional PhaseTimer (common/phase_timer.py): bench.py's per-phase split

    def attach_phase_timer(self, timer):
        """Record HIP events at the policy / render / physics / glue boundaries of every env-step
        (None detaches)."""
        self.phase_timer = timer
        self.env.phase_timer = timer

    def _mark(self, label):
        if self.phase_timer is not None:
            self.phase_timer.mark(label)

    # -- arguments (RolloutBase.setup_args :165-284 + batching flags) --------------------------
    def setup_args(self, parser=None, argv=None):
        if parser is None:
            parser = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
        parser.add_argument("--checkpoint", type=str, default=None, help="checkpoint file (random init if omitted)")
        parser.add_argument("--world_idx", type=int, default=0)
        parser.add_argument("--world_idx_list", type=int, nargs="*", default=None)
        parser.add_argument("--world_random_scale", nargs="+", type=float, default=None)
        parser.add_argument("--skip", type=int, default=None)
        parser.add_argument("--skip_draw", type=int, default=None)
        parser.add_argument("--seed", type=int, default=0)
        parser.add_argument("--no_render", action="store_true")
        parser.add_argument("--no_plot", action="store_true")
        parser.add_argument("--win_xy_plot", type=int, nargs=2)
        parser.add_argument("--wait_before_start", action="store_true")
        parser.add_argument("--auto_exit", action="store_true")
        parser.add_argument("--max_duration", type=float, default=30.0)
        parser.add_argument("--result_filename", type=str, default=None)
        parser.add_argument("--save_last_image", action="store_true")
        parser.add_argument("--output_image_dir", type=str, default=".")
        # batching (this engine)
        parser.add_argument("--num_envs", type=int, default=None,
                            help="environments stepped in lockstep (default: one per --world_idx_list entry, "
                                 "the episodes the reference runs one after another)")
        parser.add_argument("--device", type=str, default="cuda:0")
        parser.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                            help="policy arithmetic: fp32 (the reference's precision, the default) or bf16 "
                                 "(opt-in throughput mode, ~1e-3 action error)")
        parser.add_argument("--max_steps", type=int, default=None, help="hard cap on env-steps")
        parser.add_argument("--num_gpus", type=int, default=1,
                            help="shard the envs over this many GPUs of the node (bin/Rollout.py launches one "
                                 "process per GPU; results all-gathered over RCCL)")
        parser.add_argument("--tactile", action="store_true",
                            help="scenes with tactile pads: info['intensity_tactile'] every env-step")
        parser.add_argument("--state_keys", type=str, nargs="*", default=None,
                            help="synthetic runs (no --checkpoint) only: state keys of the synthetic model meta "
                                 "info (TrainBase --state_keys; default measured_joint_pos)")
        parser.add_argument("--action_keys", type=str, nargs="+", default=None,
                            help="synthetic runs (no --checkpoint) only: action keys of the synthetic model meta "
                                 "info (TrainBase --action_keys; default command_joint_pos)")
        parser.add_argument("--env_offset", type=int, default=0,
                            help="global index of local env 0 (this rank's shard start under --num_gpus): world "
                                 "indices and noise streams follow the global env index")
        if self.require_task_desc:
            parser.add_argument("--task_desc", type=str, required=True)
        self.set_additional_args(parser)
        if argv is None:
            argv = sys.argv[1:]
        self.args = parser.parse_args(argv)
        if self.args.world_idx_list is None:
            self.args.world_idx_list = [self.args.world_idx]
        if self.args.num_envs is None:
            self.args.num_envs = len(self.args.world_idx_list)
        if self.args.world_random_scale is not None:
            self.args.world_random_scale = np.array(self.args.world_random_scale)
        self.args.auto_exit = True  # headless batched evaluation always auto-exits

    def set_additional_args(self, parser):
        pass

    def setup_model_meta_info(self):
        self.model_meta_info = make_meta_info(self)
        self.state_keys = self.model_meta_info["state"]["keys"]
        self.action_keys = self.model_meta_info["action"]["keys"]
        self.camera_names = self.model_meta_info["image"]["camera_names"]
        self.state_dim = len(self.model_meta_info["state"]["example"])
        self.action_dim = len(self.model_meta_info["action"]["example"])
        # device routing codes; unsupported keys raise ValueError as MotionManager does
        self._state_codes = state_key_codes(self.state_keys)
        self._action_codes = action_key_codes(self.action_keys)
        for what, keys, dim in (("state", self.state_keys, self.state_dim), ("action", self.action_keys, self.action_dim)):
            kd = sum(DataKey.get_dim(k, self.env) for k in keys)
            if kd != dim:
                raise ValueError(f"{what} keys {keys} have dimension {kd}, the model meta info {dim}")
        if self.args.skip is None:
            self.args.skip = self.model_meta_info["data"]["skip"]
        if self.args.skip_draw is None:
            self.args.skip_draw = self.args.skip

    def setup_env(self):
        raise NotImplementedError("defined by the Operation mixin")

    def setup_policy(self):
        raise NotImplementedError

    def get_pre_motion_phases(self):
        return []

    def reset_variables(self):
        pass

    def infer_policy(self):
        raise NotImplementedError

    def draw_plot(self):
        pass

    # -- state / images (RolloutBase.get_state :463-477, get_images :479-490) -----------------
    def _bind_state_stats(self):
        """The state normalisation statistics as f64 device tensors (read once per episode)."""
        st, dev = self.model_meta_info["state"], self.device
        if "mean" in st:
            self._st_mean = torch.tensor(st["mean"], dtype=torch.float64, device=dev)
            self._st_std = torch.tensor(st["std"], dtype=torch.float64, device=dev)
        if "min" in st:
            self._st_min = torch.tensor(st["min"], dtype=torch.float64, device=dev)
            self._st_range = torch.tensor(st["range"], dtype=torch.float64, device=dev)

    def get_raw_state(self):
        """RolloutBase.get_state's key concatenation (:463-473): MotionManager.get_data of every
        state key in order, f64 [n, state_dim], on the device (rmbx_motion_state)."""
        if not self.state_keys:
            return torch.zeros((self.n, 0), dtype=torch.float64, device=self.device)
        return K.motion_state(self._placement, self.obs, self.q_cmd, self.grip_cmd, self._tgt_R, self._tgt_p,
                              self._state_codes, self.state_dim)

    def get_state(self):
        """RolloutBase.get_state (:463-477): the routed state, normalised, as f32 [n, state_dim]."""
        return self.normalize_state(self.get_raw_state())

    def normalize_state(self, x):
        """normalize_data (DataUtils.py:9-24) in f64 (same operations and order as numpy), then the
        f32 cast of RolloutBase.get_state (:475)."""
        if x.shape[-1] == 0:
            return x.to(torch.float32)
        st = self.model_meta_info["state"]
        if st.get("norm_config", {}).get("type", "gaussian") == "gaussian":
            return ((x - self._st_mean) / self._st_std).to(torch.float32)
        scale = (st["norm_config"]["out_max"] - st["norm_config"]["out_min"]) / self._st_range
        return (scale * (x - self._st_min) + st["norm_config"]["out_min"]).to(torch.float32)

    # per-channel (mean, std) the renderer applies to [0, 1] pixels for the policy tensor:
    # identity = RolloutBase.image_transforms (v2.ToDtype(float32, scale=True), :353); the ACT
    # policy overrides it with its ImageNet normalisation
    image_norm = ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0))

    def get_images(self, dtype):
        """RolloutBase.get_images (:479-490): stack info["rgb_images"][camera] of every policy
        camera -> CHW -> ToDtype(scale) (and the policy's image normalisation).  Fused: every
        policy camera of the current state is rendered straight into the normalised policy tensor
        [n,ncam,3,H,W] (or, for a device policy that accepts it, the bf16 / f32 / 8-bit
        space-to-depth form [n,ncam,H/2,W/2,16] its fused stem kernel reads) -- the same values as
        normalising info["rgb_images"] (tests/test_env_info_gpu.py), without the u8 frame round
        trip through HBM."""
        H, W = self.env.renderer.height, self.env.renderer.width
        mean, std = self.image_norm
        # (the fused f32 stem kernel takes space-to-depth rows of at most STEM_POOL_MAX_WS: wider
        # f32 images go through the NCHW path)
        s2d = (dtype in (torch.bfloat16, torch.float32) and self.device.type == "cuda"
               and getattr(self.policy, "accepts_s2d", False) and H % 2 == 0 and W % 2 == 0
               and (dtype == torch.bfloat16 or W // 2 <= K.STEM_POOL_MAX_WS))
        shape = (H // 2, W // 2, 16) if s2d else (3, H, W)
        if s2d and dtype == torch.float32 and getattr(self.policy, "accepts_u8_s2d", False):
            # the f32 policy folds mean / std into its stem: the renderer hands over the 8-bit values
            dtype = torch.uint8
        if getattr(self, "_img", None) is None or self._img.dtype != dtype or tuple(self._img.shape[2:]) != shape:
            self._img = torch.empty((self.n, len(self.camera_names)) + shape, dtype=dtype, device=self.device)
            self._img_cam = [torch.empty((self.n,) + shape, dtype=dtype, device=self.device) for _ in self.camera_names]
        self._mark("render")
        if len(self.camera_names) == 1:
            self.env.render_images(self.camera_names[0], policy=self._img.view((self.n,) + shape), mean=mean, std=std)
        else:
            for i, cam in enumerate(self.camera_names):
                self.env.render_images(cam, policy=self._img_cam[i], mean=mean, std=std)
                self._img[:, i].copy_(self._img_cam[i])
        self._mark("policy")
        return self._img

    # -- command routing (MotionManager / ArmManager) ------------------------------------------
    def _reset_motion(self):
        """ArmManager.reset (:75-86): arm / gripper command = the initial pose, IK target = its FK."""
        env, dev = self.env, self.device
        self.q_cmd = torch.tensor(np.tile(env.init_qpos[:6], (self.n, 1)), dtype=torch.float64, device=dev)
        self.grip_cmd = torch.zeros((self.n, 1), dtype=torch.float64, device=dev)
        self._placement = torch.tensor(env.arrays["arm_placement"], dtype=torch.float64, device=dev).contiguous()
        self._glo, self._ghi = float(env.action_low[6]), float(env.action_high[6])
        self._tgt_R = torch.empty((self.n, 9), dtype=torch.float64, device=dev)
        self._tgt_p = torch.empty((self.n, 3), dtype=torch.float64, device=dev)
        from .. import _native as N

        N.call("rmbx_arm_fk", N.ptr(self._placement), N.ptr(self.q_cmd), N.ptr(self._tgt_R), N.ptr(self._tgt_p),
               self.n, N.stream_ptr())

    def set_command_data(self):
        """RolloutBase.set_command_data (:496-509): the policy action routed key by key through
        MotionManager / ArmManager (joint / relative joint / gripper / eef pose / relative eef
        pose commands, rmbx_motion_command), with is_skip = rollout_time_idx % skip != 0."""
        is_skip = self.rollout_time_idx % self.args.skip != 0
        K.motion_command(self._placement, self.policy_action, self._action_codes, is_skip, self._glo, self._ghi,
                         self.q_cmd, self.grip_cmd, self._tgt_R, self._tgt_p)

    def env_action(self):
        return torch.cat([self.q_cmd, self.grip_cmd], dim=1)

    def _set_reach_target(self, pos_z):
        """OperationMujocoUR5eCable.get_target_se3 (:8-11): cable_end xy, fixed z, R=diag(-1,1,-1)."""
        end = self.env.get_body_pose("cable_end")[:, :3].clone()
        end[:, 2] = pos_z
        self._tgt_p.copy_(end)
        R = torch.tensor([-1.0, 0, 0, 0, 1.0, 0, 0, 0, -1.0], dtype=torch.float64, device=self.device)
        self._tgt_R.copy_(R.expand(self.n, 9))

    def _ik_step(self):
        from .. import _native as N

        N.call("rmbx_arm_ik", N.ptr(self._placement), N.ptr(self.q_cmd), N.ptr(self._tgt_R), N.ptr(self._tgt_p),
               None, self.n, 1, N.stream_ptr())

    # -- episode --------------------------------------------------------------------------------
    def reset(self):
        self._reset_motion()
        g0, wl = self.args.env_offset, self.args.world_idx_list
        world = np.array([wl[(g0 + e) % len(wl)] for e in range(self.n)])
        self.env.world_random_scale = self.args.world_random_scale
        self.world_idx = self.env.modify_world(world_idx=world)
        self.obs, self.info = self.env.reset(seed=self.args.seed)
        self._bind_state_stats()
        dev = self.device
        self.sched = K.sched_alloc(self.n, dev)
        K.sched_reset(self.sched, self.env.get_time())
        # device-side step mask: an env stops stepping at its RolloutPhase -> EndRolloutPhase
        # transition (rmbx_sched_active), freezing the state its results were recorded from
        self._step_mask = torch.ones(self.n, dtype=torch.uint8, device=dev)
        self._pre = torch.tensor(self.pre_durations, dtype=torch.float64, device=dev)
        # host mirror of the (env-independent) pre-rollout clock
        self.phase_idx = 0
        self.host_time = 0.0
        self.phase_start = 0.0
        self.rollout_time_idx = 0
        self.policy_action = torch.zeros((self.n, self.action_dim), dtype=torch.float64, device=dev)
        self.reset_variables()

    def _pre_update(self):
        n_pre = len(self.pre_durations)
        if self.phase_idx == 0:
            return
        if self.phase_idx < n_pre:
            ph = self.pre_phases[self.phase_idx - 1]
            if ph.kind == "reach":
                self._ik_step()
            elif ph.kind == "grasp":
                # GraspPhaseBase.pre_update (:66-69): set_target_close / set_target_open
                # (action_space high / low, :78-104) or a fixed value
                g = self._ghi if ph.grip is None else (self._glo if ph.grip == "low" else float(ph.grip))
                self.grip_cmd.fill_(g)
        elif self.phase_idx == n_pre:
            if self.rollout_time_idx % self.args.skip == 0:
                self._timed_infer()
            self.set_command_data()

    def _timed_infer(self):
        """infer_policy timed like the reference's figure (RolloutAct.py:74-76 includes the .cpu()
        sync): device events around the call on the current stream, read in finish() so the
        loop never waits on the device; wall clock on a CPU device."""
        if self.device.type == "cuda":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            self._mark("policy")
            e0.record()
            self.infer_policy()
            e1.record()
            self._mark("glue")
            self._infer_events.append((e0, e1))
        else:
            t0 = time.time()
            self.infer_policy()
            self.inference_duration_list.append(time.time() - t0)

    def _collect_inference_durations(self):
        if self._infer_events:
            self._infer_events[-1][1].synchronize()
            self.inference_duration_list.extend(a.elapsed_time(b) / 1e3 for a, b in self._infer_events)
            self._infer_events = []

    def _host_transition(self):
        """Host mirror of the pre-rollout phase clock (PhaseBase.get_elapsed_duration)."""
        n_pre = len(self.pre_durations)
        if self.phase_idx < n_pre:
            if self.host_time - self.phase_start > self.pre_durations[self.phase_idx]:
                self.phase_idx += 1
                self.phase_start = self.host_time
                if self.phase_idx < n_pre:
                    ph = self.pre_phases[self.phase_idx - 1]
                    if ph.kind == "reach":
                        if ph.target is not None:
                            R, p = ph.target(self)
                            self._tgt_R.copy_(R)
                            self._tgt_p.copy_(p)
                        else:
                            self._set_reach_target(ph.pos_z)
                else:
                    self.rollout_time_idx = 0
        elif self.phase_idx == n_pre:
            self.rollout_time_idx += 1

    def step_once(self):
        self._mark("glue")
        self._pre_update()
        active = self._active if self._active is not None else self._step_mask
        self.obs, self.reward, _, _, self.info = self.env.step(self.env_action(), active=active)
        for _ in range(self.env.frame_skip):
            self.host_time += self.env.sim_timestep
        K.sched_update(self.sched, self.env.get_time(), self.reward, self._pre, self.args.max_duration)
        K.sched_active(self.sched, len(self.pre_durations), out=self._step_mask)
        self._host_transition()

    def run(self, max_steps=None):
        self.reset()
        max_steps = max_steps or self.args.max_steps or 10**9
        steps = 0
        while steps < max_steps:
            self.step_once()
            steps += 1
            # finished envs are frozen on the device (step mask); the host only polls for the end
            if self.phase_idx >= len(self.pre_durations) and steps % 16 == 0:
                if K.sched_view(self.sched)["done"].all():
                    break
        self.finish()
        return steps

    def _dist_world(self):
        """(rank, world) of the torch.distributed group this rollout is a shard of (bin/Rollout.py
        --num_gpus), else (0, 1)."""
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
        return 0, 1

    def finish(self):
        """RolloutPhase / EndRolloutPhase result bookkeeping (RolloutBase.py:96-110, 417-422) for
        every env.  Under --num_gpus the per-env records of all shards are all-gathered (one RCCL
        all_gather, distributed.py) and rank 0 prints and writes them in global env order."""
        v = K.sched_view(self.sched)
        succ, rew, dur = v["success"].astype(bool), v["result_reward"].astype(np.float64), v["duration"]
        rank, world = self._dist_world()
        if world > 1:
            import torch.distributed as dist

            from ..distributed import gather_results, pack_results

            dev = self.device if dist.get_backend() == "nccl" else "cpu"
            g = gather_results(pack_results(succ, rew, dur, v["rollout_time_idx"]), dev)
            succ, rew, dur = g[:, 0] != 0, g[:, 1], g[:, 2]
        if rank == 0:
            for e in range(len(succ)):
                print(f"Rollout result: {'success' if succ[e] else 'failure'}", flush=True)
                self.result["success"].append(bool(succ[e]))
                self.result["reward"].append(float(rew[e]))
                self.result["duration"].append(float(dur[e]))
        if self.args.save_last_image:
            self.save_rgb_images(v)
        if rank == 0 and self.args.result_filename is not None:
            print(f"[{self.__class__.__name__}] Save the rollout results: {self.args.result_filename}")
            with open(self.args.result_filename, "w") as f:
                yaml.dump(self.result, f)
        if rank == 0:
            self.print_statistics()

    def save_rgb_images(self, v=None):
        """RolloutBase.save_rgb_image (:541-561) for every env: the last frame of all cameras side
        by side (cv2.hconcat of info["rgb_images"]), named
        Rollout<Policy>_<Env>_world<idx>_<success|failure>_<datetime>.png in --output_image_dir.
        Each env is frozen at its episode's end, so its frame is the transition step's."""
        from .image_io import write_png

        if v is None:
            v = K.sched_view(self.sched)
        # cv2.hconcat(list(self.info["rgb_images"].values())): the envs are frozen at their last
        # step, whose info this is
        image = torch.cat([self.info["rgb_images"][cam] for cam in self.env.camera_names], dim=2).cpu().numpy()
        demo_name = self.env.demo_name
        os.makedirs(self.args.output_image_dir, exist_ok=True)
        for e in range(self.n):
            success_str = "success" if v["success"][e] else "failure"
            path = os.path.abspath(os.path.join(
                self.args.output_image_dir,
                f"Rollout{self.policy_name}_{demo_name}_world{int(self.world_idx[e]):0>1}_{success_str}_"
                f"{self.datetime_now:%Y%m%d_%H%M%S}_env{self.args.env_offset + e}.png"))
            print(f"[{self.__class__.__name__}] Save the observation image of the last frame: {path}")
            write_png(path, image[e])

    def print_statistics(self):
        self._collect_inference_durations()
        print(f"[{self.__class__.__name__}] Statistics on policy inference")
        if self.inference_duration_list:
            a = np.array(self.inference_duration_list)
            print(f"  - Inference duration [s] | mean: {a.mean():.2e}, std: {a.std():.2e} min: {a.min():.2e}, max: {a.max():.2e}")
            print(f"  - Inference duration per env [us] | mean: {1e6 * a.mean() / self.n:.2f}")
        if torch.cuda.is_available():
            print(f"  - GPU memory usage [GB] | {torch.cuda.max_memory_reserved() / 1024**3:.3f}")
