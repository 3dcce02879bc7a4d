"""Operation mixin for the pick task (envs/operation/OperationMujocoUR5ePick.py): env
construction and the one scripted pre-rollout phase, Grasp with the gripper opened
(set_target_open, 0.5 s)."""

from ...common.rollout_base import PhaseSpec
from ..ur5e_pick import BatchedMujocoUR5ePickEnv


class OperationMujocoUR5ePick:
    def setup_env(self, render_mode=None):
        self.env = BatchedMujocoUR5ePickEnv(
            self.args.num_envs, self.args.device, world_random_scale=self.args.world_random_scale, seed=self.args.seed,
            env_offset=self.args.env_offset, tactile=getattr(self.args, "tactile", False),
        )

    def get_pre_motion_phases(self):
        return [PhaseSpec("GraspPhase", 0.5, "grasp", grip="low")]
