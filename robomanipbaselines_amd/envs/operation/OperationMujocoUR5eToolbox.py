"""Operation mixin for the toolbox task (envs/operation/OperationMujocoUR5eToolbox.py:1-18): env
construction and the scripted pre-rollout phase Grasp with the gripper opened
(GraspPhaseBase.set_target_open = action_space.low, PhaseBase.py:81-82), 0.5 s."""

from ...common.rollout_base import PhaseSpec
from ..ur5e_toolbox import BatchedMujocoUR5eToolboxEnv


class OperationMujocoUR5eToolbox:
    def setup_env(self, render_mode=None):
        self.env = BatchedMujocoUR5eToolboxEnv(
            self.args.num_envs, self.args.device, world_random_scale=self.args.world_random_scale, seed=self.args.seed,
            env_offset=self.args.env_offset,
        )

    def get_pre_motion_phases(self):
        return [PhaseSpec("GraspPhase", 0.5, "grasp", grip="low")]
