"""Operation mixin for the cabinet task (envs/operation/OperationMujocoUR5eCabinet.py:1-18): env
construction and the scripted pre-rollout phase Grasp with the gripper closed
(GraspPhaseBase.set_target_close = action_space.high, PhaseBase.py:78-79), 0.5 s."""

from ...common.rollout_base import PhaseSpec
from ..ur5e_cabinet import BatchedMujocoUR5eCabinetEnv


class OperationMujocoUR5eCabinet:
    def setup_env(self, render_mode=None):
        self.env = BatchedMujocoUR5eCabinetEnv(
            self.args.num_envs, self.args.device, world_random_scale=self.args.world_random_scale, seed=self.args.seed,
            env_offset=self.args.env_offset,
        )

    def get_pre_motion_phases(self):
        return [PhaseSpec("GraspPhase", 0.5, "grasp")]
