"""Operation mixin for the peg-in-hole task (envs/operation/OperationMujocoUR5eInsert.py:1-22):
env construction and the scripted pre-rollout phase Grasp (gripper command 170, 0.5 s); the
peg is welded to the gripper base by the scene's equality, so no reach phase precedes it."""

from ...common.rollout_base import PhaseSpec
from ..ur5e_insert import BatchedMujocoUR5eInsertEnv


class OperationMujocoUR5eInsert:
    def setup_env(self, render_mode=None):
        self.env = BatchedMujocoUR5eInsertEnv(
            self.args.num_envs, self.args.device, world_random_scale=self.args.world_random_scale, seed=self.args.seed,
            env_offset=self.args.env_offset,
        )

    def get_pre_motion_phases(self):
        return [PhaseSpec("GraspPhase", 0.5, "grasp", grip=170.0)]
