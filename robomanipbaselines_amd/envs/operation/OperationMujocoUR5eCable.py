"""Operation mixin for the cable task (envs/operation/OperationMujocoUR5eCable.py:8-47):
env construction and the scripted pre-rollout phases Reach1 (z = 1.02 m, 0.7 s),
Reach2 (z = 0.995 m, 0.3 s) and Grasp (close, 0.5 s)."""

from ...common.rollout_base import PhaseSpec
from ..ur5e_cable import BatchedMujocoUR5eCableEnv


class OperationMujocoUR5eCable:
    def setup_env(self, render_mode=None):
        self.env = BatchedMujocoUR5eCableEnv(
            self.args.num_envs, self.args.device, world_random_scale=self.args.world_random_scale, seed=self.args.seed,
            env_offset=self.args.env_offset,
        )

    def get_pre_motion_phases(self):
        return [
            PhaseSpec("ReachPhase1", 0.7, "reach", pos_z=1.02),
            PhaseSpec("ReachPhase2", 0.3, "reach", pos_z=0.995),
            PhaseSpec("GraspPhase", 0.5, "grasp"),
        ]
