"""Batched MujocoUR5eCable environment: envs/mujoco/ur5e/MujocoUR5eCableEnv.py of the reference
on the batched UR5e base (ur5e_base.py); success predicate = rmbx_cable_reward."""

import numpy as np

from .. import kernels as K
from .ur5e_base import ARM_JOINTS, GRIPPER_JOINTS, BatchedMujocoUR5eEnvBase  # noqa: F401

# MujocoUR5eCableEnv.py:20-30 (init_qpos[:14])
CABLE_INIT_QPOS = np.array([np.pi, -np.pi / 2, -0.75 * np.pi, -0.25 * np.pi, np.pi / 2, np.pi / 2, *np.zeros(8)])
# MujocoUR5eCableEnv.py:35-44
POLE_POS_OFFSETS = np.array(
    [[-0.03, 0.0, 0.0], [0.0, 0.0, 0.0], [0.03, 0.0, 0.0], [0.06, 0.0, 0.0], [0.09, 0.0, 0.0], [0.12, 0.0, 0.0]]
)


class BatchedMujocoUR5eCableEnv(BatchedMujocoUR5eEnvBase):
    model_name = "ur5e_cable"
    demo_name = "MujocoUR5eCable"
    init_qpos_head = CABLE_INIT_QPOS
    world_body = "poles"
    world_offsets = POLE_POS_OFFSETS

    def _setup_task(self):
        names, inf = self._names_body, self.info
        self._cable_bodies = [i for i, n in enumerate(names) if n.startswith("cable_B")]
        assert self._cable_bodies == list(range(self._cable_bodies[0], self._cable_bodies[0] + len(self._cable_bodies)))
        self._cable_end = names.index("cable_end")
        self._pole_geoms = [inf.geom["pole1"], inf.geom["pole2"]]
        self.original_pole_pos = self.original_world_pos

    def _get_reward(self):
        """MujocoUR5eCableEnv._get_reward (:48-105)."""
        e = self.engine
        c0, c1 = self._cable_bodies[0], self._cable_bodies[-1] + 1
        cable = e.xpos[:, c0:c1].contiguous()
        end = e.xpos[:, self._cable_end].contiguous()
        p1 = e.gxpos[:, self._pole_geoms[0]].contiguous()
        p2 = e.gxpos[:, self._pole_geoms[1]].contiguous()
        return K.cable_reward(cable, end, p1, p2, out=self.reward if self.reward.is_contiguous() else None)
