"""Batched MujocoUR5eInsert environment: envs/mujoco/ur5e/MujocoUR5eInsertEnv.py of the reference
on the batched UR5e base (ur5e_base.py) — the peg-in-hole scene runs on the same physics, render
and glue kernels as the cable task; success predicate = rmbx_insert_reward."""

import numpy as np

from .. import kernels as K
from .ur5e_base import BatchedMujocoUR5eEnvBase

# MujocoUR5eInsertEnv.py:15-29 (init_qpos[:14])
INSERT_INIT_QPOS = np.array([np.pi, -np.pi / 2, -0.55 * np.pi, -0.45 * np.pi, np.pi / 2, np.pi / 2, *np.zeros(8)])
# MujocoUR5eInsertEnv.py:32-41
HOLE_POS_OFFSETS = np.array(
    [[0.0, -0.06, 0.0], [0.0, -0.03, 0.0], [0.0, 0.0, 0.0], [0.0, 0.03, 0.0], [0.0, 0.06, 0.0], [0.0, 0.09, 0.0]]
)
# MujocoUR5eInsertEnv.py:49-51: xy_thre 0.012 m, z_thre = hole z + 0.05 m, tilt_thre 10 deg
INSERT_XY_THRE = 0.012
INSERT_Z_OFFSET = 0.05
INSERT_COS_TILT = float(np.cos(np.deg2rad(10)))


class BatchedMujocoUR5eInsertEnv(BatchedMujocoUR5eEnvBase):
    model_name = "ur5e_insert"
    demo_name = "MujocoUR5eInsert"
    init_qpos_head = INSERT_INIT_QPOS
    world_body = "hole"
    world_offsets = HOLE_POS_OFFSETS

    def _setup_task(self):
        self._peg = self._names_body.index("peg")
        self._hole = self._world_body
        self.original_hole_pos = self.original_world_pos

    def _get_reward(self):
        """MujocoUR5eInsertEnv._get_reward (:43-63)."""
        e = self.engine
        peg = e.xpos[:, self._peg].contiguous()
        hole = e.xpos[:, self._hole].contiguous()
        quat = e.xquat[:, self._peg].contiguous()
        return K.insert_reward(peg, hole, quat, INSERT_XY_THRE, INSERT_Z_OFFSET, INSERT_COS_TILT,
                               out=self.reward if self.reward.is_contiguous() else None)
