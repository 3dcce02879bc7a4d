"""Batched MujocoUR5eToolbox environment: envs/mujoco/ur5e/MujocoUR5eToolboxEnv.py of the reference on
the batched UR5e base (ur5e_base.py) — a free-floating toolbox carried onto a mat, on the same
physics, render and glue kernels as the cable task; reward = rmbx_toolbox_reward (binary)."""

import numpy as np

from .. import kernels as K
from .ur5e_base import BatchedMujocoUR5eEnvBase

# MujocoUR5eToolboxEnv.py:19-31 (init_qpos[:14])
TOOLBOX_INIT_QPOS = np.array([np.pi, -np.pi / 2, -0.55 * np.pi, -0.45 * np.pi, np.pi / 2, np.pi, *np.zeros(8)])
# MujocoUR5eToolboxEnv.py:34-44
TOOLBOX_POS_OFFSETS = np.array(
    [[0.0, -0.06, 0.0], [0.0, -0.03, 0.0], [0.0, 0.0, 0.0], [0.0, 0.03, 0.0], [0.0, 0.06, 0.0], [0.0, 0.09, 0.0]]
)
# MujocoUR5eToolboxEnv.py:50-51: within 3 cm of the mat in x/y, below the mat height + 5 mm
TOOLBOX_XY_THRE = 0.03
TOOLBOX_Z_OFFSET = 0.005


class BatchedMujocoUR5eToolboxEnv(BatchedMujocoUR5eEnvBase):
    model_name = "ur5e_toolbox"
    demo_name = "MujocoUR5eToolbox"
    init_qpos_head = TOOLBOX_INIT_QPOS
    world_body = "toolbox"
    world_offsets = TOOLBOX_POS_OFFSETS

    def _setup_task(self):
        self._toolbox = self.info.body["toolbox"]
        self._mat = self.info.body["mat"]
        self._free_qadr = self.info.qposadr("toolbox_freejoint")
        self.original_toolbox_pos = self.original_world_pos

    def modify_world(self, world_idx=None, cumulative_idx=None):
        """MujocoUR5eToolboxEnv.modify_world (:59-75): the toolbox is a free body, so the world's
        offset (+ noise) goes into the free joint's initial position, per env."""
        world_idx, pos = self._world_positions(world_idx, cumulative_idx)
        q = np.repeat(self.init_qpos[None], self.num_envs, axis=0)
        q[:, self._free_qadr: self._free_qadr + 3] = pos
        self.init_qpos_env = q
        self.world_idx = world_idx
        return world_idx

    def _get_reward(self):
        """MujocoUR5eToolboxEnv._get_reward (:46-57)."""
        e = self.engine
        box = e.xpos[:, self._toolbox].contiguous()
        mat = e.xpos[:, self._mat].contiguous()
        return K.toolbox_reward(box, mat, TOOLBOX_XY_THRE, TOOLBOX_Z_OFFSET,
                                out=self.reward if self.reward.is_contiguous() else None)
