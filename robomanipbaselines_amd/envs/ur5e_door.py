"""Batched MujocoUR5eDoor environment: envs/mujoco/ur5e/MujocoUR5eDoorEnv.py of the reference on the
batched UR5e base (ur5e_base.py) — the hinged door runs on the same physics, render and glue kernels
as the cable task; reward = rmbx_door_reward (continuous, success iff it reaches 1.0)."""

import numpy as np

from .. import kernels as K
from .ur5e_base import BatchedMujocoUR5eEnvBase

# MujocoUR5eDoorEnv.py:21-36 (init_qpos[:14])
DOOR_INIT_QPOS = np.array([np.pi, -0.4 * np.pi, -0.65 * np.pi, -0.25 * np.pi, np.pi / 2, np.pi / 2, *np.zeros(8)])
# MujocoUR5eDoorEnv.py:39-49
DOOR_POS_OFFSETS = np.array(
    [[0.0, -0.06, 0.0], [0.0, -0.03, 0.0], [0.0, 0.0, 0.0], [0.0, 0.03, 0.0], [0.0, 0.06, 0.0], [0.0, 0.09, 0.0]]
)
# MujocoUR5eDoorEnv.py:56, 62: reaching margin 0.08 m, opening target -45 deg
DOOR_HANDLE_MARGIN = 0.08
DOOR_TARGET_ANGLE = float(np.deg2rad(-45.0))


class BatchedMujocoUR5eDoorEnv(BatchedMujocoUR5eEnvBase):
    model_name = "ur5e_door"
    demo_name = "MujocoUR5eDoor"
    init_qpos_head = DOOR_INIT_QPOS
    world_body = "door"
    world_offsets = DOOR_POS_OFFSETS

    def _setup_task(self):
        sites = [str(x) for x in self.arrays["names_site"]]
        self._pinch = sites.index("pinch")
        self._handle = self.info.geom["door_handle"]
        self._door_qadr = self.info.qposadr("door")
        self.original_door_pos = self.original_world_pos

    def _get_reward(self):
        """MujocoUR5eDoorEnv._get_reward (:52-67)."""
        e = self.engine
        pinch = e.ws("sxpos")[:, 3 * self._pinch: 3 * self._pinch + 3].contiguous()
        handle = e.gxpos[:, self._handle].contiguous()
        angle = e.qpos[:, self._door_qadr].contiguous()
        return K.door_reward(pinch, handle, angle, DOOR_HANDLE_MARGIN, DOOR_TARGET_ANGLE,
                             out=self.reward if self.reward.is_contiguous() else None)
