"""Batched MujocoUR5eCabinet environment: envs/mujoco/ur5e/MujocoUR5eCabinetEnv.py of the reference on
the batched UR5e base (ur5e_base.py) — the cabinet's hinged lid and sliding drawer run on the same
physics, render and glue kernels as the cable task; reward = rmbx_cabinet_reward (binary)."""

import numpy as np

from .. import kernels as K
from .ur5e_base import BatchedMujocoUR5eEnvBase

# MujocoUR5eCabinetEnv.py:21-36 (init_qpos[:14])
CABINET_INIT_QPOS = np.array([np.pi, -0.4 * np.pi, -0.65 * np.pi, -0.2 * np.pi, np.pi / 2, np.pi / 2, *np.zeros(8)])
# MujocoUR5eCabinetEnv.py:39-49
CABINET_POS_OFFSETS = np.array(
    [[0.0, -0.06, 0.0], [0.0, -0.03, 0.0], [0.0, 0.0, 0.0], [0.0, 0.03, 0.0], [0.0, 0.06, 0.0], [0.0, 0.09, 0.0]]
)
# MujocoUR5eCabinetEnv.py:58-61: hinge past 120 deg, drawer past 0.12 m
CABINET_HINGE_THRE = float(np.deg2rad(120.0))
CABINET_SLIDE_THRE = 0.12


class BatchedMujocoUR5eCabinetEnv(BatchedMujocoUR5eEnvBase):
    model_name = "ur5e_cabinet"
    demo_name = "MujocoUR5eCabinet"
    init_qpos_head = CABINET_INIT_QPOS
    world_body = "cabinet"
    world_offsets = CABINET_POS_OFFSETS

    def _setup_task(self):
        self._hinge_qadr = self.info.qposadr("hinge")
        self._slide_qadr = self.info.qposadr("slide")
        self.original_cabinet_pos = self.original_world_pos
        self.target_task = None  # One of [None, "hinge", "slide"] (MujocoUR5eCabinetEnv.py:51)

    def _get_reward(self):
        """MujocoUR5eCabinetEnv._get_reward (:57-73)."""
        return K.cabinet_reward(self.engine.qpos, self._hinge_qadr, self._slide_qadr, CABINET_HINGE_THRE,
                                CABINET_SLIDE_THRE, self.target_task,
                                out=self.reward if self.reward.is_contiguous() else None)
