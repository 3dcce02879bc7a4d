"""Batched MujocoUR5eRing environment: envs/mujoco/ur5e/MujocoUR5eRingEnv.py of the reference on
the batched UR5e base (ur5e_base.py).

Scene: env_ur5e_ring.xml compiled with convex_meshes (gripper meshes through their convex hulls,
the hooks and the pole as true cylinders) and its `<composite type="loop">` ring expanded by the
MJCF compiler (mjcf/compiler.py `_expand_composites`: 11 capsule elements on a closed polygon,
two hinges per joint vertex, a connect equality closing the loop).  modify_world moves the pole
by one of six y offsets plus U(-s, s)^3 noise (:78-90); success = rmbx_ring_reward (:46-75)."""

import numpy as np

from .. import kernels as K
from .ur5e_base import BatchedMujocoUR5eEnvBase

# MujocoUR5eRingEnv.py:19-30 (init_qpos[:14])
RING_INIT_QPOS = np.array([np.pi, -np.pi / 2, -0.75 * np.pi, -0.75 * np.pi, -0.5 * np.pi, 0.0, *np.zeros(8)])
# MujocoUR5eRingEnv.py:34-43
POLE_POS_OFFSETS = np.array(
    [[0.0, 0.0, 0.0], [0.0, 0.04, 0.0], [0.0, 0.08, 0.0], [0.0, 0.12, 0.0], [0.0, 0.16, 0.0], [0.0, 0.20, 0.0]]
)


class BatchedMujocoUR5eRingEnv(BatchedMujocoUR5eEnvBase):
    model_name = "ur5e_ring"
    demo_name = "MujocoUR5eRing"
    init_qpos_head = RING_INIT_QPOS
    world_body = "pole"
    world_offsets = POLE_POS_OFFSETS

    def _setup_task(self):
        names = self._names_body
        # ring_body_ids: bodies named ring_B* in body-id order (:48-55)
        self._ring_bodies = [i for i, n in enumerate(names) if n.startswith("ring_B")]
        assert self._ring_bodies == list(range(self._ring_bodies[0], self._ring_bodies[0] + len(self._ring_bodies)))
        self._pole = names.index("pole")
        self.original_pole_pos = self.original_world_pos

    def _get_reward(self):
        """MujocoUR5eRingEnv._get_reward (:46-75)."""
        e = self.engine
        r0, r1 = self._ring_bodies[0], self._ring_bodies[-1] + 1
        ring = e.xpos[:, r0:r1].contiguous()
        pole = e.xpos[:, self._pole].contiguous()
        return K.ring_reward(ring, pole, out=self.reward if self.reward.is_contiguous() else None)
