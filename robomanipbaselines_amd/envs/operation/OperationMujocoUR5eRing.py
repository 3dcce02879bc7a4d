"""Operation mixin for the ring task (envs/operation/OperationMujocoUR5eRing.py:1-64): env
construction and the scripted pre-rollout phases Reach1 (0.7 s) and Reach2 (0.3 s) towards the
midpoint of the two hooks plus an offset, with the hand orientation rpyToMatrix(pi/2, 0, pi/2),
then Grasp (close, 0.5 s)."""

import numpy as np
import torch

from ...common.rollout_base import PhaseSpec
from ..ur5e_ring import BatchedMujocoUR5eRingEnv


def _rpy_to_matrix(r, p, y):
    """pinocchio.rpy.rpyToMatrix: Rz(y) Ry(p) Rx(r)."""
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rz = np.array([[cy, -sy, 0.0], [sy, cy, 0.0], [0.0, 0.0, 1.0]])
    Ry = np.array([[cp, 0.0, sp], [0.0, 1.0, 0.0], [-sp, 0.0, cp]])
    Rx = np.array([[1.0, 0.0, 0.0], [0.0, cr, -sr], [0.0, sr, cr]])
    return Rz @ Ry @ Rx


HAND_R = _rpy_to_matrix(np.pi / 2, 0.0, np.pi / 2)


def hook_target(offset_pos):
    """get_target_se3 (:8-19): 0.5 (fook1 + fook2) + offset_pos, R = rpyToMatrix(pi/2, 0, pi/2)."""
    off = np.asarray(offset_pos, dtype=np.float64)

    def target(ro):
        env = ro.env
        p = 0.5 * (env.get_geom_pose("fook1")[:, :3] + env.get_geom_pose("fook2")[:, :3])
        p = p + torch.tensor(off, dtype=torch.float64, device=p.device)
        R = torch.tensor(HAND_R.reshape(9), dtype=torch.float64, device=p.device).expand(p.shape[0], 9)
        return R, p

    return target


class OperationMujocoUR5eRing:
    def setup_env(self, render_mode=None):
        self.env = BatchedMujocoUR5eRingEnv(
            self.args.num_envs, self.args.device, world_random_scale=self.args.world_random_scale, seed=self.args.seed,
            env_offset=self.args.env_offset,
        )

    def get_pre_motion_phases(self):
        return [
            PhaseSpec("ReachPhase1", 0.7, "reach", target=hook_target([-0.15, 0.05, -0.05])),
            PhaseSpec("ReachPhase2", 0.3, "reach", target=hook_target([-0.1, 0.05, -0.05])),
            PhaseSpec("GraspPhase", 0.5, "grasp"),
        ]
