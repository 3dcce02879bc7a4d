"""Batched MujocoUR5ePick environment: envs/mujoco/ur5e/MujocoUR5ePickEnv.py of the reference
(BASELINE configs 4 and 5) on the batched UR5e base (ur5e_base.py).

The compiled scene is env_ur5e_pick.xml minus its YCB_sim objects (the third_party/YCB_sim
submodule is absent from the checkout: the cracker box, pudding box and potted-meat can and their
free bodies are dropped -- documented substitution), with the six mujoco_scanned_objects free
bodies plus the basket and the bin colliding through the convex hulls of their 32 collision
meshes each (MPR narrow phase, as MuJoCo's mjc_Convex), dt 0.002 x frame_skip 16
(MujocoUR5ePickEnv.py:8-18).  modify_world keeps world 0 (:55-71, the offsets are commented
out) and the reward is MujocoEnvBase's 0.0 (the reference defines none).

Tactile (BASELINE config 5): the reference's MujocoTactileSensorPlugin is an external C++
plugin, commented out of the MJCF (env_ur5e_pick.xml:8-9, ur5e_tactile_sensor_config.xml: two
5 x 8 grids, 4 mm pitch, on the left/right_tactile_sensor sites) and absent here; `tactile()`
is a SYNTHETIC stand-in of the same shape, info["intensity_tactile"]-like (MujocoEnvBase.py:
128-153): per taxel, the penetration depth (mm) of every contact on the pad's body, weighted by
a Gaussian of the in-plane distance to the taxel (sigma = the pitch)."""

import numpy as np
import torch

from .ur5e_base import BatchedMujocoUR5eEnvBase

# MujocoUR5ePickEnv.py:24-37 (init_qpos[:14])
PICK_INIT_QPOS = np.array([np.pi, -np.pi / 2, -0.55 * np.pi, -0.45 * np.pi, np.pi / 2, np.pi, *np.zeros(8)])
# ur5e_tactile_sensor_config.xml: sensor_nums "5 8", sensor_interval 0.004
TACTILE_SHAPE = (5, 8)
TACTILE_INTERVAL = 0.004
TACTILE_SITES = ("left_tactile_sensor", "right_tactile_sensor")


def _quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class BatchedMujocoUR5ePickEnv(BatchedMujocoUR5eEnvBase):
    sim_timestep = 0.002  # MujocoUR5ePickEnv.py:9
    frame_skip = 16  # MujocoUR5ePickEnv.py:10
    model_name = "ur5e_pick"
    demo_name = "MujocoUR5ePick"
    init_qpos_head = PICK_INIT_QPOS
    world_body = "table"  # unused: modify_world keeps world 0
    world_offsets = np.zeros((1, 3))
    intensity_tactile_names = TACTILE_SITES

    def __init__(self, *args, tactile=False, **kw):
        # tactile=True: step() returns info["intensity_tactile"] every env-step, as
        # MujocoEnvBase._get_info does when the scene declares tactile sensors (:128-153)
        self.tactile_enabled = bool(tactile)
        super().__init__(*args, **kw)

    def _get_info(self):
        info = super()._get_info()
        if self.tactile_enabled:
            tac = self.tactile()
            info["intensity_tactile"] = {name: tac[:, s] for s, name in enumerate(TACTILE_SITES)}
        return info

    def _setup_task(self):
        a = self.arrays
        sites = [str(x) for x in a["names_site"]]
        self._tac_site = [sites.index(s) for s in TACTILE_SITES]
        self._tac_body = torch.tensor([int(a["site_body"][i]) for i in self._tac_site], device=self.device)
        rows, cols = TACTILE_SHAPE
        gy, gx = np.meshgrid((np.arange(rows) - (rows - 1) / 2) * TACTILE_INTERVAL,
                             (np.arange(cols) - (cols - 1) / 2) * TACTILE_INTERVAL, indexing="ij")
        self._tac_grid = torch.tensor(np.stack([gx, gy, np.zeros_like(gx)], -1), dtype=torch.float64,
                                      device=self.device)  # [rows, cols, 3] in the site frame
        self._tac_R = torch.tensor(np.stack([_quat2mat(a["site_quat"][i]) for i in self._tac_site]),
                                   dtype=torch.float64, device=self.device)  # site in its body frame

    def modify_world(self, world_idx=None, cumulative_idx=None):
        """MujocoUR5ePickEnv.modify_world (:55-71): world 0, nothing moved."""
        self.world_idx = np.zeros(self.num_envs, dtype=np.int64)
        return self.world_idx

    def _get_reward(self):
        """MujocoEnvBase._get_reward (:160-161): 0.0."""
        return self.reward.zero_()

    def tactile(self):
        """Synthetic tactile intensities [n, 2 (left, right), 5, 8] f64 (see the module docstring)."""
        e = self.engine
        n = self.num_envs
        xmat = e.ws("xmat").view(n, -1, 3, 3)
        sxpos = e.ws("sxpos").view(n, -1, 3)[:, self._tac_site]  # [n, 2, 3]
        Rs = xmat[:, self._tac_body] @ self._tac_R  # [n, 2, 3, 3] site frames in world
        taxel = sxpos[:, :, None, None, :] + torch.einsum("nsij,rcj->nsrci", Rs, self._tac_grid)
        ncon = e.stats[:, 0].to(torch.int64)
        mc = e.ws("con_dist").shape[1]
        valid = torch.arange(mc, device=self.device)[None] < ncon[:, None]  # [n, mc]
        b1, b2 = e.wsi("con_b1"), e.wsi("con_b2")
        pen = (-e.ws("con_dist")).clamp(min=0.0) * 1000.0 * valid  # mm
        on_pad = (b1[:, None] == self._tac_body[None, :, None]) | (b2[:, None] == self._tac_body[None, :, None])
        w_con = pen[:, None] * on_pad  # [n, 2, mc]
        d = e.ws("con_pos").view(n, 1, 1, 1, mc, 3) - taxel[..., None, :]  # [n, 2, r, c, mc, 3]
        nrm = Rs[..., 2][:, :, None, None, None, :]
        d = d - (d * nrm).sum(-1, keepdim=True) * nrm
        w = torch.exp(-(d * d).sum(-1) / (2 * TACTILE_INTERVAL ** 2))
        return (w * w_con[:, :, None, None, :]).sum(-1)
