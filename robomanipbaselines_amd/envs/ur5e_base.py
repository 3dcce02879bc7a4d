"""Batched UR5e MuJoCo environment base (n_env instances in lockstep on one GPU).

Counterpart of envs/mujoco/ur5e/MujocoUR5eEnvBase.py + envs/mujoco/MujocoEnvBase.py of the
reference, with the gymnasium-style API and the Isaac-style vector attributes (num_envs,
rep_env_idx; envs/isaac/IsaacUR5eEnvBase.py:104-106, 379-431) the reference's only vectorised env
exposes.  Every per-step computation runs in HIP kernels behind the C ABI: physics
(rmbx_engine_step), observation mapping (rmbx_ur5e_obs), the task's success predicate and camera
rendering (rmbx_render).  Tensors stay resident on the device.  Task subclasses
(ur5e_cable.py, ur5e_insert.py, ur5e_door.py, ur5e_cabinet.py, ur5e_toolbox.py) name the
compiled scene, the initial arm/gripper pose, the body
that modify_world moves per world index, and the reward kernel.
"""

from collections.abc import Mapping

import numpy as np
import torch

from .. import _native as N  # noqa: F401  (fails loudly if librmbx.so is missing)
from .. import kernels as K
from .. import model as MD
from ..engine import PhysicsEngine
from ..render import Renderer

ARM_JOINTS = ["shoulder_pan_joint", "shoulder_lift_joint", "elbow_joint", "wrist_1_joint", "wrist_2_joint", "wrist_3_joint"]
GRIPPER_JOINTS = ["right_driver_joint", "right_spring_link_joint", "left_driver_joint", "left_spring_link_joint"]


class BatchedMujocoUR5eEnvBase:
    sim_timestep = 0.004  # MujocoEnvBase.py:12
    frame_skip = 8  # MujocoEnvBase.py:13
    command_keys_for_step = ["command_joint_pos"]  # EnvDataMixin.py:5-7
    # task definition (subclasses)
    model_name = None
    demo_name = None  # remove_suffix(env.spec.name, "Env") (RolloutBase.py:545)
    init_qpos_head = None  # the env's init_qpos[:14] (6 arm joints + 8 gripper joints)
    world_body = None  # body moved by modify_world
    world_offsets = None  # [n_world, 3] offsets of world_body per world index

    def __init__(self, num_envs, device="cuda:0", world_random_scale=None, seed=0, image_size=(480, 640),
                 model_name=None, env_offset=0):
        model_name = model_name or self.model_name
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.arrays = MD.load(model_name)
        self.info = MD.ModelInfo(self.arrays)
        self.engine = PhysicsEngine(self.arrays, self.num_envs, device)
        self.renderer = Renderer(self.arrays, device, width=image_size[1], height=image_size[0])
        self.world_random_scale = world_random_scale
        self.seed = int(seed)
        # global index of local env 0 (the rank's shard start): noise streams are keyed by the
        # GLOBAL env index so placements do not depend on the GPU count (distributed.py)
        self.env_offset = int(env_offset)
        self.rep_env_idx = 0
        inf = self.info
        self._arm_qadr = torch.tensor([inf.qposadr(j) for j in ARM_JOINTS], device=self.device)
        self._arm_dadr = torch.tensor([inf.dofadr(j) for j in ARM_JOINTS], device=self.device)
        self._grip_qadr = torch.tensor([inf.qposadr(j) for j in GRIPPER_JOINTS], device=self.device)
        names = [str(x) for x in self.arrays["names_body"]]
        self._names_body = names
        self._world_body = names.index(self.world_body)
        self.original_world_pos = self.arrays["body_pos"][self._world_body].copy()
        self.init_qpos = self.arrays["qpos0"].copy()
        self.init_qpos[: len(self.init_qpos_head)] = self.init_qpos_head
        self.init_qpos_env = None  # [n, nq] when the task's modify_world writes init qpos per env
        self._setup_task()
        ctrl = self.arrays["act_ctrlrange"]
        self.action_low, self.action_high = ctrl[:, 0].copy(), ctrl[:, 1].copy()
        self.camera_names = [str(x) for x in self.arrays["names_cam"]]
        self.reward = torch.zeros(self.num_envs, dtype=torch.float64, device=self.device)
        self.world_idx = np.zeros(self.num_envs, dtype=np.int64)
        # MuJoCo's bad-state resets (mj_checkAcc -> mj_resetData) per env
        self.bad_resets = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
        # the info dict's camera frames (_get_info): rendered on first access within an env-step
        self._step_id = 0
        self._frames = {}  # camera -> [step id, rgb u8 [n,H,W,3], depth f32 [n,H,W]]
        self.phase_timer = None  # optional PhaseTimer: marks the physics segment of step()

    # -- reference API ----------------------------------------------------------------------
    def _setup_task(self):
        pass

    def modify_world(self, world_idx=None, cumulative_idx=None):
        """<Task>Env.modify_world for every env (MujocoUR5eCableEnv.py:107-118,
        MujocoUR5eInsertEnv.py:65-76): the task body's offset per world index plus U(-s, s)^3
        noise from a per-env Philox stream (seed, global env index)."""
        world_idx, pos = self._world_positions(world_idx, cumulative_idx)
        bp = self.engine.body_pos
        bp[:, self._world_body, :] = torch.tensor(pos, dtype=torch.float64, device=self.device)
        self.world_idx = world_idx
        # the world changed: an earlier step's lazily rendered info frames would show it, so they
        # become stale (reading them raises, as after the next step)
        self._step_id += 1
        return world_idx

    def _world_positions(self, world_idx, cumulative_idx):
        """Per-env world index and task-body position: offset per world index plus U(-s, s)^3
        noise from a per-env Philox stream (seed, global env index = env_offset + local index)."""
        n = self.num_envs
        offsets = np.asarray(self.world_offsets, dtype=np.float64)
        if world_idx is None:
            world_idx = np.asarray(cumulative_idx) % len(offsets)
        world_idx = np.broadcast_to(np.asarray(world_idx, dtype=np.int64), (n,)).copy()
        pos = self.original_world_pos[None] + offsets[world_idx]
        if self.world_random_scale is not None:
            s = np.asarray(self.world_random_scale, dtype=np.float64)
            for e in range(n):
                rng = np.random.Generator(np.random.Philox(key=self.seed, counter=[self.env_offset + e, 0, 0, 0]))
                pos[e] += rng.uniform(low=-1.0 * s, high=s, size=3)
        return world_idx, pos

    def reset(self, seed=None, mask=None):
        """MujocoEnvBase.reset_model (:163-165): qpos = init_qpos, qvel = 0, time = 0, then
        mj_forward; returns (obs, info)."""
        e = self.engine
        # per-env initial qpos when modify_world placed a free body (init_qpos_env), else shared
        init = self.init_qpos if self.init_qpos_env is None else self.init_qpos_env
        q0 = torch.tensor(init, dtype=torch.float64, device=self.device)
        ctrl0 = torch.tensor(np.concatenate([self.init_qpos[:6], [0.0]]), dtype=torch.float64, device=self.device)
        if mask is None:
            e.qpos.copy_(q0.expand_as(e.qpos))
            e.qvel.zero_()
            e.qacc_ws.zero_()
            e.time.zero_()
            e.ctrl.copy_(ctrl0.expand_as(e.ctrl))
            e.stats.zero_()
            self.bad_resets.zero_()
        else:
            m = mask.bool()
            e.qpos[m] = q0 if q0.dim() == 1 else q0[m]
            e.qvel[m] = 0
            e.qacc_ws[m] = 0
            e.time[m] = 0
            e.ctrl[m] = ctrl0
            e.stats[m] = 0
            self.bad_resets[m] = 0
        e.forward()
        self.reward = self._get_reward()
        self._step_id += 1
        return self._get_obs(), self._get_info()  # _get_reset_info = _get_info (MujocoEnvBase.py:157-158)

    def step(self, action, active=None):
        """MujocoEnvBase.step (:82-97): ctrl = action; frame_skip x mj_step; obs; reward.
        action: f64 [n, nu] device tensor.  Images are rendered on demand (render_images)."""
        e = self.engine
        if action is not None:
            e.ctrl.copy_(action)
        if self.phase_timer is not None:
            self.phase_timer.mark("physics")
        e.step(self.frame_skip, active=active)
        if self.phase_timer is not None:
            self.phase_timer.mark("glue")
        self._reset_bad_states()
        self._step_id += 1
        obs = self._get_obs()
        self.reward = self._get_reward()
        return obs, self.reward, False, False, self._get_info()

    def _get_info(self):
        """MujocoEnvBase._get_info (:103-155) for every env: info["rgb_images"][camera] u8
        [n, H, W, 3] and info["depth_images"][camera] f32 [n, H, W] (the linearised camera depth,
        :122-125) for every camera of the scene, device tensors.  The reference renders all
        cameras on every step; here a camera is ray-cast (rgb and depth together) the first time
        either of its images is read within an env-step and cached until the next one, so steps
        whose images nobody reads cost nothing.  The tensors are the env's buffers: they hold this
        env-step's frames until the next step renders the camera again (copy to keep them).
        Tactile scenes add info["intensity_tactile"] (ur5e_pick.py)."""
        if not self.camera_names:
            return {}
        return {"rgb_images": CameraImages(self, "rgb", self._step_id),
                "depth_images": CameraImages(self, "depth", self._step_id)}

    def _info_frame(self, camera_name, kind, step_id):
        if step_id != self._step_id:
            raise RuntimeError("info images of an earlier env-step: they are rendered on first access, copy "
                               "them before the next step")
        if camera_name not in self.camera_names:
            raise KeyError(camera_name)
        ent = self._frames.get(camera_name)
        if ent is None:
            n, H, W = self.num_envs, self.renderer.height, self.renderer.width
            ent = [-1, torch.empty((n, H, W, 3), dtype=torch.uint8, device=self.device),
                   torch.empty((n, H, W), dtype=torch.float32, device=self.device)]
            self._frames[camera_name] = ent
        if ent[0] != step_id:
            self.render_images(camera_name, rgb=ent[1], depth=ent[2])
            ent[0] = step_id
        return ent[1] if kind == "rgb" else ent[2]

    def _reset_bad_states(self):
        """MuJoCo's divergence guard (mj_step -> mj_checkAcc -> mj_resetData, [ext] mujoco 3.1.6):
        the physics kernel resets an env whose forward qacc went non-finite or above 1e10 inside
        the substep where it happened (the model's qpos0, zero velocity / warm start / ctrl, time
        0), the env-step integrates its full count of substeps from the reset state (the engine's
        redo pass) and the substep of the reset is reported in stats[:, 3].  Here the resets are
        counted per env (MuJoCo's mjWARN_BADQACC counter) and the marker consumed.  Device-side,
        no host sync."""
        e = self.engine
        sub = e.stats[:, 3]
        self.bad_resets += (sub != 0).to(torch.int32)
        e.stats[:, 3] = 0

    def get_time(self):
        return self.engine.time

    def get_camera_fovy(self, camera_name):
        return float(self.arrays["cam_fovy"][self.camera_names.index(camera_name)])

    def get_body_pose(self, body_name):
        b = self.info.body[body_name]
        return torch.cat([self.engine.xpos[:, b], self.engine.xquat[:, b]], dim=1)

    def get_geom_pose(self, geom_name):
        """MujocoEnvBase.get_geom_pose: [n, 7] = geom xpos + quaternion of geom xmat (mju_mat2Quat:
        the largest of trace / diagonal branches)."""
        g = self.info.geom[geom_name]
        pos = self.engine.gxpos[:, g]
        R = self.engine.gxmat[:, g].view(-1, 3, 3)
        return torch.cat([pos, _mat2quat(R)], dim=1)

    # -- internals ----------------------------------------------------------------------------
    def _get_obs(self):
        e = self.engine
        arm_q = e.qpos.index_select(1, self._arm_qadr).contiguous()
        arm_v = e.qvel.index_select(1, self._arm_dadr).contiguous()
        grip = e.qpos.index_select(1, self._grip_qadr).contiguous()
        force = e.sensordata[:, 0:3].contiguous()
        torque = e.sensordata[:, 3:6].contiguous()
        jp, jv, wr = K.ur5e_obs(arm_q, arm_v, grip, force, torque)
        return {"joint_pos": jp, "joint_vel": jv, "wrench": wr}

    def _get_reward(self):
        raise NotImplementedError

    def render_images(self, camera_name="front", rgb=None, depth=None, policy=None, active=None, mean=None, std=None):
        """MujocoEnvBase._get_info (:103-126) for one camera, all envs; `policy` receives
        ((rgb / 255) - mean) / std as [n, 3, H, W]."""
        self.renderer.render(self.engine, camera_name, rgb=rgb, depth=depth, policy=policy, active=active,
                             mean=mean, std=std)
        return rgb, depth, policy


class CameraImages(Mapping):
    """info["rgb_images"] / info["depth_images"] of one env-step: camera name -> [n, ...] device
    tensor, rendered lazily (BatchedMujocoUR5eEnvBase._get_info)."""

    def __init__(self, env, kind, step_id):
        self._env, self._kind, self._step_id = env, kind, step_id

    def __getitem__(self, camera_name):
        return self._env._info_frame(camera_name, self._kind, self._step_id)

    def __iter__(self):
        return iter(self._env.camera_names)

    def __len__(self):
        return len(self._env.camera_names)


def _mat2quat(R):
    """mju_mat2Quat for a batch of rotation matrices [n, 3, 3] -> [n, 4] (w, x, y, z): the branch
    of the largest of the trace and the diagonal, then normalised, as MuJoCo."""
    m = R.reshape(-1, 9)
    one = 1.0
    q0 = 0.5 * torch.sqrt((one + m[:, 0] + m[:, 4] + m[:, 8]).clamp(min=0.0))
    a = torch.stack([q0, 0.25 * (m[:, 7] - m[:, 5]) / q0, 0.25 * (m[:, 2] - m[:, 6]) / q0, 0.25 * (m[:, 3] - m[:, 1]) / q0], 1)
    q1 = 0.5 * torch.sqrt((one + m[:, 0] - m[:, 4] - m[:, 8]).clamp(min=0.0))
    b = torch.stack([0.25 * (m[:, 7] - m[:, 5]) / q1, q1, 0.25 * (m[:, 1] + m[:, 3]) / q1, 0.25 * (m[:, 2] + m[:, 6]) / q1], 1)
    q2 = 0.5 * torch.sqrt((one - m[:, 0] + m[:, 4] - m[:, 8]).clamp(min=0.0))
    c = torch.stack([0.25 * (m[:, 2] - m[:, 6]) / q2, 0.25 * (m[:, 1] + m[:, 3]) / q2, q2, 0.25 * (m[:, 5] + m[:, 7]) / q2], 1)
    q3 = 0.5 * torch.sqrt((one - m[:, 0] - m[:, 4] + m[:, 8]).clamp(min=0.0))
    d = torch.stack([0.25 * (m[:, 3] - m[:, 1]) / q3, 0.25 * (m[:, 2] + m[:, 6]) / q3, 0.25 * (m[:, 5] + m[:, 7]) / q3, q3], 1)
    tr = (m[:, 0] + m[:, 4] + m[:, 8]) > 0
    c1 = (m[:, 0] > m[:, 4]) & (m[:, 0] > m[:, 8])
    c2 = m[:, 4] > m[:, 8]
    q = torch.where(tr[:, None], a, torch.where(c1[:, None], b, torch.where(c2[:, None], c, d)))
    return q / q.norm(dim=1, keepdim=True)
