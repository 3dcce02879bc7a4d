"""ORACLE — test infrastructure only (imported by tests/; never by the product package).

The reference's evaluation loop for ONE MujocoUR5eCable env on the CPU, composed from the pinned
restatements of its parts, so that the batched HIP rollout can be run beside it in lockstep
(tests/test_closed_loop_gpu.py):

* the loop              RolloutBase.run (common/base/RolloutBase.py:387-426): phase pre_update ->
                        env action (command_keys_for_step) -> env.step -> post_update ->
                        check_transition
* the phases            InitialRolloutPhase / RolloutPhase / EndRolloutPhase (RolloutBase.py:28-132),
                        ReachPhaseBase / GraspPhaseBase (common/base/PhaseBase.py:41-106),
                        ReachPhase1/2 + GraspPhase (envs/operation/OperationMujocoUR5eCable.py:8-47);
                        elapsed durations on the env clock (PhaseBase.py:19-34)
* pre-motion commands   one DLS IK step per env-step towards the phase target (ArmManager.py:220-243,
                        oracle/arm_ik.py), the gripper at action_space.high (PhaseBase.py:78-104)
* policy bookkeeping    RolloutAct.infer_policy (policy/act/RolloutAct.py:68-101): oracle/glue.py
                        ActEnsembleOracle (pinned by the reference-minted ensemble fixtures);
                        the chunk itself comes from the caller (a CPU fp32 ACT module)
* state / command       RolloutBase.get_state / set_command_data (RolloutBase.py:463-509):
                        oracle/motion.py (pinned by tests/golden/motion.npz)
* env.step              MujocoEnvBase.step (envs/mujoco/MujocoEnvBase.py:82-97): ctrl = action,
                        frame_skip x mj_step (oracle/dyn_oracle.c), _get_obs
                        (MujocoUR5eEnvBase.py:78-119) and _get_reward (MujocoUR5eCableEnv.py:48-105)
                        from oracle/glue.py
* reset                 MujocoEnvBase.reset_model (:163-165) with the caller's pole placement
                        (modify_world, MujocoUR5eCableEnv.py:107-118)

Physics parity of dyn_oracle.c with MuJoCo is unpinned (mujoco is absent from the image); every
other part is pinned by the fixtures named above.
"""

import numpy as np

from . import arm_ik, glue, motion
from .dyn import OracleEnv

ARM_JOINTS = ["shoulder_pan_joint", "shoulder_lift_joint", "elbow_joint", "wrist_1_joint", "wrist_2_joint",
              "wrist_3_joint"]
GRIPPER_JOINTS = ["right_driver_joint", "right_spring_link_joint", "left_driver_joint", "left_spring_link_joint"]
# OperationMujocoUR5eCable.py:8-47: (phase, duration [s], reach z [m])
CABLE_PRE_PHASES = (("reach", 0.7, 1.02), ("reach", 0.3, 0.995), ("grasp", 0.5, None))
TARGET_R = np.diag([-1.0, 1.0, -1.0])  # OperationMujocoUR5eCable.get_target_se3 (:8-11)


class CableRolloutOracle:
    """One env of RolloutBase.run over the MujocoUR5eCable task.  Phase indices follow
    oracle.glue.phase_schedule: 0 Initial, 1..3 the pre-motion phases, 4 Rollout, 5 End."""

    def __init__(self, arrays, init_qpos_head, pole_pos, meta, skip=3, max_duration=30.0,
                 sim_timestep=0.004, frame_skip=8):
        self.arrays = arrays
        names_body = [str(x) for x in arrays["names_body"]]
        names_jnt = [str(x) for x in arrays["names_jnt"]]
        names_geom = [str(x) for x in arrays["names_geom"]]
        qadr = arrays["jnt_qposadr"]
        dadr = arrays["jnt_dofadr"]
        self.arm_q = [int(qadr[names_jnt.index(j)]) for j in ARM_JOINTS]
        self.arm_v = [int(dadr[names_jnt.index(j)]) for j in ARM_JOINTS]
        self.grip_q = [int(qadr[names_jnt.index(j)]) for j in GRIPPER_JOINTS]
        self.cable = [i for i, n in enumerate(names_body) if n.startswith("cable_B")]
        self.cable_end = names_body.index("cable_end")
        self.poles = [names_geom.index("pole1"), names_geom.index("pole2")]
        self.dt, self.frame_skip = sim_timestep, frame_skip
        self.skip, self.max_duration = skip, max_duration
        self.meta = meta
        self.state_keys = list(meta["state"]["keys"])
        self.action_keys = list(meta["action"]["keys"])
        ctrl = arrays["act_ctrlrange"]
        self.glo, self.ghi = float(ctrl[6, 0]), float(ctrl[6, 1])
        self.P = np.ascontiguousarray(arrays["arm_placement"], dtype=np.float64)
        # modify_world + reset_model (MujocoEnvBase.py:163-165): init_qpos, zero velocity, time 0
        self.env = OracleEnv(arrays)
        self.env.set_body_pos(names_body.index("poles"), np.asarray(pole_pos, np.float64))
        qpos = arrays["qpos0"].copy()
        qpos[: len(init_qpos_head)] = init_qpos_head
        self.init_qpos = qpos
        self.ctrl = np.concatenate([qpos[:6], [0.0]])
        self.env.set_state(0.0, qpos, np.zeros(self.env.nv), np.zeros(self.env.nv), self.ctrl)
        self.env.forward()
        # ArmManager.reset (ArmManager.py:75-86): command = initial pose, target = its FK
        self.arm = motion.ArmCommand(self.P, qpos[:6], 0.0)
        self.ens = glue.ActEnsembleOracle(meta["data"]["chunk_size"], meta["action"])
        self.phase, self.start_time = 0, 0.0
        self.rollout_time_idx, self.success_time = 0, None
        self.result = None
        self.policy_action = None
        self.obs = self._obs()
        self.reward = self._reward()

    # -- env ------------------------------------------------------------------------------------
    def time(self):
        return self.env.state()[0]

    def qpos(self):
        return self.env.state()[1]

    def _obs(self):
        """MujocoUR5eEnvBase._get_obs (:78-119)."""
        _, qp, qv, _ = self.env.state()
        s = self.env.sensor()
        jp, jv, wr = glue.ur5e_obs(qp[self.arm_q], qv[self.arm_v], qp[self.grip_q], s[0:3], s[3:6])
        return {"joint_pos": jp, "joint_vel": jv, "wrench": wr}

    def _reward(self):
        """MujocoUR5eCableEnv._get_reward (:48-105) on the oracle's body / geom positions."""
        xpos, _ = self.env.xpos()
        gx, _ = self.env.geom_frames()
        return glue.cable_reward(xpos[self.cable], xpos[self.cable_end], gx[self.poles[0]], gx[self.poles[1]])

    def _env_step(self, action):
        """MujocoEnvBase.step (:82-97)."""
        self.ctrl = np.asarray(action, np.float64).copy()
        self.env.set_ctrl(self.ctrl)
        bad = self.env.step(self.frame_skip)
        if bad:
            raise RuntimeError("oracle divergence reset inside the closed loop")
        self.obs = self._obs()
        self.reward = self._reward()

    # -- rollout --------------------------------------------------------------------------------
    @property
    def n_pre(self):
        return 1 + len(CABLE_PRE_PHASES)

    def needs_inference(self):
        """RolloutPhase.pre_update (RolloutBase.py:56-63) will call infer_policy this env-step."""
        return self.phase == self.n_pre and self.rollout_time_idx % self.skip == 0

    def policy_state(self):
        """RolloutBase.get_state (:463-477): routed keys, normalize_data, f32."""
        raw = motion.get_raw_state(self.state_keys, self.obs["joint_pos"], self.obs["joint_vel"],
                                   self.obs["wrench"], self.arm)
        return glue.normalize(raw, self.meta["state"]).astype(np.float32)

    def _start_phase(self):
        """PhaseBase.start (:19-20) and the phase's set_target."""
        self.start_time = self.time()
        if 1 <= self.phase < self.n_pre:
            kind, _, z = CABLE_PRE_PHASES[self.phase - 1]
            if kind == "reach":  # OperationMujocoUR5eCable.get_target_se3 (:8-11)
                p = self.env.xpos()[0][self.cable_end].copy()
                p[2] = z
                self.target = (TARGET_R.copy(), p)
        elif self.phase == self.n_pre:  # RolloutPhase.start (:44-47)
            self.rollout_time_idx, self.success_time = 0, None

    def step(self, chunk=None):
        """One iteration of RolloutBase.run's loop.  `chunk` (f32 [chunk_size, A]) is the policy
        output on this env-step's state and image when needs_inference(); ignored otherwise."""
        if self.phase > self.n_pre:
            return
        # phase_manager.pre_update()
        if 1 <= self.phase < self.n_pre:
            kind, _, _ = CABLE_PRE_PHASES[self.phase - 1]
            if kind == "reach":  # ReachPhaseBase.pre_update -> COMMAND_EEF_POSE (one IK step)
                R, p = self.target
                self.arm.R, self.arm.p = R.copy(), p.copy()
                self.arm.q = arm_ik.ik_step(self.P, self.arm.q, R, p)
            else:  # GraspPhaseBase.pre_update -> COMMAND_GRIPPER_JOINT_POS at action_space.high
                self.arm.g = np.clip(np.array([self.ghi]), self.glo, self.ghi)
        elif self.phase == self.n_pre:
            if self.needs_inference():
                if chunk is None:
                    raise ValueError("this env-step runs the policy: a chunk is required")
                self.policy_action = self.ens.step(lambda: chunk)
            is_skip = self.rollout_time_idx % self.skip != 0
            motion.set_command(self.action_keys, self.policy_action, is_skip, self.arm, self.glo, self.ghi)
        # env_action = command_joint_pos (EnvDataMixin command_keys_for_step); env.step
        self._env_step(np.concatenate([self.arm.q, self.arm.g]))
        # phase_manager.post_update()
        if self.phase == self.n_pre:
            self.rollout_time_idx += 1
        # phase_manager.check_transition()
        el = self.time() - self.start_time
        trans = False
        if self.phase == 0:
            trans = el > 1.0
        elif self.phase < self.n_pre:
            trans = el > CABLE_PRE_PHASES[self.phase - 1][1]
        else:
            if self.reward >= 1.0 and self.success_time is None:
                self.success_time = el
            if self.success_time is not None:
                trans = el > self.success_time + 1.0
            else:
                trans = el > self.max_duration
            if trans:
                self.result = (bool(self.reward >= 1.0), float(self.reward), el)
        if trans:
            self.phase += 1
            self._start_phase()
