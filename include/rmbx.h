/*
 * rmbx.h — C ABI of the MI355X-native batched policy-rollout engine.
 *
 * Every entry point is extern "C", takes plain pointers (device memory unless stated) and sizes,
 * returns an int status (RMBX_OK = 0, negative on error; the message is available from
 * rmbx_last_error(), thread-local) and enqueues its work on the caller's HIP stream
 * (`stream` is a hipStream_t passed as void*, NULL = the legacy default stream).
 * No call allocates, frees or synchronises on the hot path, so every hot-path call can be
 * captured in a hipGraph.  Ownership: the engine owns the device copy of the model constants;
 * per-env state (qpos, qvel, warm start, ctrl, ...) and the solver workspace are caller-owned
 * device buffers attached with rmbx_engine_bind, so the caller (torch) keeps them resident and
 * can read them zero-copy.  Threading: one host thread per engine; calls on one engine handle
 * are not re-entrant.
 *
 * Each function cites the reference (yusuke1127/RoboManipBaselines @2.0.0) interface it replaces
 * for a batch of environments; paths are relative to the reference package root
 * robo_manip_baselines/.
 */
#ifndef RMBX_H_
#define RMBX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMBX_OK 0
#define RMBX_ERR_ARG -1   /* bad argument (maps to Python ValueError) */
#define RMBX_ERR_HIP -2   /* HIP runtime failure (maps to Python RuntimeError) */
#define RMBX_ERR_STATE -3 /* engine used in a wrong state */

#define RMBX_ABI_VERSION 2

/* ---------------------------------------------------------------------------------------------
 * Library
 * ------------------------------------------------------------------------------------------- */
int rmbx_abi_version(void);
const char* rmbx_last_error(void);
/* Number of visible HIP devices (0 when none). Does not create a context. */
int rmbx_device_count(int* count);

/* ---------------------------------------------------------------------------------------------
 * ACT temporal ensembling + action denormalisation, batched over envs.
 * Replaces policy/act/RolloutAct.py:68-101 (infer_policy: history append/pop at
 * chunk_size, exponential weights k = 0.01, newest-first accumulation, and the
 * --no_temp_ensem pop(0) path) followed by common/utils/DataUtils.py:26-40 (denormalize_data).
 *
 * hist        f32 [n_env][chunk][chunk][adim]  per-env ring of past chunks (engine-owned layout)
 * hist_len    i32 [n_env]  number of valid chunks in the ring (TE) / rows left (no TE)
 * hist_head   i32 [n_env]  ring slot of the oldest chunk (TE) / next row to pop (no TE)
 * new_chunk   f32 [n_env][chunk][adim]  policy output of this call (read where push != 0)
 * push        u8  [n_env]  1 = append new_chunk (TE) / reload the buffer (no TE); NULL = all 1
 * active      u8  [n_env]  0 = env untouched this call; NULL = all active
 * w_table     f64 [chunk][chunk]  w_table[n-1][i] = exp(-k i) / sum_j exp(-k j), i < n,
 *             built on the host with numpy exactly as RolloutAct.py:90-92 (bit-exact weights)
 * dn_scale, dn_sub, dn_add  f64 [adim]: out = dn_scale * (a - dn_sub) + dn_add
 *             (gaussian: std, 0, mean; limits: range/(out_max-out_min), out_min, min)
 * out         f64 [n_env][adim]  denormalised action (RolloutAct.py:98 self.policy_action)
 * Arithmetic: f64, no contraction, reference order (bit-exact vs the reference on golden data).
 * ------------------------------------------------------------------------------------------- */
int rmbx_act_ensemble(const float* new_chunk, const uint8_t* push, const uint8_t* active,
                      float* hist, int32_t* hist_len, int32_t* hist_head,
                      const double* w_table, const double* dn_scale, const double* dn_sub,
                      const double* dn_add, double* out, int n_env, int chunk, int adim,
                      int temporal_ensemble, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Cable-threading success predicate, batched.
 * Replaces envs/mujoco/ur5e/MujocoUR5eCableEnv.py:48-105 (_get_reward).
 * cable_xpos f64 [n_env][n_cable][3] (cable_B0..B{n_cable-1} in body-id order),
 * end_xpos / pole1_xpos / pole2_xpos f64 [n_env][3]; reward f64 [n_env] in {0, 1}.
 * Bit-exact flags: same f64 comparisons, no contraction, NaN behaviour of numpy max.
 * ------------------------------------------------------------------------------------------- */
int rmbx_cable_reward(const double* cable_xpos, const double* end_xpos,
                      const double* pole1_xpos, const double* pole2_xpos, double* reward,
                      int n_env, int n_cable, void* stream);

/* Peg-in-hole success predicate, batched.
 * Replaces envs/mujoco/ur5e/MujocoUR5eInsertEnv.py:43-63 (_get_reward): 1 iff
 * max|peg.xy - hole.xy| < xy_thre (0.012), peg.z < hole.z + z_offset (0.05) and
 * dot(peg z axis, (0, 0, -1)) > cos_tilt (np.cos(np.deg2rad(10)), passed in from the host).
 * peg_xpos / hole_xpos f64 [n_env][3], peg_xquat f64 [n_env][4] (z axis = column 2 of
 * mju_quat2Mat); reward f64 [n_env].  Bit-exact: numpy's operation order, NaN -> 0. */
int rmbx_insert_reward(const double* peg_xpos, const double* hole_xpos, const double* peg_xquat, double* reward,
                       int n_env, double xy_thre, double z_offset, double cos_tilt, void* stream);

/* Cabinet reward, batched.
 * Replaces envs/mujoco/ur5e/MujocoUR5eCabinetEnv.py:57-73 (_get_reward): 1.0 when the "hinge"
 * joint exceeds hinge_thre (np.deg2rad(120)) and/or the "slide" joint exceeds slide_thre
 * (0.12 m), per target_task (0 = None: either, 1 = "hinge", 2 = "slide"; anything else is the
 * reference's ValueError -> -1).  qpos f64 [n_env][qpos_stride]; hinge_adr / slide_adr are the
 * joints' qpos addresses.  Bit-exact (comparisons only). */
int rmbx_cabinet_reward(const double* qpos, int qpos_stride, int hinge_adr, int slide_adr, double hinge_thre,
                        double slide_thre, int target_task, double* reward, int n_env, void* stream);

/* Toolbox placement reward, batched.
 * Replaces envs/mujoco/ur5e/MujocoUR5eToolboxEnv.py:46-57 (_get_reward): 1.0 iff
 * max(|toolbox - mat|_xy) < xy_thre (0.03 m; NaN fails, as numpy's max propagates it) and
 * toolbox_z < mat_z + z_offset (0.005 m).  toolbox_xpos, mat_xpos: body xpos f64 [n_env][3].
 * Bit-exact (comparisons only). */
int rmbx_toolbox_reward(const double* toolbox_xpos, const double* mat_xpos, double* reward, int n_env,
                        double xy_thre, double z_offset, void* stream);

/* Ring-on-pole reward, batched.
 * Replaces envs/mujoco/ur5e/MujocoUR5eRingEnv.py:46-75 (_get_reward): 0 if the highest ring
 * body is above pole_z + 0.08 (numpy max: NaN never compares above); else 1 iff
 * matplotlib.path.Path(ring xy + ring[0] xy).contains_point(pole xy) -- crossing-number test,
 * non-finite vertices dropped with the next finite one opening a new subpath, exactly as
 * matplotlib's point_in_path / PathNanRemover.  ring_xpos f64 [n_env][n_ring][3] (ring_B*
 * bodies in body order), pole_xpos f64 [n_env][3].  Bit-exact (no contraction). */
int rmbx_ring_reward(const double* ring_xpos, const double* pole_xpos, double* reward, int n_env, int n_ring,
                     void* stream);

/* Door-opening reward, batched.
 * Replaces envs/mujoco/ur5e/MujocoUR5eDoorEnv.py:52-67 (_get_reward): 0.5 * (reaching + opening)
 * with reaching = exp(-10 max(|pinch - handle| - margin, 0)) (1 once the door is open),
 * opening = clip(door_angle / target_angle, 0, 1); margin 0.08, target np.deg2rad(-45) from the
 * host.  pinch_xpos (site "pinch"), handle_xpos (geom "door_handle") f64 [n_env][3], door_angle
 * f64 [n_env].  The success flag (reward >= 1.0 <=> opening >= 1) is bit-exact; the reward value
 * follows numpy's operation order, exp from the device libm (within 1 ulp of numpy's). */
int rmbx_door_reward(const double* pinch_xpos, const double* handle_xpos, const double* door_angle, double* reward,
                     int n_env, double margin, double target_angle, void* stream);

/* ---------------------------------------------------------------------------------------------
 * UR5e observation mapping, batched.
 * Replaces envs/mujoco/ur5e/MujocoUR5eEnvBase.py:78-119 (_get_obs):
 * joint_pos = [6 arm qpos, rad2deg(mean(4 gripper qpos)) / 45 * 255], joint_vel = [6 arm qvel, 0],
 * wrench = [force(3), torque(3)].
 * arm_qpos, arm_qvel f64 [n][6]; grip_qpos f64 [n][4] (right_driver, right_spring_link,
 * left_driver, left_spring_link); force, torque f64 [n][3].
 * ------------------------------------------------------------------------------------------- */
int rmbx_ur5e_obs(const double* arm_qpos, const double* arm_qvel, const double* grip_qpos,
                  const double* force, const double* torque, double* joint_pos,
                  double* joint_vel, double* wrench, int n_env, void* stream);

/* ---------------------------------------------------------------------------------------------
 * OpenGL depth-buffer linearisation, batched (f32, numpy NEP-50 semantics).
 * Replaces envs/mujoco/MujocoEnvBase.py:122-125: depth = near / (1 - z * (1 - near / far)),
 * near = znear * extent, far = zfar * extent.
 * ------------------------------------------------------------------------------------------- */
int rmbx_depth_linearize(const float* zbuf, float* depth, size_t n_pix, double near_,
                         double far_, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Rollout phase schedule, batched state machine.
 * Replaces the per-step check_transition/post_update of common/base/RolloutBase.py:28-132
 * (InitialRolloutPhase, RolloutPhase with --auto_exit, EndRolloutPhase) and the timed
 * pre-motion phases of common/base/PhaseBase.py:41-106 under
 * common/manager/PhaseManager.py:20-37, driven by the env clock (MujocoEnvBase.py:201-203).
 * Called once per env-step AFTER the physics step with that step's sim time and reward.
 *
 * pre_durations f64 [n_pre]: durations of the phases before RolloutPhase (Initial first);
 * phase index n_pre = RolloutPhase, n_pre + 1 = EndRolloutPhase.
 * ------------------------------------------------------------------------------------------- */
typedef struct rmbx_sched_t {
  int32_t phase;            /* current phase index */
  int32_t rollout_time_idx; /* RolloutBase.py:47,70 */
  uint8_t done;             /* EndRolloutPhase reached and episode finished */
  uint8_t success;          /* result["success"] */
  uint8_t has_success_time; /* success_time is not None */
  uint8_t pad_[5];
  double phase_start;   /* PhaseBase.start_time */
  double success_time;  /* RolloutPhase.success_time (valid if has_success_time) */
  double result_reward; /* result["reward"] */
  double duration;      /* result["duration"] */
} rmbx_sched_t;

int rmbx_sched_reset(rmbx_sched_t* sched, const double* time, const uint8_t* mask, int n_env,
                     void* stream);
int rmbx_sched_update(rmbx_sched_t* sched, const double* time, const double* reward,
                      const double* pre_durations, int n_pre, double max_duration,
                      double post_success_duration, int n_env, void* stream);
/* active[e] = 1 while env e has not reached EndRolloutPhase (phase <= n_pre and not done), else
 * 0: the step mask that freezes each env at its RolloutPhase -> EndRolloutPhase transition, so
 * its final state (and a --save_last_image frame, RolloutBase.py:109-110, 541-561) is the
 * transition step's, as the reference's saved image is. */
int rmbx_sched_active(const rmbx_sched_t* sched, int n_pre, uint8_t* active, int n_env, void* stream);


/* ---------------------------------------------------------------------------------------------
 * Batched MuJoCo-subset physics engine (the env.step hot path).
 * Replaces, for n_env environments in lockstep, the per-env
 *   envs/mujoco/MujocoEnvBase.py:82-97 step() -> gymnasium do_simulation -> mujoco.mj_step x
 *   frame_skip (MujocoEnvBase.py:12-13: dt 0.004, frame_skip 8) + mj_rnePostConstraint,
 * and MujocoEnvBase.py:163-165 reset_model (state set by the caller).
 * Per substep two launches over all envs: a front kernel (one wavefront per env: kinematics,
 * composite inertia, RNE, collision, constraint rows) and a solver kernel (256 threads per env:
 * Newton solve, forces, sensors, implicitfast integration).  The constraint Jacobian is never
 * stored (rows are described by contact / joint / equality data; J x, J^T w and the Hessian
 * chunks are computed from the dof axes in LDS) and the mass matrix is kept as packed lower
 * 4x4 blocks.  The model comes from include/rmbx_model.h (host pointers, copied to the device
 * at create).
 * ------------------------------------------------------------------------------------------- */
typedef struct rmbx_engine rmbx_engine;
struct rmbx_model;

/* Caller-owned device buffers, all [n_env][...] row-major f64 unless noted. */
typedef struct rmbx_env_buffers {
  double* time;       /* [n]            simulation time (MujocoEnvBase.get_time) */
  double* qpos;       /* [n][nq] */
  double* qvel;       /* [n][nv] */
  double* qacc_ws;    /* [n][nv]        warm start (MuJoCo qacc_warmstart) */
  double* ctrl;       /* [n][nu] */
  double* body_pos;   /* [n][nbody][3]  per-env body offsets (modify_world pole pose) */
  double* xpos;       /* [n][nbody][3]  out: body positions of the last forward pass */
  double* xquat;      /* [n][nbody][4]  out */
  double* gxpos;      /* [n][ngeom][3]  out: geom frames (collision and render geoms) */
  double* gxmat;      /* [n][ngeom][9]  out */
  double* sensordata; /* [n][6]         out: force(3) torque(3) site sensors */
  int32_t* stats;     /* [n][4]         out: ncon, nefc, solver iterations, bad-state flag */
  void* workspace;    /* engine scratch, rmbx_engine_workspace_bytes() bytes */
} rmbx_env_buffers;

/* Model limits checked here (RMBX_ERR_ARG otherwise): npair <= 65535 (the collision stage indexes
 * pairs in 16 bits) and the front kernel's LDS (body frames + the collision scratch) <= 64 KiB.
 * The front kernel's launch LDS is sized here for n_env (padded so the envs spread evenly over the
 * CUs and rounds of blocks; RMBX_FRONT_BALANCE=0 in the environment at creation: the plain need). */
int rmbx_engine_create(const struct rmbx_model* model, int n_env, rmbx_engine** out);
int rmbx_engine_destroy(rmbx_engine* eng);
int rmbx_engine_workspace_bytes(const rmbx_engine* eng, size_t* bytes);
/* offset (in doubles, within one env's workspace slice) and element count of a named
 * workspace array (e.g. "M", "qfrc_bias", "qacc", "J", "con_pos"); per-env stride via "stride".
 * The int32 arrays "con_b1" / "con_b2" (contact bodies) report offsets in int32 units. */
int rmbx_engine_ws_offset(const rmbx_engine* eng, const char* name, size_t* offset,
                          size_t* count);
int rmbx_engine_bind(rmbx_engine* eng, const rmbx_env_buffers* bufs);
/* nsub x mj_step on every env with active[e] != 0 (NULL = all). */
int rmbx_engine_step(rmbx_engine* eng, int nsub, const uint8_t* active, void* stream);
/* mj_forward only (no integration): fills the outputs and workspace for inspection. */
int rmbx_engine_forward(rmbx_engine* eng, const uint8_t* active, void* stream);
/* Diagnostic: step all envs and accumulate per-stage shader cycles into stage_cycles
 * [n_env][32] (u64, device): kinematics, com/crb, velocity+rne+actuation, collision,
 * constraints, solver, sensors, integration; 8-15 solver sub-stages, 16-18 collision
 * sub-stages, 20-23 constraint sub-stages, 24-30 J^T w / J x / M x pass internals. */
int rmbx_engine_step_profiled(rmbx_engine* eng, int nsub, uint64_t* stage_cycles, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Arm command: batched FK and damped-least-squares IK steps (reach phases).
 * Replaces common/body/ArmManager.py:213-218 (forward_kinematics) and :220-243
 * (inverse_kinematics, one iteration per call in the reference; n_iter here) with the Pinocchio
 * URDF chain of envs/assets/common/robots/ur5e/ur5e.urdf (root pose folded into placement 0).
 * placement f64 [6][12] (R row-major, p); q_cmd f64 [n][6] updated in place; target_R f64 [n][9];
 * target_p f64 [n][3]; mask u8 [n] (NULL = all).
 * ------------------------------------------------------------------------------------------- */
int rmbx_arm_ik(const double* placement, double* q_cmd, const double* target_R,
                const double* target_p, const uint8_t* mask, int n_env, int n_iter,
                void* stream);
int rmbx_arm_fk(const double* placement, const double* q, double* R_out, double* p_out,
                int n_env, void* stream);

/* ---------------------------------------------------------------------------------------------
 * DataKey routing for the UR5e arm + gripper (one ArmManager, eef_idx 0).
 * Key codes name common/data/DataKey.py:14-58; RMBX_MAX_DATA_KEYS keys per call.
 *
 * rmbx_motion_state replaces RolloutBase.get_state's concatenation (RolloutBase.py:463-473) of
 * MotionManager.get_data (MotionManager.py:41-130): the raw f64 state [n][state_dim] of the keys
 * in order, before normalize_data.  measured_* keys read the observation (joint_pos f64 [n][7],
 * joint_vel f64 [n][7], wrench f64 [n][6]); measured_eef_pose = FK of the measured arm joints as
 * (t, qw, qx, qy, qz) (ArmManager.py:161-165, MathUtils.py:27-31); command_* keys read the command
 * state (q_cmd f64 [n][6], grip_cmd f64 [n], IK target target_R f64 [n][9] / target_p f64 [n][3]).
 * Keys the reference cannot serve as state (the *_rel keys, MotionManager.py:87-90) are
 * RMBX_ERR_ARG.
 *
 * rmbx_motion_command replaces RolloutBase.set_command_data (RolloutBase.py:496-509) ->
 * MotionManager.set_command_data (:25-39) -> ArmManager.set_command_data (ArmManager.py:88-159):
 * slices of action f64 [n][action_dim] applied key by key to the command state in place:
 * command_joint_pos (arm + gripper; IK target := FK), command_joint_pos_rel (added unless
 * is_skip), command_gripper_joint_pos (clipped to [grip_low, grip_high]), command_eef_pose
 * (target := SE3(quaternion(w, x, y, z), t), one DLS IK step), command_eef_pose_rel (target :=
 * target * SE3(rpy, t) on every call, as the reference does not forward is_skip there; one IK
 * step).  Other keys are RMBX_ERR_ARG (MotionManager.py:36-39).  mask u8 [n] (NULL = all).
 * ------------------------------------------------------------------------------------------- */
#define RMBX_MAX_DATA_KEYS 8
#define RMBX_KEY_MEASURED_JOINT_POS 1
#define RMBX_KEY_MEASURED_JOINT_VEL 2
#define RMBX_KEY_MEASURED_GRIPPER_JOINT_POS 3
#define RMBX_KEY_MEASURED_EEF_POSE 4
#define RMBX_KEY_MEASURED_EEF_WRENCH 5
#define RMBX_KEY_COMMAND_JOINT_POS 16
#define RMBX_KEY_COMMAND_JOINT_POS_REL 17
#define RMBX_KEY_COMMAND_GRIPPER_JOINT_POS 18
#define RMBX_KEY_COMMAND_EEF_POSE 19
#define RMBX_KEY_COMMAND_EEF_POSE_REL 20

int rmbx_motion_state(const double* placement, const double* joint_pos, const double* joint_vel,
                      const double* wrench, const double* q_cmd, const double* grip_cmd,
                      const double* target_R, const double* target_p, const int32_t* keys,
                      int n_keys, double* state_out, int state_dim, int n_env, void* stream);
int rmbx_motion_command(const double* placement, const double* action, int action_dim,
                        const int32_t* keys, int n_keys, int is_skip, double grip_low,
                        double grip_high, double* q_cmd, double* grip_cmd, double* target_R,
                        double* target_p, const uint8_t* mask, int n_env, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Batched camera rendering (ray casting of the scene primitives).
 * Replaces the per-camera OffScreenViewer rgb/depth renders of envs/mujoco/MujocoEnvBase.py:
 * 112-126 for one camera over n_env envs.  Primitive table (device): prim_i32 [nprim][4]
 * = (geom id, type, -, -), prim_f32 [nprim][8] = (size3, rgb3, -, -).  Geom frames come from the
 * engine outputs gxpos/gxmat; the camera frame from body xpos/xquat + camera offset.
 * Outputs (each optional): rgb u8 [n][H][W][3]; depth f32 [n][H][W] (linear camera-z distance,
 * the quantity MujocoEnvBase.py:122-125 recovers); policy tensor [n][3][H][W] in bf16 (dtype 1)
 * or f32 (dtype 0) = ((u8 / 255) - mean[c]) / std[c] (RolloutBase.py:479-490 + ImageNet
 * normalisation of the ACT/MLP backbones), or (dtype 2) the same values in bf16 as a 2x2
 * space-to-depth image [n][H/2][W/2][16] (channel (dy*2+dx)*3+c, 12..15 zero) for
 * rmbx_stem_s2d_conv (H, W even), or (dtype 3) that space-to-depth image in f32 for
 * rmbx_stem_s2d_conv_maxpool_f32, or (dtype 4) the space-to-depth image of the 8-bit values u
 * themselves (u8, mean/std not applied) for rmbx_stem_s2d_conv_maxpool_u8.
 * ------------------------------------------------------------------------------------------- */
typedef struct rmbx_camera {
  int32_t body;        /* body the camera is attached to (0 = world) */
  int32_t width, height;
  float fovy_deg;
  double pos[3];       /* camera position in the body frame */
  double quat[4];      /* camera orientation in the body frame (MuJoCo: looks along -z) */
  float znear, zfar;   /* clip distances for depth (metres) */
  float mean[3], std[3];
} rmbx_camera;

int rmbx_render(const rmbx_camera* cam, const int32_t* prim_i32, const float* prim_f32,
                int nprim, const double* gxpos, const double* gxmat, const double* xpos,
                const double* xquat, int ngeom, int nbody, uint8_t* rgb, float* depth,
                void* policy_img, int policy_dtype, const uint8_t* active, int n_env,
                void* stream);

/* The scene with its visual meshes (the reference renders every class="visual" mesh geom,
 * envs/mujoco/MujocoEnvBase.py:103-126, through MuJoCo's OpenGL viewer).  Device tables:
 * prim_i32 [nprim][4] = (geom id, type, -, -) and prim_f32 [nprim][8] = (size3, rgb3, -, -) as for
 * rmbx_render (the analytic primitives); mesh_tri f32 [ntri][16] = the visual meshes' triangles in
 * their body frames, (v0, e1 = v1 - v0, e2 = v2 - v0, unit face normal, tag = (mesh slot << 16) |
 * geom id as int32 bits, rgb), mjcf/rmesh.py builds them; per mesh slot (a body with visual
 * meshes) mesh_body [nmesh] its body id and mesh_rad [nmesh] its triangles' bounding radius about
 * the body origin.  vis: caller-provided device workspace u64 [n_env][H][W] (16-byte aligned),
 * all ones (empty) on entry, filled with each pixel's nearest triangle (depth bits << 32 | index)
 * and left empty again by the call; tflag: u8 [n_env][tiles of 16x16 pixels], zero on entry and
 * on return (the tiles the visibility pass wrote);
 * triangle hits nearer than cam->znear are clipped (OpenGL's near plane).  hit_geom (optional)
 * [n][H][W] receives the geom id of each pixel's surface, -1 for the background; the other
 * arguments and outputs are rmbx_render's.  rmbx_render is this call without meshes. */
typedef struct rmbx_scene_tables {
  const int32_t* prim_i32;
  const float* prim_f32;
  int32_t nprim;
  int32_t ntri, nmesh;
  const float* mesh_tri;
  const int32_t* mesh_body;
  const float* mesh_rad;
  unsigned long long* vis;
  uint8_t* tflag;
  /* materials (optional; geom_matinfo NULL: flat material colours, no specular term, background
   * (0.9, 1, 1) -- the round-5 shading).  Indexed by geom id: geom_texid [ngeom] the texture of
   * the geom's material (-1: none; primitives only), geom_matinfo [ngeom][6] = (specular,
   * shininess, texrepeat x, y, texuniform, emission) of MuJoCo's <material>
   * (envs/assets/mujoco/envs/ur5e/env_ur5e_common.xml:13-25); textures tex_desc [ntex][4] =
   * (type 0 "2d" / 1 "cube", height, width, first texel), texels tex_rgba as RGBA8 words (R in the
   * low byte, rows in file order), each texture followed by its box-filtered mip levels, whose
   * first texels tex_level_adr lists (relative to the texture's; level l
   * max(H >> l, 1) x max(W >> l, 1) down to 1 x 1, texel = (sum of the 2 x 2 texels above, rows /
   * columns clamped, + 2) / 4); sky_rgb = the gradient skybox's rgb1 (up), rgb2 (down).
   * Sampling (trilinear as GL_LINEAR_MIPMAP_LINEAR with an isotropic footprint: level of detail
   * log2(t pix / max(n.v, 1e-3) x density), t the camera depth, pix = 2 tan(fovy / 2) / height, the
   * density in base texels per metre -- 2d: max(rx W, ry H) per metre of repeat, cube: max(W, H) /
   * (2 |major axis coordinate|); bilinear per level, texel centres at +0.5): 2d from the hit's
   * local (x, y), repeated
   * texrepeat times over the geom's (2 size_x, 2 size_y) extent, or per metre when texuniform or
   * the plane is infinite; cube from the local hit point (divided by the geom's half extents when
   * texuniform) as a cube-map direction, the same image on all six faces, OpenGL's face
   * orientation, clamped at the face edges.  Shading: material colour x texture x (0.1 ambient +
   * 0.6 headlight |n.v| + 0.3 max(0, n.z) + emission) + specular x 0.3 x max(0, n.h)^(128
   * shininess) for the directional light (world +z towards it, h the half vector), clamped at 1. */
  const int32_t* geom_texid;
  const float* geom_matinfo;
  const uint32_t* tex_rgba;
  const int32_t* tex_desc;
  const int32_t* tex_level_adr; /* [ntex][RMBX_TEX_LEVELS]: first texel of each mip level */
  int32_t ntex;
  float sky_rgb[6];
} rmbx_scene_tables;
#define RMBX_TEX_LEVELS 16 /* mip levels per texture (images up to 32768 texels wide) */

int rmbx_render_scene(const rmbx_camera* cam, const rmbx_scene_tables* scene, const double* gxpos,
                      const double* gxmat, const double* xpos, const double* xquat, int ngeom,
                      int nbody, uint8_t* rgb, float* depth, int32_t* hit_geom, void* policy_img,
                      int policy_dtype, const uint8_t* active, int n_env, void* stream);

/* Static-background cache of one camera (rmbx_render_scene_cached; the caller keeps one per
 * camera and image size).  A primitive is static when its body is welded to the world
 * (prim_static [nprim] = 1; static_prims [nstatic] their indices); for a camera whose pose does not
 * change either (a world camera: the rollout's policy camera), every pixel whose nearest surface
 * among the static primitives is drawn once per episode: cache u32 [n_env][H][W][2] (8-byte
 * aligned) = (its camera depth bits, 8-bit rgb | primitive << 24; primitive 0xff: none) is rebuilt
 * for an env whenever the camera body's pose or a static primitive's pose differs from the snapshot
 * snap f64 [n_env][7 + 12 nstatic] (caller-initialised to NaN: the first call builds every cache)
 * it was built from; dirty u8 [n_env] is workspace.  Each call then casts only the other primitives
 * and the meshes against the cached depth and primitive (the same nearest-hit order: meshes keep
 * ties, primitives by index), so every output (rgb, depth, hit_geom, policy) equals
 * rmbx_render_scene's, which is this call with cache NULL.  RMBX_RENDER_CACHE=0 ignores the
 * cache. */
typedef struct rmbx_render_cache {
  const uint8_t* prim_static;
  const int32_t* static_prims;
  int32_t nstatic;
  uint32_t* cache;
  double* snap;
  uint8_t* dirty;
} rmbx_render_cache;

int rmbx_render_scene_cached(const rmbx_camera* cam, const rmbx_scene_tables* scene, const double* gxpos,
                             const double* gxmat, const double* xpos, const double* xquat, int ngeom,
                             int nbody, uint8_t* rgb, float* depth, int32_t* hit_geom, void* policy_img,
                             int policy_dtype, const uint8_t* active, int n_env,
                             const rmbx_render_cache* cache, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Policy vision-trunk epilogues (ResNet-18 with frozen BN folded into the convs), NHWC.
 * Replace the per-element tail of torchvision's BasicBlock / stem as used by ACT's DETR backbone
 * (third_party/act, absent submodule) and policy/mlp/MlpPolicy.py:34-39:
 *   conv -> BN -> ReLU [-> maxpool 3x3/2 pad 1]   and   conv -> BN -> (+ identity/downsample) -> ReLU.
 * x, res, out: [n_pix][C] activations in the storage dtype (dtype 1 = bf16, 0 = f32), 16-byte
 * aligned, C a multiple of 8 (bf16) / 4 (f32); bias, res_bias: f32 [C] (values representable in
 * the storage dtype).  out = relu?(rnd(rnd(x + bias) + rnd(res + res_bias))), res / res_bias
 * optional (NULL), every intermediate rounded to the storage dtype as the unfused path does.
 * out may alias x.
 * ------------------------------------------------------------------------------------------- */
int rmbx_nhwc_bias_act(const void* x, const float* bias, const void* res, const float* res_bias,
                       void* out, size_t n_pix, int C, int relu, int dtype, void* stream);
/* Implicit-GEMM convolution (MFMA, bf16 NHWC) with the fused epilogue
 * out = relu?(conv(in, weight) + bias + residual), one bf16 rounding; replaces conv -> BN ->
 * (+ identity/downsample) -> ReLU of the ResNet-18 BasicBlocks (BN folded into weight/bias).
 * in [N][H][W][Cin], weight [Cout][KH][KW][Cin], residual/out [N][Ho][Wo][Cout] bf16, bias f32;
 * Cin % 64 == 0, Cout % 64 == 0, residual optional (NULL). */
int rmbx_conv2d_nhwc(const void* in, const void* weight, const float* bias, const void* residual,
                     void* out, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                     int pad, int relu, void* stream);
/* The same conv in f32 (the reference's fp32 policy): in/weight/residual/out f32 in the layouts
 * above, exact f32 products with f32 accumulation (v_mfma_f32_32x32x2_f32), bias + residual +
 * ReLU applied to the accumulators before the single store.  Implemented for the ResNet-18
 * layer-1 conv only (KH = KW = 3, stride 1, pad 1, Cin = Cout = 64); other shapes return
 * RMBX_ERR_ARG. */
int rmbx_conv2d_nhwc_f32(const float* in, const float* weight, const float* bias, const float* residual,
                         float* out, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad, int relu, void* stream);
/* Winograd F(2x2, 3x3) form of the fp32 stride-1 / pad-1 3x3 conv of the ResNet-18 BasicBlocks
 * (Cin = Cout = C in {64, 128, 256, 512}; replaces the same conv -> FrozenBN -> (+ residual) ->
 * ReLU steps as rmbx_conv2d_nhwc_f32, for every stride-1 layer of the fp32 policy trunk):
 * in / residual / out [N][H][W][C] f32 (out must not alias in or residual), u_packed = the
 * filter transform G g G^T of the BN-folded weights in the kernel's staging order
 * [C/64][C/8][16][2][32][8] f32 (robomanipbaselines_amd.kernels.pack_winograd_f32), bias [C] f32.
 * out = relu?(conv + bias + residual), f32 MFMA products, f32 accumulation. */
int rmbx_conv3x3_winograd_f32(const float* in, const float* u_packed, const float* bias,
                              const float* residual, float* out, int N, int H, int W, int C, int relu,
                              void* stream);
/* Winograd F(4x4, 3x3) form of the same conv (2.25 products per output instead of 4): same
 * operands and result as rmbx_conv3x3_winograd_f32 with u_packed = G g G^T for the 6x3 G of the
 * points {0, +-1, +-2, inf} in the staging order [C/64][C/4][36][64][4] f32
 * (robomanipbaselines_amd.kernels.pack_winograd4_f32).  f32 MFMA products, f32 accumulation. */
int rmbx_conv3x3_winograd4_f32(const float* in, const float* u_packed, const float* bias,
                               const float* residual, float* out, int N, int H, int W, int C, int relu,
                               void* stream);
/* ResNet stem on a 2x2 space-to-depth image: in [N][Hs][Ws][16] bf16 (channel (dy*2+dx)*3+c,
 * 12..15 zero; rmbx_render policy_dtype 2 writes this layout), weight packed [Cout][4][4][16] bf16
 * (the 7x7 / stride-2 / pad-3 conv1 re-indexed), out [N][Hs][Ws][Cout] bf16 = relu?(conv + bias).
 * Replaces conv1 -> BN -> ReLU of the backbone's stem (max-pool: rmbx_nhwc_bias_relu_maxpool). */
int rmbx_stem_s2d_conv(const void* in, const void* weight, const float* bias, void* out, int N, int Hs,
                       int Ws, int Cout, int relu, void* stream);
/* The whole stem in one pass: out [N][Hp][Wp][64] bf16 = maxpool3x3s2p1(relu(conv + bias)) with
 * Hp = (Hs-1)/2+1, Wp = (Ws-1)/2+1, Cout = 64, Ws <= 320; same in/weight/bias as
 * rmbx_stem_s2d_conv and bit-identical to rmbx_stem_s2d_conv followed by
 * rmbx_nhwc_bias_relu_maxpool (zero bias), without the full-resolution stem map in HBM.
 * band_rows: pool rows per block (<= 0: chosen from N).  Replaces conv1 -> bn1 -> relu -> maxpool
 * of the backbones' resnet18 (third_party/act [absent]; policy/mlp/MlpPolicy.py:34-39). */
int rmbx_stem_s2d_conv_maxpool(const void* in, const void* weight, const float* bias, void* out, int N,
                               int Hs, int Ws, int band_rows, void* stream);
/* The same fused stem in f32 (the reference's precision): in [N][Hs][Ws][16] f32 (rmbx_render
 * policy_dtype 3; channels 12..15 ignored), weight packed [64][4][4][16] f32, bias f32 [64],
 * out [N][Hp][Wp][64] f32 = maxpool3x3s2p1(relu(conv + bias)); exact f32 products with f32
 * accumulation (v_mfma_f32_32x32x2_f32).  The weight must be a re-indexed 7x7 filter as
 * pack_stem_s2d writes it: the taps ky = 0 / dy = 0 and kx = 0 / dx = 0 (outside the 7x7 window)
 * are zero and are not multiplied.  Replaces the same reference ops as above. */
int rmbx_stem_s2d_conv_maxpool_f32(const float* in, const float* weight, const float* bias, float* out,
                                   int N, int Hs, int Ws, int band_rows, void* stream);
/* The f32 stem on the quantised image (the reference's precision, fewer MFMA cycles): in
 * [N][Hs][Ws][16] u8 (rmbx_render policy_dtype 4: the 8-bit pixel values u, channel
 * (dy*2+dx)*3+c, 12..15 zero); w_planes bf16 [3][64][16 taps][16] = the three exact bf16 pieces
 * (RNE at each level) of W'[co][tap][ch] = W[co][tap][ch] / (255 std[ch % 3]) for the packed
 * filter W of pack_stem_s2d; bias f32 [64] = conv bias - sum over all taps of W mean/std; edge f32
 * [16][16][64] = the mean/std term of the out-of-image taps, indexed by the row mask of ky and the
 * column mask of kx that fall outside the image.  out [N][Hp][Wp][64] f32 =
 * maxpool3x3s2p1(relu(conv(x) + bias)) for x = (u / 255 - mean) / std, the renderer's policy
 * pixels: the piece products are exact and accumulate in f32 (v_mfma_f32_32x32x16_bf16).
 * Replaces the same reference ops as rmbx_stem_s2d_conv_maxpool_f32 plus the image
 * normalisation (RolloutBase.py:479-490, the ACT backbone's ImageNet Normalize). */
int rmbx_stem_s2d_conv_maxpool_u8(const uint8_t* in, const void* w_planes, const float* bias, const float* edge,
                                  float* out, int N, int Hs, int Ws, int band_rows, void* stream);
/* The same stem in the f16 form: w_planes [2 pieces][64][16 taps][16] f16 bits of W / (255 std) * 2^s
 * (hi = f16(x), lo = f16(x - hi); one power of two for the whole bank, max in [2^13, 2^14)) and
 * wscale = 2^-s: the integer pixels times the two pieces on the f16 matrix cores, one accumulator,
 * scaled by wscale before bias_eff / edge (2 MFMAs per tap instead of 3; weights to 2^-22). */
int rmbx_stem_s2d_conv_maxpool_u8h(const uint8_t* in, const void* w_planes, float wscale, const float* bias,
                                   const float* edge, float* out, int N, int Hs, int Ws, int band_rows, void* stream);
/* Multi-head attention forward, bf16: out[b][i][h*64 + d] = sum_j softmax_j(scale * q_i . k_j) v_j[d]
 * over the heads of q/k/v rows [b][row][h*64 .. h*64+63] (row/batch strides in elements, last dim
 * contiguous), f32 softmax and accumulation, head dim 64, Lk <= 320, no mask; out contiguous
 * [B][Lq][heads*64].  Replaces scaled_dot_product_attention inside nn.MultiheadAttention of ACT's
 * transformer (third_party/act transformer.py [absent]; d 512, 8 heads, policy/act/TrainAct.py:46-58). */
int rmbx_attention_bf16(const void* q, const void* k, const void* v, void* out, int B, int heads, int Lq, int Lk,
                        long long q_bstride, int q_rstride, long long k_bstride, int k_rstride, long long v_bstride,
                        int v_rstride, float scale, void* stream);
/* The same attention in f32 (the reference's fp32 policy): q/k/v/out f32 with the layouts and
 * strides above (strides multiples of 4 elements, 16-byte aligned), any Lk; exact f32 products
 * and accumulation (v_mfma_f32_32x32x2_f32), f32 online softmax in the log2 domain. */
int rmbx_attention_f32(const float* q, const float* k, const float* v, float* out, int B, int heads, int Lq, int Lk,
                       long long q_bstride, int q_rstride, long long k_bstride, int k_rstride, long long v_bstride,
                       int v_rstride, float scale, void* stream);
/* fp32-accurate linear layer on the bf16 matrix cores (replaces the fp32 nn.Linear /
 * MultiheadAttention in-projections of ACT's transformer, third_party/act detr/models/transformer.py
 * [absent submodule], run by policy/act/RolloutAct.py in fp32): c[M][N] = relu?(a[M][K] . W^T + bias)
 * with a, c f32 (row strides lda, ldc) and W given as its three bf16 pieces W = W0 + W1 + W2
 * (rmbx_split_bf16x3; plane p, row n at w_planes + p * w_plane_stride + n * ldw elements); a is split
 * the same way in registers and the six piece products with i + j <= 2 are accumulated in f32 (error
 * of the f32 GEMM class).  N % 128 == 0, K % 32 == 0, a and w_planes 16-byte aligned, bias [N] or NULL. */
int rmbx_linear_f32x6(const float* a, long long lda, const void* w_planes, long long ldw, long long w_plane_stride,
                      const float* bias, float* c, long long ldc, int M, int N, int K, int relu, void* stream);
/* The same fp32-accurate bf16x6 products as an implicit-GEMM convolution (replaces the stride-2
 * 3x3 convs and 1x1 downsample convs + FrozenBatchNorm of the fp32 ResNet-18 trunk in ACT's backbone,
 * third_party/act [absent], torchvision resnet18): out[N][Ho][Wo][Cout] = relu?(conv(in) + bias + res)
 * with in NHWC f32 [N][H][W][C], w_planes = rmbx_split_bf16x3 of the weight laid out [Cout][KH][KW][C],
 * res NHWC like out or NULL.  C % 32 == 0, Cout % 128 == 0. */
int rmbx_conv2d_f32x6(const float* in, int N, int H, int W, int C, const void* w_planes, const float* bias,
                      const float* res, float* out, int Cout, int KH, int KW, int stride, int pad, int relu,
                      void* stream);
/* rmbx_linear_f32x6 over `batch` independent problems: item b reads a + b * a_bs, w_planes + b * w_bs
 * and writes c + b * c_bs (element strides; the 36 position GEMMs of the explicit Winograd conv). */
int rmbx_linear_f32x6_batched(const float* a, long long lda, long long a_bs, const void* w_planes, long long ldw,
                              long long w_plane_stride, long long w_bs, const float* bias, float* c, long long ldc,
                              long long c_bs, int batch, int M, int N, int K, int relu, void* stream);
/* Winograd F(4x4, 3x3) transforms of the explicit fp32 Winograd conv (the stride-1 3x3 convs of the
 * 256/512-channel ResNet-18 layers in ACT's backbone, third_party/act [absent]): V[36][T][C] =
 * B^T d B of every 6x6 input window (in NHWC [N][H][W][C], T = N * ceil(H/4) * ceil(W/4) tiles), and
 * out NHWC = relu?(A^T M A + bias + res) from the position GEMM results M[36][T][C]. */
int rmbx_wino4_input_f32(const float* in, int N, int H, int W, int C, float* V, void* stream);
/* rmbx_wino4_input_f32 emitting V in rmbx_linear_f16x3_presplit's A form: V_planes [2][36][T][C] f16
 * bits, each tile's 36 x C values scaled by one power of two (max in [2^13, 2^14)), rinv [T] = the
 * inverse scales (the same for the tile's 36 position rows).  C <= 512. */
int rmbx_wino4_input_split(const float* in, int N, int H, int W, int C, void* V_planes, float* rinv, void* stream);
int rmbx_wino4_output_f32(const float* M, int N, int H, int W, int C, const float* bias, const float* res, float* out,
                          int relu, void* stream);
/* Direct f32 convolution for few input channels (the 3-channel 7x7 / stride-2 stem of the diffusion
 * policy's GroupNorm ResNet-18 encoder, third_party/diffusion_policy [absent]): out NHWC [N][Ho][Wo][Cout]
 * = conv(in NHWC [N][H][W][C], w [Cout][KH][KW][C]) + bias (NULL: none); fixed f32 summation order
 * (deterministic).  Cout % 16 == 0, Cout * KH * KW * C <= 12544. */
int rmbx_conv2d_direct_f32(const float* in, int N, int H, int W, int C, const float* w, const float* bias, float* out,
                           int Cout, int KH, int KW, int stride, int pad, void* stream);
/* planes[p * n + i] = bf16 piece p of x[i], x = x0 + x1 + x2 exactly (round-to-nearest-even at each
 * level): the weight form rmbx_linear_f32x6 reads. */
int rmbx_split_bf16x3(const float* x, void* planes, long long n, void* stream);
/* f16x3 form of the fp32-accurate GEMM (two f16 pieces per operand, three products on the f16
 * matrix cores at the bf16 rate: half the MFMA work of bf16x6, error measured below hipBLASLt's f32
 * GEMM against an f64 product).  rmbx_split_f16x2 packs an f32 weight w [N][K] (contiguous) as
 * planes [2][N][K] f16 bits, hi = f16(w[n] s_n) and lo = f16((w[n] s_n - hi) 2^11), with s_n a power
 * of two putting the row's max |w| in [2^13, 2^14), and scale[n] = 1 / s_n.  rmbx_linear_f16x3,
 * rmbx_linear_f16x3_batched and rmbx_conv2d_f16x3 take the arguments of their f32x6 counterparts
 * plus that scale (w_scale [N], 16-byte aligned for the vector epilogue; batched: item b reads
 * w_scale + b * ws_bs); the activations are split in registers, a block whose |a| max lies outside
 * [2^-6, 2^15] re-runs its tile on a power-of-two-scaled copy (f16's range, handled exactly). */
int rmbx_split_f16x2(const float* w, int N, int K, void* planes, float* scale, void* stream);
int rmbx_linear_f16x3(const float* a, long long lda, const void* w_planes, long long ldw, long long w_plane_stride,
                      const float* w_scale, const float* bias, float* c, long long ldc, int M, int N, int K, int relu,
                      void* stream);
int rmbx_linear_f16x3_batched(const float* a, long long lda, long long a_bs, const void* w_planes, long long ldw,
                              long long w_plane_stride, long long w_bs, const float* w_scale, long long ws_bs,
                              const float* bias, float* c, long long ldc, long long c_bs, int batch, int M, int N,
                              int K, int relu, void* stream);
/* rmbx_linear_f16x3 with the activations already split by their producer (rmbx_add_layernorm_split):
 * a_planes [2][M][K] f16 bits (plane stride a_plane_stride, row stride lda elements, both multiples
 * of 8) with a[m] = a_rinv[m] (hi + lo), hi = f16(a[m] 2^t_m), lo = f16(a[m] 2^t_m - hi), 2^t_m putting
 * the row's max |a| in [2^13, 2^14) and a_rinv[m] = 2^-t_m.  Both operands move by LDS-DMA, no split
 * or range pass in the GEMM.  c = relu?(a . w^T + bias + res) (bias / res nullable, res [M][ldc]);
 * N % 128 == 0, K % 32 == 0, 16-byte aligned operands, ldc % 4 == 0.  Replaces the same nn.Linear
 * call sites as rmbx_linear_f16x3 (ACT transformer in-projections and FFN, third_party/act). */
int rmbx_linear_f16x3_presplit(const void* a_planes, long long lda, long long a_plane_stride, const float* a_rinv,
                               const void* w_planes, long long ldw, long long w_plane_stride, const float* w_scale,
                               const float* bias, const float* res, float* c, long long ldc, int M, int N, int K,
                               int relu, void* stream);
/* rmbx_linear_f16x3_presplit whose outputs c = relu?(a . w^T + bias) leave in the same pre-split
 * form (the next GEMM's A): out_planes [2][M][ldo] f16 bits (plane stride out_plane_stride), row m
 * scaled by 2^u_m with B_m (1 + 2^-10) in [2^13, 2^14), B_m = a_norm[m] w_norm_max + b_abs_max an
 * upper bound of the row's |c| (a_norm: upper bounds of the A rows' 2-norms, rmbx_add_layernorm_split;
 * w_norm_max >= max_n |w_n|_2, b_abs_max >= max |bias|), out_rinv[m] = 2^-u_m.  Replaces ACT's FFN
 * first Linear + ReLU (its output only feeds the second Linear).  ldo and out_plane_stride % 8 == 0,
 * 16-byte aligned operands. */
int rmbx_linear_f16x3_presplit_split(const void* a_planes, long long lda, long long a_plane_stride, const float* a_rinv,
                                     const float* a_norm, const void* w_planes, long long ldw, long long w_plane_stride,
                                     const float* w_scale, float w_norm_max, float b_abs_max, const float* bias,
                                     int relu, void* out_planes, long long ldo, long long out_plane_stride,
                                     float* out_rinv, int M, int N, int K, void* stream);
/* rmbx_linear_f16x3_presplit over `batch` items: item b reads a_planes + b a_bs, a_rinv + b r_bs,
 * w_planes + b w_bs, w_scale + b ws_bs and writes c + b c_bs (bias shared, no residual).  The 36
 * Winograd position GEMMs of rmbx_wino4_input_split's output. */
int rmbx_linear_f16x3_presplit_batched(const void* a_planes, long long lda, long long a_plane_stride, long long a_bs,
                                       const float* a_rinv, long long r_bs, const void* w_planes, long long ldw,
                                       long long w_plane_stride, long long w_bs, const float* w_scale, long long ws_bs,
                                       const float* bias, float* c, long long ldc, long long c_bs, int batch, int M,
                                       int N, int K, int relu, void* stream);
/* 3x3 / stride-1 / pad-1 rmbx_conv2d_f16x3 with each input pixel split once per output tile: the
 * block stages the input patch of its 16 x 16 (Cout % 128 == 0) or 16 x 32 output tile for one
 * 32-channel chunk as two f16 pieces in LDS, scaled per (tile, chunk) by a power of two, and all
 * nine taps read it.  w_planes / w_scale: rmbx_split_f16x2 of the [Cout][3][3][C] filter (plane
 * stride w_plane_stride elements); C % 32 == 0, Cout % 64 == 0; res / bias nullable; NHWC. */
int rmbx_conv3x3_f16x3_patch(const float* in, int N, int H, int W, int C, const void* w_planes,
                             long long w_plane_stride, const float* w_scale, const float* bias, const float* res,
                             float* out, int Cout, int relu, void* stream);
int rmbx_conv2d_f16x3(const float* in, int N, int H, int W, int C, const void* w_planes, const float* w_scale,
                      const float* bias, const float* res, float* out, int Cout, int KH, int KW, int stride, int pad,
                      int relu, void* stream);
/* rmbx_attention_f32 with fp32-accurate products on the bf16 matrix cores: Q, K, V and the softmax
 * probabilities split into three bf16 pieces, six piece products per product accumulated in f32 (the
 * rmbx_linear_f32x6 scheme); same layouts, strides and output as rmbx_attention_f32. */
int rmbx_attention_f32x6(const float* q, const float* k, const float* v, float* out, int B, int heads, int Lq, int Lk,
                         long long q_bstride, int q_rstride, long long k_bstride, int k_rstride, long long v_bstride,
                         int v_rstride, float scale, void* stream);
/* rmbx_attention_f32 with fp32-accurate products in the f16x3 form (rmbx_linear_f16x3's scheme): K, V
 * split as h + 2^-11 l, Q and the probabilities (scaled by 2^14) as h + l, three f16 piece products per
 * product accumulated in f32.  A block (one head of one batch item, up to 160 queries) whose |q|, |k|
 * or |v| reaches 2^15, or with a head dimension whose max |v| lies in (0, 2^-6), is re-run on the
 * rmbx_attention_f32x6 kernel.  redo: int32 workspace of at least B * heads * ceil(Lq / 32) entries
 * (one flag per block, written here).  Replaces the same call site as rmbx_attention_f32. */
int rmbx_attention_f16x3(const float* q, const float* k, const float* v, float* out, int* redo, int B, int heads,
                         int Lq, int Lk, long long q_bstride, int q_rstride, long long k_bstride, int k_rstride,
                         long long v_bstride, int v_rstride, float scale, void* stream);
/* Residual add + LayerNorm over the last dim of [rows][D] rows (D <= 2048, multiple of 8 bf16 / 4
 * f32): out = LayerNorm(rnd(x + r)) * weight + bias (f32 weight/bias), r optional (NULL); replaces
 * the add + nn.LayerNorm pair of the ACT transformer's post-norm layers (third_party/act). */
/* GroupNorm(groups, C) over x [B][C][T] f32 with the affine (weight, bias [C]), then Mish when
 * mish & 1 (the DiffusionPolicy / DP3 UNet's Conv1dBlock: policy/diffusion/unet1d.py); mish & 2:
 * x is laid out [B][T][C] (the conv GEMM's rows; out is [B][C][T] either way).  out may alias x
 * only without bit 1. */
int rmbx_groupnorm_act(const float* x, const float* weight, const float* bias, float* out, int B, int C, int T,
                       int groups, float eps, int mish, void* stream);
int rmbx_add_layernorm(const void* x, const void* r, const float* weight, const float* bias, void* out,
                       int rows, int D, float eps, int dtype, void* stream);
/* rmbx_add_layernorm that also writes out_pos = rnd(out + pos[row % pos_rows]) (pos [pos_rows][D] in
 * the storage dtype): the `src + pos` / `tgt + query_pos` query input of the next attention block
 * of ACT's post-norm transformer layers, fused into the LayerNorm pass (out_pos NULL: plain). */
int rmbx_add_layernorm_pos(const void* x, const void* r, const float* weight, const float* bias, void* out,
                           const void* pos, int pos_rows, void* out_pos, int rows, int D, float eps, int dtype,
                           void* stream);
/* f32 rmbx_add_layernorm_pos that also emits its outputs in rmbx_linear_f16x3_presplit's A form:
 * y = LayerNorm(rnd(x + r)) (out f32, nullable), y_planes [2][rows][D] + y_rinv [rows] (nullable
 * together), y_norm [rows] (nullable) an upper bound of each row's |y|_2 (the f32 norm times
 * 1 + 2^-12; rmbx_linear_f16x3_presplit_split bounds the next GEMM's outputs with it), y +
 * pos[row % pos_rows] (out_pos f32 and pos_planes + pos_rinv, each nullable; pos needed if either
 * is set); every row's values from that row alone (batch-invariant).  D % 4 == 0, 8-byte aligned
 * planes. */
int rmbx_add_layernorm_split(const float* x, const float* r, const float* weight, const float* bias, float* out,
                             void* y_planes, float* y_rinv, float* y_norm, const float* pos, int pos_rows,
                             float* out_pos, void* pos_planes, float* pos_rinv, int rows, int D, float eps,
                             void* stream);
/* out [N][Ho][Wo][C] = maxpool3x3s2p1(relu(rnd(x + bias))), Ho = (H-1)/2+1, Wo = (W-1)/2+1. */
int rmbx_nhwc_bias_relu_maxpool(const void* x, const float* bias, void* out, int N, int H, int W,
                                int C, int dtype, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Diffusion-policy sampler steps, batched over envs (all tensors f32 device, n elements).
 * Replace one `noise_scheduler.step(model_output, t, sample).prev_sample` of the reference's
 * conditional_sample loop (diffusion_policy / 3D-Diffusion-Policy submodules, absent; schedulers
 * from diffusers==0.11.1, pyproject.toml:69), called from
 * policy/diffusion_policy/RolloutDiffusionPolicy.py:66-87 (DDPMScheduler,
 * TrainDiffusionPolicy.py:130-138) and policy/diffusion_policy_3d/RolloutDiffusionPolicy3d.py:83-101
 * (DDIMScheduler, TrainDiffusionPolicy3d.py:203-211).  `coeffs` is a HOST array of per-timestep
 * f32 scalars computed as the scheduler computes them (robomanipbaselines_amd/policy/diffusion/
 * schedulers.py); element arithmetic is f32 in the scheduler's order, no contraction.
 *
 * DDPM (epsilon, clip_sample, fixed_small): coeffs = {sqrt(1-acp_t), 1/sqrt(acp_t), x0 coeff,
 *   x_t coeff, sigma_t, t > 0}; noise [n] is read only when t > 0.
 * DDIM (eta 0, prediction "sample", clip_sample): coeffs = {sqrt(acp_prev),
 *   sqrt(1-acp_prev), sqrt(acp_t), 1/sqrt(1-acp_t)}; eps_mode 0 = diffusers 0.11.1 direction
 *   term (the model output), 1 = epsilon re-derived from the unclipped x0 (later releases).
 * ------------------------------------------------------------------------------------------- */
int rmbx_ddpm_step(const float* model_output, const float* sample, const float* noise,
                   float* prev_sample, size_t n, const float* coeffs, void* stream);
int rmbx_ddim_step(const float* model_output, const float* sample, float* prev_sample, size_t n,
                   const float* coeffs, int eps_mode, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Policy-input image preprocessing, batched over envs.
 * rmbx_resize_crop_u8: src u8 [n][H][W][C] (renderer frames) -> dst [n][C][ch][cw] (f32 dtype 0 /
 * bf16 dtype 1) = (v * (1/255)) * a + b, v = cv2.resize(src, (rw, rh), INTER_LINEAR)[y0+y, x0+x];
 * dst_dtype 2 writes v itself as u8 [n][ch][cw][C] (the resized frame).
 * Replaces RolloutDiffusionPolicy.get_images (policy/diffusion_policy/RolloutDiffusionPolicy.py:
 * 107-138: resize, ToDtype(scale), * 2 - 1) plus the obs encoder's eval centre crop.
 * rmbx_resize_f32: cv2.resize of f32 [n][H][W] depth to [n][rh][rw]
 * (RolloutDiffusionPolicy3d.py:138-145).
 * ------------------------------------------------------------------------------------------- */
int rmbx_resize_crop_u8(const uint8_t* src, int n_env, int H, int W, int C, int rh, int rw, int y0,
                        int x0, int ch, int cw, float a, float b, void* dst, int dst_dtype,
                        void* stream);
int rmbx_resize_f32(const float* src, float* dst, int n_env, int H, int W, int rh, int rw,
                    void* stream);

/* ---------------------------------------------------------------------------------------------
 * 3D-diffusion-policy point-cloud observation, batched (one workgroup per env).
 * Replaces RolloutDiffusionPolicy3d.get_pointcloud (policy/diffusion_policy_3d/
 * RolloutDiffusionPolicy3d.py:132-160) after the image resize: convert_depth_image_to_pointcloud
 * (common/utils/VisionUtils.py:55-87), crop_pointcloud_bb (common/utils/Vision3dUtils.py:6-14),
 * downsample_pointcloud_fps (Vision3dUtils.py:17-25, pytorch3d FPS from index 0) and
 * normalize_data (common/utils/DataUtils.py:9-24).
 * depth f32 [n][H][W], rgb u8 [n][H][W][3] (H*W <= 8192); focal_scaling = (1 / tan(fovy/2)) * H / 2;
 * min_bound / max_bound f64[3] host (NULL = no bound); norm_type 0 gaussian ((x - a) / b) or
 * 1 limits (b * (x - a) + c), a/b/c f64[6] host; out f32 [n][K][6] normalised (x, y, z, r, g, b),
 * raw f64 [n][K][6] optional (before normalisation), count i32 [n] = points after the crop.
 * ------------------------------------------------------------------------------------------- */
int rmbx_pointcloud_fps(const float* depth, const uint8_t* rgb, int n_env, int H, int W,
                        double focal_scaling, const double* min_bound, const double* max_bound,
                        int K, int norm_type, const double* norm_a, const double* norm_b,
                        const double* norm_c, float* out, double* raw, int32_t* count,
                        void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RMBX_H_ */
