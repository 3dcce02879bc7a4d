"""ORACLE — test infrastructure only (imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py; never by the product package).

numpy restatements of the reference's per-env hot-path glue, one function per reference
function, each citing the reference file:line it follows (paths relative to
robo_manip_baselines/ in yusuke1127/RoboManipBaselines @2.0.0).  They are pinned against the
golden vectors in tests/golden/ that tools/gen_golden.py minted by running the reference's own
code (see tests/test_oracle_golden.py).
"""

import numpy as np


# ------------------------------------------------------------------------------------------
# policy/act/RolloutAct.py:68-101 + common/utils/DataUtils.py:26-40
# ------------------------------------------------------------------------------------------
def denormalize(data, stats):
    """common/utils/DataUtils.py:26-40"""
    norm_type = stats["norm_config"]["type"] if "norm_config" in stats else "gaussian"
    if norm_type == "gaussian":
        return stats["std"] * data + stats["mean"]
    cfg = stats["norm_config"]
    scale = stats["range"] / (cfg["out_max"] - cfg["out_min"])
    return scale * (data - cfg["out_min"]) + stats["min"]


def normalize(data, stats):
    """common/utils/DataUtils.py:9-24"""
    norm_type = stats["norm_config"]["type"] if "norm_config" in stats else "gaussian"
    if norm_type == "gaussian":
        return (data - stats["mean"]) / stats["std"]
    cfg = stats["norm_config"]
    scale = (cfg["out_max"] - cfg["out_min"]) / stats["range"]
    return scale * (data - stats["min"]) + cfg["out_min"]


class ActEnsembleOracle:
    """Single-env restatement of RolloutAct.infer_policy's action bookkeeping
    (policy/act/RolloutAct.py:62-101)."""

    def __init__(self, chunk_size, stats, temporal_ensemble=True, k=0.01):
        self.chunk_size = chunk_size
        self.stats = stats
        self.te = temporal_ensemble
        self.k = k
        self.buf = []
        self.hist = []

    def step(self, chunk_fn):
        """chunk_fn() -> f32 [chunk, A]; called only when the reference would run the policy."""
        if self.te or len(self.buf) == 0:
            self.buf = list(np.asarray(chunk_fn()).astype(np.float64))
            if self.te:
                self.hist.append(self.buf)
                if len(self.hist) > self.chunk_size:
                    self.hist.pop(0)
        if not self.te:
            action = self.buf.pop(0)
        else:
            n = len(self.hist)
            w = np.exp(-self.k * np.arange(n))
            w = w / w.sum()
            action = np.zeros(len(self.hist[0][0]))
            for j, h in enumerate(reversed(self.hist)):
                action += w[::-1][j] * h[j]
        return denormalize(action, self.stats)


# ------------------------------------------------------------------------------------------
# envs/mujoco/ur5e/MujocoUR5eCableEnv.py:48-105
# ------------------------------------------------------------------------------------------
def cable_reward(cable, end, p1, p2):
    """_get_reward for one env: cable f64 [25, 3], end/p1/p2 f64 [3]."""
    z_thre = p1[2] + 0.01
    if cable[:, 2].max() > z_thre:
        return 0.0
    if end[0] < p2[0] or end[1] > p1[1] - 0.05:
        return 0.0
    pd = p2[:2] - p1[:2]

    def ccw(a, b, c):
        return (c[1] - a[1]) * (b[0] - a[0]) > (b[1] - a[1]) * (c[0] - a[0])

    for i in range(len(cable) - 1):
        a, b = cable[i, :2], cable[i + 1, :2]
        if (ccw(a, p1[:2], p2[:2]) != ccw(b, p1[:2], p2[:2])) and (
            ccw(a, b, p1[:2]) != ccw(a, b, p2[:2])
        ):
            cd = b - a
            if pd[0] * cd[1] - pd[1] * cd[0] > 0:
                return 1.0
    return 0.0


# ------------------------------------------------------------------------------------------
# envs/mujoco/ur5e/MujocoUR5eEnvBase.py:78-119
# ------------------------------------------------------------------------------------------
def quat2mat(q):
    """mju_quat2Mat (mujoco==3.1.6 engine_util_spatial.c, external): row-major 3x3."""
    q = np.asarray(q, dtype=np.float64)
    if q[0] == 1 and q[1] == 0 and q[2] == 0 and q[3] == 0:
        return np.eye(3)
    q00, q01, q02, q03 = q[0] * q[0], q[0] * q[1], q[0] * q[2], q[0] * q[3]
    q11, q12, q13 = q[1] * q[1], q[1] * q[2], q[1] * q[3]
    q22, q23, q33 = q[2] * q[2], q[2] * q[3], q[3] * q[3]
    return np.array([[q00 + q11 - q22 - q33, 2 * (q12 - q03), 2 * (q13 + q02)],
                     [2 * (q12 + q03), q00 - q11 + q22 - q33, 2 * (q23 - q01)],
                     [2 * (q13 - q02), 2 * (q23 + q01), q00 - q11 - q22 + q33]])


def insert_reward(peg_pos, hole_pos, peg_quat):
    """envs/mujoco/ur5e/MujocoUR5eInsertEnv.py:43-63 (_get_reward), with the peg's xmat from its
    xquat (the engine keeps body orientations as quaternions)."""
    peg_z_axis = quat2mat(peg_quat)[:, 2]
    world_z_axis = np.array([0.0, 0.0, -1.0])
    xy_thre = 0.012
    z_thre = hole_pos[2] + 0.05
    tilt_thre = 10
    if (np.max(np.abs(peg_pos[:2] - hole_pos[:2])) < xy_thre) and (peg_pos[2] < z_thre) and (
            np.dot(peg_z_axis, world_z_axis) > np.cos(np.deg2rad(tilt_thre))):
        return 1.0
    return 0.0


def door_reward(gripper_pos, handle_pos, door_angle):
    """envs/mujoco/ur5e/MujocoUR5eDoorEnv.py:52-67 (_get_reward)."""
    gripper_handle_dist = np.linalg.norm(gripper_pos - handle_pos)
    gripper_handle_dist_margin = 0.08
    reaching_reward = np.exp(-10.0 * np.max([gripper_handle_dist - gripper_handle_dist_margin, 0.0]))
    door_angle_target = np.deg2rad(-45.0)
    opening_reward = np.clip(door_angle / door_angle_target, 0.0, 1.0)
    if opening_reward >= 1.0:
        reaching_reward = 1.0
    return 0.5 * (reaching_reward + opening_reward)


def ur5e_obs(arm_qpos, arm_qvel, grip_qpos, force, torque):
    g = np.rad2deg(np.asarray(grip_qpos, np.float64).mean(keepdims=True)) / 45.0 * 255.0
    return (
        np.concatenate([arm_qpos, g]),
        np.concatenate([arm_qvel, np.zeros(1)]),
        np.concatenate([force, torque]),
    )


# ------------------------------------------------------------------------------------------
# envs/mujoco/MujocoEnvBase.py:122-125
# ------------------------------------------------------------------------------------------
def depth_linearize(zbuf, extent, znear, zfar):
    near = znear * extent
    far = zfar * extent
    return near / (1 - zbuf * (1 - near / far))


# ------------------------------------------------------------------------------------------
# common/utils/VisionUtils.py:55-87, common/utils/Vision3dUtils.py:6-14
# ------------------------------------------------------------------------------------------
def depth_to_pointcloud(depth, fovy, rgb=None, near_clip=0.0, far_clip=np.inf):
    H, W = depth.shape[:2]
    f = (1.0 / np.tan(np.deg2rad(fovy) / 2.0)) * H / 2.0
    ij = np.stack(np.meshgrid(np.arange(H), np.arange(W), indexing="ij"), -1).reshape(-1, 2)
    ij = ij.astype(np.float32)
    xy = (ij - 0.5 * np.array((H, W), dtype=np.float32)) / f
    d = depth.reshape(-1)
    xy = xy * d[:, None]
    xyz = np.hstack((xy[:, [1, 0]], d[:, None]))
    keep = np.argwhere((near_clip < d) & (d < far_clip))[:, 0]
    xyz = xyz[keep]
    if rgb is None:
        return xyz
    col = (rgb.reshape(-1, 3).astype(np.float32) / 255.0)[keep]
    return xyz, col


def crop_bb(pc, lo=None, hi=None):
    if lo is not None:
        pc = pc[np.all(pc[:, :3] > lo, axis=1)]
    if hi is not None:
        pc = pc[np.all(pc[:, :3] < hi, axis=1)]
    return pc


# ------------------------------------------------------------------------------------------
# Phase schedule: common/base/RolloutBase.py:28-132, PhaseBase.py:19-106,
# PhaseManager.py:20-37, OperationMujocoUR5eCable.py:14-34 (durations), MujocoEnvBase.py:12-13
# ------------------------------------------------------------------------------------------
CABLE_PRE_DURATIONS = (1.0, 0.7, 0.3, 0.5)  # Initial, Reach1, Reach2, Grasp


def phase_schedule(reward_fn, pre_durations=CABLE_PRE_DURATIONS, skip=3, max_duration=30.0,
                   dt=0.004, frame_skip=8, max_steps=100000):
    """Run the single-env schedule; reward_fn(step) -> reward after that step.
    Returns dict(phase[], infer_steps[], success, reward, duration, n_steps)."""
    n_pre = len(pre_durations)
    t = 0.0
    phase, start = 0, 0.0
    ridx, succ_t = 0, None
    phases, infer = [], []
    result = None
    step = 0
    while step < max_steps:
        if phase == n_pre and ridx % skip == 0:
            infer.append(step)
        for _ in range(frame_skip):
            t += dt
        r = reward_fn(step)
        el = t - start
        trans = False
        done = False
        if phase < n_pre:
            trans = el > pre_durations[phase]
        elif phase == n_pre:
            ridx += 1
            if r >= 1.0 and succ_t is None:
                succ_t = el
            if succ_t is not None:
                trans = el > succ_t + 1.0
            else:
                trans = el > max_duration
            if trans:
                result = (bool(r >= 1.0), float(r), el)
        else:
            done = True
        if trans:
            phase += 1
            start = t
            if phase == n_pre:
                ridx, succ_t = 0, None
        phases.append(phase)
        step += 1
        if done:
            break
    return dict(phase=np.array(phases), infer_steps=np.array(infer), result=result, n_steps=step)


def cabinet_reward(hinge_qpos, slide_qpos, target_task=None):
    """envs/mujoco/ur5e/MujocoUR5eCabinetEnv.py:57-73 (_get_reward)."""
    hinge_success = hinge_qpos > np.deg2rad(120.0)
    slide_success = slide_qpos > 0.12
    if target_task is None:
        return 1.0 if hinge_success or slide_success else 0.0
    if target_task == "hinge":
        return 1.0 if hinge_success else 0.0
    if target_task == "slide":
        return 1.0 if slide_success else 0.0
    raise ValueError(f"Invalid target task: {target_task}")


def toolbox_reward(toolbox_pos, mat_pos):
    """envs/mujoco/ur5e/MujocoUR5eToolboxEnv.py:46-57 (_get_reward)."""
    xy_thre = 0.03
    z_thre = mat_pos[2] + 0.005
    if (np.max(np.abs(toolbox_pos[:2] - mat_pos[:2])) < xy_thre) and (toolbox_pos[2] < z_thre):
        return 1.0
    return 0.0


def _finite(v):
    return np.isfinite(v)


def point_in_polygon_mpl(xy, tx, ty):
    """matplotlib Path(xy).contains_point((tx, ty)) for a code-less path, radius 0, identity
    transform ([ext] matplotlib 3.x src/_path.h point_in_path_impl, src/path_converters.h
    PathNanRemover fast path, agg conv_transform): the identity affine maps a vertex to
    (x*1 + y*0 + 0, x*0 + y*1 + 0), so a non-finite coordinate poisons both; non-finite
    vertices are dropped and the next finite one opens a new subpath (MOVETO); each subpath is
    tested with the crossing-number rule and closed back to its start only when the path ends
    (a subpath cut by a MOVETO is left open); the point is inside if any subpath says so."""
    if not (_finite(tx) and _finite(ty)):
        return False
    verts = []
    for x, y in xy:
        x, y = float(x), float(y)
        X = x * 1.0 + y * 0.0 + 0.0
        Y = x * 0.0 + y * 1.0 + 0.0
        verts.append((X, Y))
    # vertex stream after the NaN remover: (code, x, y); code 1 MOVETO, 2 LINETO, 0 STOP
    stream = []
    first = True
    pending_move = False
    for X, Y in verts:
        if not (_finite(X) and _finite(Y)):
            pending_move = True
            continue
        stream.append((1 if (first or pending_move) else 2, X, Y))
        first = False
        pending_move = False
    stream.append((0, 0.0, 0.0))
    pos = 0

    def nxt():
        nonlocal pos
        c = stream[pos]
        pos += 1
        return c

    inside = False
    code = -1
    x = y = 0.0
    while True:
        if code != 1:
            code, x, y = nxt()
            if code == 0:
                break
        sx = vtx0 = vtx1 = x
        sy = vty0 = vty1 = y
        yflag0 = vty0 >= ty
        flag = False
        while True:
            code, x, y = nxt()
            if code == 0:
                x, y = sx, sy
            elif code == 1:
                break
            yflag1 = vty1 >= ty
            if yflag0 != yflag1:
                if ((vty1 - ty) * (vtx0 - vtx1) >= (vtx1 - tx) * (vty0 - vty1)) == yflag1:
                    flag = not flag
            yflag0 = yflag1
            vtx0, vty0 = vtx1, vty1
            vtx1, vty1 = x, y
            if code == 0:
                break
        yflag1 = vty1 >= ty
        if yflag0 != yflag1:
            if ((vty1 - ty) * (vtx0 - vtx1) >= (vtx1 - tx) * (vty0 - vty1)) == yflag1:
                flag = not flag
        inside = inside or flag
        if inside or code == 0:
            break
    return inside


def ring_reward(ring_pos, pole_pos):
    """envs/mujoco/ur5e/MujocoUR5eRingEnv.py:46-75 (_get_reward): 0 if the highest ring body
    is above pole z + 0.08 (numpy max: NaN never compares above), else 1 iff the pole's xy lies
    in the polygon of the ring bodies' xy closed by repeating the first (matplotlib Path)."""
    z_thre = pole_pos[2] + 0.08
    if np.max(ring_pos[:, 2]) > z_thre:
        return 0.0
    xy = np.vstack([ring_pos[:, :2], ring_pos[:1, :2]])
    return 1.0 if point_in_polygon_mpl(xy, pole_pos[0], pole_pos[1]) else 0.0
