"""ORACLE — test infrastructure only.  numpy restatement of the reference's DataKey routing for
the single UR5e arm + gripper (one ArmManager, eef_idx 0), the checker of rmbx_motion_state /
rmbx_motion_command:

* state:   RolloutBase.get_state (common/base/RolloutBase.py:463-473) -> MotionManager.get_data
           (common/manager/MotionManager.py:41-130) -> ArmManager.get_eef_pose_from_joint_pos /
           get_command_data (common/body/ArmManager.py:161-186)
* command: RolloutBase.set_command_data (RolloutBase.py:496-509) -> MotionManager.set_command_data
           (MotionManager.py:25-39) -> ArmManager.set_command_data (ArmManager.py:88-159)

The SE3 <-> pose helpers restate the Eigen routines pinocchio binds (MathUtils.py:27-46):
Eigen's matrix -> quaternion, Quaternion::toRotationMatrix (of the unnormalised quaternion, as
pin.SE3(pin.Quaternion(w, x, y, z), t) does) and pin.rpy.rpyToMatrix as the AngleAxis product
z * y * x.  The routing logic is pinned by tests/golden/motion.npz, minted by running the
reference's own RolloutBase / MotionManager / ArmManager (tools/gen_golden.py gen_motion); the
pinocchio / Eigen arithmetic under it is this restatement (pinocchio is absent: unpinned)."""

import numpy as np

from . import arm_ik

DIMS = {"measured_joint_pos": 7, "measured_joint_vel": 7, "measured_gripper_joint_pos": 1,
        "measured_eef_pose": 7, "measured_eef_wrench": 6, "command_joint_pos": 7,
        "command_joint_pos_rel": 7, "command_gripper_joint_pos": 1, "command_eef_pose": 7,
        "command_eef_pose_rel": 6}


def quat_from_mat(m):
    """Eigen's QuaternionBase::operator=(MatrixBase) -> (w, x, y, z)."""
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0.0:
        t = np.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        return np.array([w, (m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t])
    i = 0
    if m[1, 1] > m[0, 0]:
        i = 1
    if m[2, 2] > m[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
    v = np.zeros(3)
    v[i] = 0.5 * t
    t = 0.5 / t
    w = (m[k, j] - m[j, k]) * t
    v[j] = (m[j, i] + m[i, j]) * t
    v[k] = (m[k, i] + m[i, k]) * t
    return np.array([w, v[0], v[1], v[2]])


def mat_from_quat(w, x, y, z):
    """Eigen's QuaternionBase::toRotationMatrix (no normalisation)."""
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1.0 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1.0 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1.0 - (txx + tyy)]])


def quat_mul(a, b):
    """Eigen's quaternion product a * b, (w, x, y, z)."""
    return np.array([a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                     a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                     a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3],
                     a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1]])


def rpy_to_mat(r, p, y):
    """pin.rpy.rpyToMatrix: (AngleAxis(y, z) * AngleAxis(p, y) * AngleAxis(r, x)).toRotationMatrix()."""
    qz = np.array([np.cos(0.5 * y), 0.0, 0.0, np.sin(0.5 * y)])
    qy = np.array([np.cos(0.5 * p), 0.0, np.sin(0.5 * p), 0.0])
    qx = np.array([np.cos(0.5 * r), np.sin(0.5 * r), 0.0, 0.0])
    q = quat_mul(quat_mul(qz, qy), qx)
    return mat_from_quat(*q)


def pose_from_se3(R, p):
    """MathUtils.get_pose_from_se3 (:27-31): (tx, ty, tz, qw, qx, qy, qz)."""
    return np.concatenate([p, quat_from_mat(R)])


class ArmCommand:
    """ArmManager's command state: arm_joint_pos, gripper_joint_pos, target_se3 (ArmManager.py:75-86)."""

    def __init__(self, placement, q0, g0=0.0):
        self.P = placement
        self.q = np.array(q0, dtype=np.float64)
        self.g = np.array([g0], dtype=np.float64)
        self.R, self.p = arm_ik.fk(placement, self.q)[-1]

    def copy(self):
        c = object.__new__(ArmCommand)
        c.P, c.q, c.g, c.R, c.p = self.P, self.q.copy(), self.g.copy(), self.R.copy(), self.p.copy()
        return c


def get_raw_state(keys, joint_pos, joint_vel, wrench, arm):
    """MotionManager.get_data of every key, concatenated (RolloutBase.py:467-472)."""
    out = []
    for key in keys:
        if key == "measured_joint_pos":
            out.append(joint_pos)
        elif key == "measured_joint_vel":
            out.append(joint_vel)
        elif key == "measured_gripper_joint_pos":
            out.append(joint_pos[6:7])
        elif key == "measured_eef_pose":
            R, p = arm_ik.fk(arm.P, joint_pos[:6])[-1]
            out.append(pose_from_se3(R, p))
        elif key == "measured_eef_wrench":
            out.append(wrench)
        elif key == "command_joint_pos":
            out.append(np.concatenate([arm.q, arm.g]))
        elif key == "command_gripper_joint_pos":
            out.append(arm.g.copy())
        elif key == "command_eef_pose":
            out.append(pose_from_se3(arm.R, arm.p))
        else:
            raise ValueError(f"invalid state key {key}")
    return np.concatenate(out) if out else np.zeros(0)


def set_command(keys, action, is_skip, arm, glo, ghi):
    """RolloutBase.set_command_data -> ArmManager.set_command_data, keys in order."""
    i = 0
    for key in keys:
        a = action[i:i + DIMS[key]]
        if key in ("command_joint_pos", "command_joint_pos_rel"):
            if key == "command_joint_pos":
                q, g = a[:6].copy(), a[6:7].copy()
            else:
                q, g = arm.q.copy(), arm.g.copy()
                if not is_skip:
                    q += a[:6]
                    g += a[6:7]
            arm.q = q
            arm.R, arm.p = arm_ik.fk(arm.P, q)[-1]
            arm.g = np.clip(g, glo, ghi)
        elif key == "command_gripper_joint_pos":
            arm.g = np.clip(a[0:1], glo, ghi)
        elif key == "command_eef_pose":
            arm.p, arm.R = a[:3].copy(), mat_from_quat(*a[3:7])
            arm.q = arm_ik.ik_step(arm.P, arm.q, arm.R, arm.p)
        elif key == "command_eef_pose_rel":
            # ArmManager.py:115-119 does not forward is_skip: composes on every call
            Rr = rpy_to_mat(*a[3:6])
            arm.p, arm.R = arm.p + arm.R @ a[:3], arm.R @ Rr
            arm.q = arm_ik.ik_step(arm.P, arm.q, arm.R, arm.p)
        else:
            raise ValueError(f"invalid command key {key}")
        i += DIMS[key]
    return np.concatenate([arm.q, arm.g])
