"""ORACLE — test infrastructure only.  numpy restatement of the reference's arm FK / one-step
damped-least-squares IK (common/body/ArmManager.py:213-243) and of the Pinocchio functions it
calls (pin.forwardKinematics, pin.log, pin.computeJointJacobian in the LOCAL joint frame,
pin.Jlog6, pin.integrate for revolute joints).  Pinocchio is absent from this image: parity
against the real library is UNPINNED; this is the checker for the HIP IK kernel.
Motion vectors are Pinocchio-ordered [linear; angular]."""

import numpy as np


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def rotz(q):
    c, s = np.cos(q), np.sin(q)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def fk(placement, q):
    """Frames (R, p) of joints 1..6: oMi = oMi-1 * placement_i * Rz(q_i)."""
    R, p = np.eye(3), np.zeros(3)
    frames = []
    for k in range(6):
        Pr, Pp = placement[k, :9].reshape(3, 3), placement[k, 9:12]
        p = p + R @ Pp
        R = R @ Pr @ rotz(q[k])
        frames.append((R.copy(), p.copy()))
    return frames


TAYLOR3 = np.finfo(np.float64).eps ** 0.25  # Pinocchio's TaylorSeriesExpansion precision<3>()


def log3(R):
    """pin.log3 (spatial/log.hxx [ext]): within 1e-2 of pi the axis comes from the diagonal
    (the antisymmetric part has lost its digits there), signs from R - R^T; below eps^(1/4) the
    factor theta / sin(theta) is 1."""
    tr = np.trace(R)
    if tr >= 3.0:
        t = 0.0
    elif tr <= -1.0:
        t = np.pi
    else:
        t = np.arccos((tr - 1.0) / 2.0)
    if t >= np.pi - 1e-2:
        cphi = np.cos(t - np.pi)
        beta = t * t / (1.0 + cphi)
        tmp = (np.diag(R) + cphi) * beta
        sgn = np.array([1.0 if R[2, 1] > R[1, 2] else -1.0, 1.0 if R[0, 2] > R[2, 0] else -1.0,
                        1.0 if R[1, 0] > R[0, 1] else -1.0])
        return sgn * np.where(tmp > 0, np.sqrt(np.maximum(tmp, 0.0)), 0.0), t
    f = (t / np.sin(t) if t > TAYLOR3 else 1.0) / 2.0
    return f * np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]), t


def log6(R, p):
    w, t = log3(R)
    if t < TAYLOR3:
        alpha, beta = 1 - t * t / 12 - t ** 4 / 720, 1.0 / 12 + t * t / 720
    else:
        st, ct = np.sin(t), np.cos(t)
        alpha = t * st / (2 * (1 - ct))
        beta = 1 / (t * t) - st / (2 * t * (1 - ct))
    v = alpha * p - 0.5 * np.cross(w, p) + beta * np.dot(w, p) * w
    return np.concatenate([v, w])


def jlog3(t, w):
    if t < TAYLOR3:
        return np.eye(3) + 0.5 * skew(w)
    st, ct = np.sin(t), np.cos(t)
    st1mct = st / (1 - ct)
    return 0.5 * t * st1mct * np.eye(3) + (1 / (t * t) - 0.5 * st1mct / t) * np.outer(w, w) + 0.5 * skew(w)


def jlog6(R, p):
    w, t = log3(R)
    A = jlog3(t, w)
    if t < TAYLOR3:
        beta, bdot = 1.0 / 12 + t * t / 720, 1.0 / 360
    else:
        st, ct = np.sin(t), np.cos(t)
        tinv = 1 / t
        t2inv = tinv * tinv
        inv_2_2ct = 1 / (2 * (1 - ct))
        beta = t2inv - st * tinv * inv_2_2ct
        bdot = -2 * t2inv * t2inv + (1 + st * tinv) * t2inv * inv_2_2ct
    wTp = np.dot(w, p)
    v3 = (bdot * wTp) * w - (t * t * bdot + 2 * beta) * p
    C = np.outer(v3, w) + beta * np.outer(w, p) + wTp * beta * np.eye(3) + 0.5 * skew(p)
    B = C @ A
    J = np.zeros((6, 6))
    J[:3, :3] = A
    J[:3, 3:] = B
    J[3:, 3:] = A
    return J


def joint_jacobian_local(frames):
    R6, p6 = frames[-1]
    J = np.zeros((6, 6))
    for k, (Rk, pk) in enumerate(frames):
        wz = Rk[:, 2]
        J[3:, k] = R6.T @ wz
        J[:3, k] = R6.T @ np.cross(pk - p6, wz)
    return J


def ik_step(placement, q, Rt, pt):
    """One ArmManager.inverse_kinematics iteration (ArmManager.py:220-243)."""
    frames = fk(placement, q)
    R6, p6 = frames[-1]
    Re, pe = R6.T @ Rt, R6.T @ (pt - p6)  # current.actInv(target)
    e = log6(Re, pe)
    J = joint_jacobian_local(frames)
    J = -jlog6(Re.T, -Re.T @ pe) @ J  # Jlog6(error.inverse())
    dq = -J.T @ np.linalg.solve(J @ J.T + (e @ e + 1e-6) * np.eye(6), e)
    return q + dq
