"""Arm FK / one-step DLS IK (common/body/ArmManager.py:213-243): the HIP kernels rmbx_arm_fk /
rmbx_arm_ik (through the C ABI) against oracle/arm_ik.py, and the oracle's Pinocchio
restatement against closed-form properties on CPU.

Pinocchio is absent from the image, so the oracle is pinned by properties only (log3 inverts the
Rodrigues exponential over the whole angle range including within 1e-3 of pi; DLS iterations
converge onto reachable targets); parity against the real library is unpinned."""

import numpy as np
import pytest

from oracle import arm_ik


def _placement():
    from robomanipbaselines_amd import model as MD

    return np.ascontiguousarray(MD.load("ur5e_cable")["arm_placement"], dtype=np.float64)


def exp3(w):
    t = np.linalg.norm(w)
    if t == 0:
        return np.eye(3)
    k = arm_ik.skew(w / t)
    return np.eye(3) + np.sin(t) * k + (1 - np.cos(t)) * k @ k


def _axis(rng):
    a = rng.standard_normal(3)
    return a / np.linalg.norm(a)


@pytest.mark.parametrize("delta", [0.5, 1e-2, 5e-3, 1e-3, 1e-5, 1e-7])
def test_log3_inverts_exp3_near_pi(delta):
    rng = np.random.default_rng(int(1 / delta) % 1000)
    for _ in range(64):
        n = _axis(rng)
        t = np.pi - delta
        w, th = arm_ik.log3(exp3(t * n))
        assert abs(th - t) < 1e-7
        # accuracy of the antisymmetric form degrades as 1/sin(theta); the diagonal branch keeps
        # sqrt(eps)-level accuracy right up to pi
        np.testing.assert_allclose(w, t * n, atol=2e-7)


@pytest.mark.parametrize("t", [0.0, 1e-9, 1e-5, 1e-4, 2e-4, 0.3, 2.0])
def test_log3_inverts_exp3_small_and_mid(t):
    rng = np.random.default_rng(5)
    for _ in range(16):
        n = _axis(rng)
        w, _ = arm_ik.log3(exp3(t * n))
        np.testing.assert_allclose(w, t * n, atol=1e-12)


def test_ik_iterations_converge_to_reachable_target():
    P = _placement()
    rng = np.random.default_rng(2)
    for _ in range(16):
        q_goal = rng.uniform(-2.5, 2.5, 6)
        R6, p6 = arm_ik.fk(P, q_goal)[-1]
        q = q_goal + rng.uniform(-0.2, 0.2, 6)
        for _ in range(60):
            q = arm_ik.ik_step(P, q, R6, p6)
        R, p = arm_ik.fk(P, q)[-1]
        np.testing.assert_allclose(p, p6, atol=1e-9)
        np.testing.assert_allclose(R, R6, atol=1e-9)


def _cases(P, n, rng):
    """q, target (R, p) of n envs: near-converged, far, error rotations within [1e-9, 1e-3] of pi,
    tiny error rotations (below the Taylor threshold) and exact targets."""
    q = rng.uniform(-np.pi, np.pi, (n, 6))
    Rt = np.empty((n, 3, 3))
    pt = np.empty((n, 3))
    kinds = np.arange(n) % 6
    for e in range(n):
        R6, p6 = arm_ik.fk(P, q[e])[-1]
        k = kinds[e]
        if k == 0:  # near the target
            Rt[e] = R6 @ exp3(rng.normal(0, 0.05, 3))
            pt[e] = p6 + rng.normal(0, 0.01, 3)
        elif k == 1:  # anywhere
            Rt[e] = exp3(rng.uniform(-np.pi, np.pi) * _axis(rng))
            pt[e] = rng.uniform(-0.6, 0.6, 3) + [0, 0, 0.9]
        elif k in (2, 3):  # rotation error within 1e-3 of pi
            delta = 10 ** rng.uniform(-9, -3)
            Rt[e] = R6 @ exp3((np.pi - delta) * _axis(rng))
            pt[e] = p6 + rng.normal(0, 0.02, 3)
        elif k == 4:  # below the Taylor threshold
            Rt[e] = R6 @ exp3(10 ** rng.uniform(-10, -4.5) * _axis(rng))
            pt[e] = p6 + rng.normal(0, 1e-6, 3)
        else:  # exact
            Rt[e], pt[e] = R6, p6
    return q, Rt, pt


@pytest.mark.gpu
@pytest.mark.parametrize("n_iter", [1, 3])
def test_arm_ik_kernel_matches_oracle(n_iter):
    import torch

    from robomanipbaselines_amd import _native as N

    P = _placement()
    rng = np.random.default_rng(11 + n_iter)
    n = 768
    q, Rt, pt = _cases(P, n, rng)
    dev = "cuda:0"
    # (operands held in locals: a temporary's block would return to the caching allocator before
    # the kernel runs and be reused by the next operand)
    qd, Pd = torch.tensor(q, device=dev), torch.tensor(P, device=dev)
    Rd, pd = torch.tensor(Rt.reshape(n, 9), device=dev), torch.tensor(pt, device=dev)
    N.call("rmbx_arm_ik", N.ptr(Pd), N.ptr(qd), N.ptr(Rd), N.ptr(pd), None, n, n_iter, N.stream_ptr())
    got = qd.cpu().numpy()
    for e in range(n):
        want = q[e]
        for _ in range(n_iter):
            want = arm_ik.ik_step(P, want, Rt[e], pt[e])
        # f64 through a 6x6 damped solve (condition up to ~1e4 at random poses): 1e-8 of the step
        np.testing.assert_allclose(got[e], want, rtol=0, atol=1e-8 * max(1.0, np.abs(want - q[e]).max()),
                                   err_msg=f"env {e} kind {e % 6}")


@pytest.mark.gpu
def test_arm_ik_mask_leaves_inactive_envs():
    import torch

    from robomanipbaselines_amd import _native as N

    P = _placement()
    rng = np.random.default_rng(3)
    n = 130
    q, Rt, pt = _cases(P, n, rng)
    dev = "cuda:0"
    qd, Pd = torch.tensor(q, device=dev), torch.tensor(P, device=dev)
    Rd, pd = torch.tensor(Rt.reshape(n, 9), device=dev), torch.tensor(pt, device=dev)
    mask = torch.tensor(np.arange(n) % 3 != 1, dtype=torch.uint8, device=dev)
    N.call("rmbx_arm_ik", N.ptr(Pd), N.ptr(qd), N.ptr(Rd), N.ptr(pd), N.ptr(mask), n, 1, N.stream_ptr())
    got = qd.cpu().numpy()
    off = np.arange(n) % 3 == 1
    np.testing.assert_array_equal(got[off], q[off])
    assert np.abs(got[~off] - q[~off]).max() > 0


@pytest.mark.gpu
def test_arm_fk_kernel_matches_oracle():
    import torch

    from robomanipbaselines_amd import _native as N

    P = _placement()
    rng = np.random.default_rng(4)
    n = 1000
    q = rng.uniform(-2 * np.pi, 2 * np.pi, (n, 6))
    dev = "cuda:0"
    R = torch.empty((n, 9), dtype=torch.float64, device=dev)
    p = torch.empty((n, 3), dtype=torch.float64, device=dev)
    Pd, qd = torch.tensor(P, device=dev), torch.tensor(q, device=dev)
    N.call("rmbx_arm_fk", N.ptr(Pd), N.ptr(qd), N.ptr(R), N.ptr(p), n, N.stream_ptr())
    R, p = R.cpu().numpy(), p.cpu().numpy()
    for e in range(n):
        R6, p6 = arm_ik.fk(P, q[e])[-1]
        np.testing.assert_allclose(R[e].reshape(3, 3), R6, rtol=0, atol=1e-14)
        np.testing.assert_allclose(p[e], p6, rtol=0, atol=1e-14)


def test_fk_restatement_agrees_with_the_reference_mjcf():
    """Known answer from independent reference data: the oracle's Pinocchio FK runs on the URDF
    chain (envs/assets/common/robots/ur5e/ur5e.urdf, as ArmManager does), MuJoCo on the MJCF
    (ur5e_integrated_body.xml) -- the same arm described twice.  Up to one constant frame offset
    (fixed at the init pose), the wrist_3 frame orientations agree to 1e-9 over random joint
    angles (axes and rotation order pinned); positions agree within 2 mm, the link-offset
    difference between the two reference assets (1.46 mm max measured)."""
    from scipy.spatial.transform import Rotation

    from oracle.dyn import OracleEnv
    from robomanipbaselines_amd import model as MD

    a = MD.load("ur5e_cable")
    P = _placement()
    jn = [str(x) for x in a["names_jnt"]]
    b6 = int(a["jnt_body"][jn.index("wrist_3_joint")])
    qadr = [int(a["jnt_qposadr"][jn.index(str(n))]) for n in a["arm_joint_names"]]
    o = OracleEnv(a)

    def mjcf_frame(q):
        qp = a["qpos0"].copy()
        qp[qadr] = q
        o.set_state(0.0, qp, np.zeros(o.nv), np.zeros(o.nv), np.zeros(max(o.nu, 1)))
        o.forward()
        xp, xq = o.xpos()
        return Rotation.from_quat(xq[b6][[1, 2, 3, 0]]).as_matrix(), xp[b6]

    q0 = a["qpos0"][qadr]
    Ru0, pu0 = arm_ik.fk(P, q0)[-1]
    Rm0, pm0 = mjcf_frame(q0)
    TR, Tp = Ru0.T @ Rm0, Ru0.T @ (pm0 - pu0)
    np.testing.assert_allclose(np.abs(TR).max(0), 1.0, atol=1e-9)  # a signed axis permutation
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.uniform(-np.pi, np.pi, 6)
        Ru, pu = arm_ik.fk(P, q)[-1]
        Rm, pm = mjcf_frame(q)
        np.testing.assert_allclose(Ru @ TR, Rm, rtol=0, atol=1e-9)
        np.testing.assert_allclose(pu + Ru @ Tp, pm, rtol=0, atol=2e-3)
