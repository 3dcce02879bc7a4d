"""MuJoCo's divergence guard on the batched env (mj_step -> mj_checkAcc -> mj_resetData, [ext]
mujoco 3.1.6; the reference inherits it through gymnasium do_simulation, MujocoEnvBase.py:82-83):
an env driven to a non-finite qacc is reset inside that substep to the model's qpos0 with zero
velocity, warm start, ctrl and time, forwarded and integrated from there in the same substep (as
mj_step does after mj_checkAcc; the engine's redo pass), the remaining substeps of the env-step
run from there (ctrl 0, as MuJoCo's do_simulation leaves it), the reset is counted, and the other
envs are untouched bit for bit.  The C oracle restates the same guard (CPU test); the engine must match it."""

import numpy as np
import pytest

DEV = "cuda:0"


def _cable_start():
    from robomanipbaselines_amd import model as MD
    from robomanipbaselines_amd.envs.ur5e_cable import CABLE_INIT_QPOS

    a = MD.load("ur5e_cable")
    q = a["qpos0"].copy()
    q[:14] = CABLE_INIT_QPOS
    ctrl = np.r_[CABLE_INIT_QPOS[:6] + 0.05, 100.0]
    return a, q, ctrl


def test_oracle_resets_diverged_state_like_mujoco():
    from oracle.dyn import OracleEnv

    a, q, ctrl = _cable_start()
    env = OracleEnv(a)
    env.set_state(0.0, q, np.zeros(env.nv), np.zeros(env.nv), ctrl)
    assert env.step(24) == 0
    bad = ctrl.copy()
    bad[2] = np.nan
    env.set_ctrl(bad)
    assert env.step(8) == 1  # reset in the first substep
    t, qpos, qvel, _ = env.state()
    h = float(a["_timestep"])
    want = 0.0
    for _ in range(8):  # reset + mj_forward + integration in substep 1, then the 7 remaining
        want += h
    assert t == want
    assert np.isfinite(qpos).all() and np.isfinite(qvel).all()
    assert env.step(8) == 0  # ctrl is 0 after the reset: no further divergence


@pytest.mark.gpu
def test_nan_ctrl_resets_only_that_env_and_matches_oracle():
    import torch

    from oracle.dyn import OracleEnv
    from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv

    n = 4
    a = BatchedMujocoUR5eCableEnv(n, DEV)
    b = BatchedMujocoUR5eCableEnv(n, DEV)
    a.reset()
    b.reset()
    act = torch.tensor(np.tile(np.r_[a.init_qpos[:6] + 0.05, 100.0], (n, 1)), dtype=torch.float64, device=DEV)
    for _ in range(3):
        a.step(act)
        b.step(act)
    bad = act.clone()
    bad[1, 2] = float("nan")
    a.step(bad)
    b.step(act)
    torch.cuda.synchronize()
    assert a.bad_resets.tolist() == [0, 1, 0, 0]
    assert b.bad_resets.tolist() == [0, 0, 0, 0]
    ea, eb = a.engine, b.engine
    assert int(ea.stats[1, 3]) == 0  # consumed by the env
    assert float(ea.ctrl[1].abs().max()) == 0.0
    keep = [0, 2, 3]
    for name in ("qpos", "qvel", "qacc_ws", "time", "xpos", "sensordata"):
        assert torch.equal(getattr(ea, name)[keep], getattr(eb, name)[keep]), name
    # the reset env against the oracle's guard on the same inputs
    _, q, ctrl = _cable_start()
    o = OracleEnv(a.arrays)
    o.set_state(0.0, a.init_qpos, np.zeros(o.nv), np.zeros(o.nv), act[1].cpu().numpy())
    o.step(24)
    c = act[1].cpu().numpy().copy()
    c[2] = np.nan
    o.set_ctrl(c)
    assert o.step(8) == 1
    t, qpos, qvel, _ = o.state()
    assert float(ea.time[1]) == t
    np.testing.assert_allclose(ea.qpos[1].cpu().numpy(), qpos, rtol=0, atol=1e-8)
    np.testing.assert_allclose(ea.qvel[1].cpu().numpy(), qvel, rtol=0, atol=1e-6)
    for _ in range(2):
        a.step(act)
    assert torch.isfinite(ea.qpos).all()
    assert a.bad_resets.tolist() == [0, 1, 0, 0]
