"""The front kernel's launch LDS (csrc/rmbx_engine.hip front_launch_lds): padding it so the envs
spread evenly over CUs and rounds of blocks (RMBX_FRONT_BALANCE, default on; read when an engine is
created) changes only where blocks run, never a result -- 1024 cable envs (four per CU, padded) and
256 Pick envs (the collision scratch running past the dead region of the front LDS) stepped with and
without it from the same reset are bitwise equal."""

import os

import pytest
import torch

from robomanipbaselines_amd.envs.ur5e_cable import BatchedMujocoUR5eCableEnv
from robomanipbaselines_amd.envs.ur5e_pick import BatchedMujocoUR5ePickEnv

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _run(cls, n, grip, balance):
    old = os.environ.get("RMBX_FRONT_BALANCE")
    os.environ["RMBX_FRONT_BALANCE"] = balance
    try:
        env = cls(n, DEV)
    finally:
        if old is None:
            os.environ.pop("RMBX_FRONT_BALANCE")
        else:
            os.environ["RMBX_FRONT_BALANCE"] = old
    env.reset()
    a = env.engine.ctrl.clone()
    a[:, 6] = grip
    for _ in range(4):
        env.step(a)
    torch.cuda.synchronize()
    return env.engine.qpos.clone(), env.engine.qvel.clone(), env.engine.stats.clone()


@pytest.mark.parametrize("cls,n,grip", [(BatchedMujocoUR5eCableEnv, 1024, 255.0), (BatchedMujocoUR5ePickEnv, 256, 0.0)])
def test_front_lds_padding_changes_nothing(cls, n, grip):
    q0, v0, s0 = _run(cls, n, grip, "0")
    q1, v1, s1 = _run(cls, n, grip, "1")
    assert torch.equal(q0, q1) and torch.equal(v0, v1)
    assert torch.equal(s0[:, :3], s1[:, :3])  # contacts, constraint rows, Newton iterations
    assert int(s1[:, 0].sum()) > 0  # contacts were made
