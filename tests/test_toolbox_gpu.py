"""MujocoUR5eToolbox on the batched kernels: the compiled toolbox scene (a free
body placed per world index through its free joint's initial position) steps on the GPU engine in
agreement with the C oracle, rmbx_toolbox_reward is bit-exact against the reference's _get_reward
golden vectors, and the AutoEval command line runs the task."""

import os

import numpy as np
import pytest
import torch
import yaml

from conftest import GOLDEN
from oracle.dyn import OracleEnv
from robomanipbaselines_amd import kernels as K
from robomanipbaselines_amd import model as MD
from robomanipbaselines_amd.engine import PhysicsEngine
from robomanipbaselines_amd.envs.ur5e_toolbox import (TOOLBOX_INIT_QPOS, TOOLBOX_POS_OFFSETS, TOOLBOX_XY_THRE,
                                                      TOOLBOX_Z_OFFSET)

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_toolbox_engine_matches_oracle():
    arrays = MD.load("ur5e_toolbox")
    fq = MD.ModelInfo(arrays).qposadr("toolbox_freejoint")
    rng = np.random.default_rng(5)
    states = []
    for i in range(4):
        e = OracleEnv(arrays)
        qpos = arrays["qpos0"].copy()
        qpos[:14] = TOOLBOX_INIT_QPOS
        qpos[fq: fq + 3] += TOOLBOX_POS_OFFSETS[i] + np.array([0.0, 0.0, 0.01 * i])  # dropped from up to 3 cm
        ctrl = np.concatenate([TOOLBOX_INIT_QPOS[:6] + rng.normal(0, 0.05, 6), [rng.uniform(0, 255)]])
        e.set_state(0.0, qpos, np.zeros(e.nv), np.zeros(e.nv), ctrl)
        for _ in range((0, 5, 20, 40)[i]):
            e.step(8)
        states.append((*e.state(), ctrl))
    eng = PhysicsEngine(arrays, 4, DEV)
    eng.time.copy_(torch.tensor([s[0] for s in states], dtype=torch.float64))
    for k, name in ((1, "qpos"), (2, "qvel"), (3, "qacc_ws"), (4, "ctrl")):
        getattr(eng, name).copy_(torch.tensor(np.array([s[k] for s in states])))
    eng.step(8)
    torch.cuda.synchronize()
    qp1 = eng.qpos.cpu().numpy()
    for _ in range(24):
        eng.step(8)
    qp25 = eng.qpos.cpu().numpy()
    for i, (t, qp, qv, qa, c) in enumerate(states):
        o = OracleEnv(arrays)
        o.set_state(t, qp, qv, qa, c)
        o.step(8)
        np.testing.assert_allclose(qp1[i], o.state()[1], rtol=0, atol=1e-8)
        for _ in range(24):
            o.step(8)
        np.testing.assert_allclose(qp25[i], o.state()[1], rtol=0, atol=1e-4)


def test_toolbox_reward_matches_golden():
    d = np.load(os.path.join(GOLDEN, "reward_toolbox.npz"))
    box = torch.from_numpy(d["toolbox"]).to(DEV)
    mat = torch.from_numpy(d["mat"]).to(DEV)
    r = K.toolbox_reward(box, mat, TOOLBOX_XY_THRE, TOOLBOX_Z_OFFSET).cpu().numpy()
    np.testing.assert_array_equal(r, d["reward"])


def test_toolbox_world_placement_and_reward():
    from robomanipbaselines_amd.envs.ur5e_toolbox import BatchedMujocoUR5eToolboxEnv

    env = BatchedMujocoUR5eToolboxEnv(6, DEV, world_random_scale=[0.01, 0.01, 0.0])
    env.modify_world(world_idx=np.arange(6))
    env.reset()
    box = env.engine.xpos[:, env._toolbox].cpu().numpy()
    base = env.original_toolbox_pos + TOOLBOX_POS_OFFSETS
    assert np.all(np.abs(box[:, :2] - base[:, :2]) <= 0.01 + 1e-12)  # world offset + U(-s, s) noise
    np.testing.assert_allclose(box[:, 2], base[:, 2], rtol=0, atol=1e-12)
    assert (env._get_reward().cpu().numpy() == 0).all()  # on the table, not on the mat
    mat = env.engine.xpos[:, env._mat]
    env.engine.qpos[:, env._free_qadr: env._free_qadr + 3] = mat + torch.tensor([0.01, -0.01, 0.002], device=DEV,
                                                                                   dtype=torch.float64)
    env.engine.forward()
    assert (env._get_reward().cpu().numpy() == 1).all()


def test_toolbox_autoeval_command_line(tmp_path):
    from robomanipbaselines_amd.bin.Rollout import main

    res = os.path.join(tmp_path, "result.yaml")
    ro = main(["Mlp", "MujocoUR5eToolbox", "--auto_exit", "--no_plot", "--no_render", "--world_idx_list", "2", "3",
               "--result_filename", res, "--max_duration", "1.0"])
    with open(res) as f:
        data = yaml.safe_load(f)
    assert len(data["success"]) == 2
    for d in data["duration"]:
        assert 1.0 < d <= 1.0 + 0.032 + 1e-9
    assert np.isfinite(ro.env.engine.qpos.cpu().numpy()).all()
