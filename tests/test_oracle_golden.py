"""Pin the numpy oracle (oracle/glue.py) against golden vectors minted from the reference's own
code by tools/gen_golden.py.  CPU only."""

import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import glue


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.mark.parametrize(
    "case", ["gauss_te", "gauss_te_chunk20", "limits_te", "gauss_no_te"]
)
def test_ensemble_oracle_bitexact(case):
    d = _load(f"ensemble_{case}.npz")
    chunks = d["chunks"]
    if int(d["norm_limits"]):
        stats = {
            "norm_config": {"type": "limits", "out_min": -1.0, "out_max": 1.0},
            "min": d["mean"],
            "range": d["std"],
        }
    else:
        stats = {"norm_config": {"type": "gaussian"}, "mean": d["mean"], "std": d["std"]}
    o = glue.ActEnsembleOracle(int(d["chunk_size"]), stats, temporal_ensemble=not int(d["no_temp_ensem"]))
    it = iter(chunks)
    got = np.array([o.step(lambda: next(it)) for _ in range(len(d["actions"]))])
    np.testing.assert_array_equal(got, d["actions"])


def test_reward_oracle_bitexact():
    d = _load("reward_cable.npz")
    got = np.array(
        [glue.cable_reward(c, e, p, q) for c, e, p, q in zip(d["cable"], d["cable_end"], d["pole1"], d["pole2"])]
    )
    np.testing.assert_array_equal(got, d["reward"])
    assert 0 < d["reward"].sum() < len(d["reward"])  # both outcomes are covered


def test_insert_reward_oracle_bitexact():
    """oracle/glue.insert_reward vs MujocoUR5eInsertEnv._get_reward (MujocoUR5eInsertEnv.py:43-63)."""
    d = _load("reward_insert.npz")
    got = np.array([glue.insert_reward(p, h, q) for p, h, q in zip(d["peg"], d["hole"], d["quat"])])
    np.testing.assert_array_equal(got, d["reward"])
    assert 0 < d["reward"].sum() < len(d["reward"])
    assert float(d["cos_tilt"]) == float(np.cos(np.deg2rad(10)))


def test_door_reward_oracle_bitexact():
    """oracle/glue.door_reward vs MujocoUR5eDoorEnv._get_reward (MujocoUR5eDoorEnv.py:52-67)."""
    d = _load("reward_door.npz")
    got = np.array([glue.door_reward(p, h, a) for p, h, a in zip(d["pinch"], d["handle"], d["angle"])])
    np.testing.assert_array_equal(got, d["reward"])  # NaN where the reference gives NaN
    assert 0 < (d["reward"] >= 1.0).sum() < len(d["reward"])


def test_cabinet_reward_oracle_bitexact():
    """oracle/glue.cabinet_reward vs MujocoUR5eCabinetEnv._get_reward (MujocoUR5eCabinetEnv.py:57-73),
    every target task, thresholds hit exactly and by one ulp, NaN joints."""
    d = _load("reward_cabinet.npz")
    tasks = [None, "hinge", "slide"]
    got = np.array([glue.cabinet_reward(h, s, tasks[t]) for h, s, t in zip(d["hinge"], d["slide"], d["task"])])
    np.testing.assert_array_equal(got, d["reward"])
    assert 0 < d["reward"].sum() < len(d["reward"])
    with pytest.raises(ValueError):
        glue.cabinet_reward(0.0, 0.0, "lid")


def test_toolbox_reward_oracle_bitexact():
    """oracle/glue.toolbox_reward vs MujocoUR5eToolboxEnv._get_reward (MujocoUR5eToolboxEnv.py:46-57)."""
    d = _load("reward_toolbox.npz")
    got = np.array([glue.toolbox_reward(b, t) for b, t in zip(d["toolbox"], d["mat"])])
    np.testing.assert_array_equal(got, d["reward"])
    assert 0 < d["reward"].sum() < len(d["reward"])


def test_ring_reward_oracle_bitexact():
    """oracle/glue.ring_reward vs MujocoUR5eRingEnv._get_reward (MujocoUR5eRingEnv.py:46-75,
    matplotlib Path.contains_point): ties on vertices and edges, self-intersecting rings, the z
    gate at its threshold, NaN / inf vertices (dropped, subpath split) and NaN poles."""
    d = _load("reward_ring.npz")
    got = np.array([glue.ring_reward(r, p) for r, p in zip(d["ring"], d["pole"])])
    np.testing.assert_array_equal(got, d["reward"])
    assert 0 < d["reward"].sum() < len(d["reward"])


def test_obs_oracle_bitexact():
    d = _load("obs_ur5e.npz")
    for n in range(len(d["qpos"])):
        jp, jv, wr = glue.ur5e_obs(
            d["qpos"][n, :6], d["qvel"][n, :6], d["qpos"][n, 6:10], d["force"][n], d["torque"][n]
        )
        np.testing.assert_array_equal(jp, d["joint_pos"][n])
        np.testing.assert_array_equal(jv, d["joint_vel"][n])
        np.testing.assert_array_equal(wr, d["wrench"][n])


def test_depth_and_pointcloud_oracle_bitexact():
    d = _load("depth_pointcloud.npz")
    depth = glue.depth_linearize(d["zbuf"], float(d["extent"]), float(d["znear"]), float(d["zfar"]))
    assert depth.dtype == np.float32
    np.testing.assert_array_equal(depth, d["depth"])
    xyz, col = glue.depth_to_pointcloud(
        d["depth"], float(d["fovy"]), d["rgb"], float(d["near_clip"]), float(d["far_clip"])
    )
    pc = np.concatenate([xyz, col], 1)
    np.testing.assert_array_equal(pc, d["pointcloud"])
    np.testing.assert_array_equal(glue.crop_bb(pc, d["bb_min"], d["bb_max"]), d["cropped"])


def _phase_cases():
    d = _load("phase_schedule.npz")
    return [{k[len(f"c{i}_"):]: d[k] for k in d.files if k.startswith(f"c{i}_")} for i in range(int(d["n_cases"]))]


@pytest.mark.parametrize("case", _phase_cases(), ids=lambda c: str(c["name"]))
def test_phase_schedule_oracle_bitexact(case):
    rewards = case["reward"]
    out = glue.phase_schedule(
        lambda s: rewards[s], skip=int(case["skip"]), max_duration=float(case["max_duration"])
    )
    assert out["n_steps"] == int(case["n_steps"])
    np.testing.assert_array_equal(out["phase"], case["phase"])
    np.testing.assert_array_equal(out["infer_steps"], case["infer_steps"])
    succ, rew, dur = out["result"]
    assert succ == bool(case["success"][0])
    assert rew == float(case["result_reward"][0])
    assert dur == float(case["duration"][0])  # bit-exact fp64 time accumulation


@pytest.mark.parametrize("case", ["gauss", "gauss_noconfig", "limits", "limits01"])
def test_normalize_oracle_bitexact(case):
    from test_product_schedule import NORM_CASES

    d = _load("normalize.npz")
    st = NORM_CASES[case](d)
    np.testing.assert_array_equal(glue.normalize(d["data"], st), d[f"{case}_norm"])
    np.testing.assert_array_equal(glue.denormalize(d["data"], st), d[f"{case}_denorm"])
